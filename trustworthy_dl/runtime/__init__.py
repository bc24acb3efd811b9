"""Host-side runtime: native (C++) token loader and the heartbeat watchdog."""
