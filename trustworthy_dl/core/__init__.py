"""Core: trust manager, node monitor, distributed trainer."""
