"""Parallelism: partitioner, flat buffers, P2P comm, pipeline engine, re-sharding."""
