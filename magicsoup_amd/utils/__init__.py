"""Helpers: sequence utilities, profiling / tracing, checkpointing."""
