"""Tracing and counters (filled in below)."""
