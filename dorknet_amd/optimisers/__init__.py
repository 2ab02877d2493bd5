"""Optimisers (the reference's `optimisers` package)."""
