"""Lasso placeholder (filled in below)."""
__all__ = []
