"""Utilities (reference ``heat/utils``)."""
