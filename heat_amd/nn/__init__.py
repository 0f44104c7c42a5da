"""Neural networks (reference ``heat/nn``)."""
