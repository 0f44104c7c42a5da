"""Classification (reference ``heat/classification``)."""
