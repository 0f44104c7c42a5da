"""Naive Bayes (reference ``heat/naive_bayes``)."""
