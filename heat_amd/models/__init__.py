"""Model zoo index: every estimator of the framework in one place."""
