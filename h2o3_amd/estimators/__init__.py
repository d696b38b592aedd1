"""Estimator classes (h2o.estimators.*)."""
from ..models.tree.gbm import H2OGradientBoostingEstimator  # noqa: F401
