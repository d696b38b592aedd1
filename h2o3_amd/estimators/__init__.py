"""Estimator classes (h2o.estimators.*)."""
from ..models.tree.gbm import H2OGradientBoostingEstimator  # noqa: F401
from ..models.glm.glm import H2OGeneralizedLinearEstimator  # noqa: F401
