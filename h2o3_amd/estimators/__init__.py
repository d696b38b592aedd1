"""Estimator classes (h2o.estimators.*)."""
from ..models.tree.gbm import H2OGradientBoostingEstimator  # noqa: F401
from ..models.glm.glm import H2OGeneralizedLinearEstimator  # noqa: F401
from ..models.tree.drf import H2ORandomForestEstimator, H2OExtremelyRandomizedTreesEstimator  # noqa: F401
from ..models.tree.xgboost import H2OXGBoostEstimator  # noqa: F401
from ..models.tree.isofor import H2OIsolationForestEstimator, H2OExtendedIsolationForestEstimator  # noqa: F401
from ..models.clustering import (H2OKMeansEstimator, H2ONaiveBayesEstimator,  # noqa: F401
                                 H2OPrincipalComponentAnalysisEstimator, H2OSingularValueDecompositionEstimator)
from ..models.deeplearning import H2ODeepLearningEstimator  # noqa: F401


class H2OAutoEncoderEstimator(H2ODeepLearningEstimator):
    """Deep Learning with autoencoder=True by default (h2o-py
    estimators/deeplearning.py H2OAutoEncoderEstimator)."""

    def __init__(self, **kw):
        kw.setdefault("autoencoder", True)
        super().__init__(**kw)
from ..models.ensemble import H2OStackedEnsembleEstimator  # noqa: F401
from ..models.generic import H2OGenericEstimator  # noqa: F401
from ..models.isotonic import H2OIsotonicRegressionEstimator  # noqa: F401
from ..models.targetencoder import H2OTargetEncoderEstimator  # noqa: F401
from ..models.aggregator import H2OAggregatorEstimator  # noqa: F401
from ..models.coxph import H2OCoxProportionalHazardsEstimator  # noqa: F401
from ..models.glrm import H2OGeneralizedLowRankEstimator  # noqa: F401
from ..models.word2vec import H2OWord2vecEstimator  # noqa: F401
from ..models.psvm import H2OSupportVectorMachineEstimator  # noqa: F401
from ..models.rulefit import H2ORuleFitEstimator  # noqa: F401
from ..models.glm.gam import H2OGeneralizedAdditiveEstimator  # noqa: F401
from ..models.glm.anovaglm import H2OANOVAGLMEstimator  # noqa: F401
from ..models.glm.modelselection import H2OModelSelectionEstimator  # noqa: F401
from ..models.infogram import H2OInfogram  # noqa: F401
from ..models.tree.uplift import H2OUpliftRandomForestEstimator  # noqa: F401
from ..models.grep import H2OGrepModel  # noqa: F401
