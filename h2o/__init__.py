"""Drop-in `import h2o` surface backed by h2o3_amd (MI355X-native)."""
from h2o3_amd.api import *  # noqa: F401,F403
from h2o3_amd.api import H2OFrame, init  # noqa: F401
from h2o3_amd import estimators  # noqa: F401
__version__ = "3.46.0.99-amd"
