from h2o3_amd.estimators import *  # noqa: F401,F403
