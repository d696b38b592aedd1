from h2o3_amd.automl import H2OAutoML, get_automl, get_leaderboard  # noqa: F401
