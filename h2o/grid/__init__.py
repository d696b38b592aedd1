from h2o3_amd.grid import H2OGridSearch  # noqa: F401
