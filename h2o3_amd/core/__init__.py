from .frame import H2OFrame  # noqa: F401
