from . import cloud, collectives  # noqa: F401
