from . import _native  # noqa: F401
