from builtins import range, filter, map, zip  # noqa: F401
