from .rest import create_app, start  # noqa: F401
