from .rest import create_app, create_server_app, start  # noqa: F401
