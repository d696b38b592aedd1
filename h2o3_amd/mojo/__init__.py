"""MOJO export / standalone scoring."""
from .genmodel import MojoModel, load  # noqa: F401
