"""Python-3-only stand-in for python-future (see ../README.md)."""
