from builtins import chr, input, open, next, round, super  # noqa: F401
