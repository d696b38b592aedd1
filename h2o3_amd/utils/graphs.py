"""hipGraph capture without a collector pass inside it.

Destroying a captured graph while ANOTHER capture is in progress is an
illegal stream operation (hipErrorStreamCaptureUnsupported from
~CUDAGraph, which terminates the process).  A model that owns a graph (the
device-resident tree, the DL step) becomes garbage when the next model is
built, and Python's cyclic collector can run at any allocation -- including
the allocations made while the next model captures its own graph.  So the
collector runs once before a capture and is off during it.
"""
from __future__ import annotations

import contextlib
import gc

import torch


@contextlib.contextmanager
def capture(graph: "torch.cuda.CUDAGraph", **kw):
    """`with capture(g): ...` == `with torch.cuda.graph(g): ...` with no
    garbage collection (and so no graph destructor) during the capture."""
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        with torch.cuda.graph(graph, **kw):
            yield
    finally:
        if was:
            gc.enable()
