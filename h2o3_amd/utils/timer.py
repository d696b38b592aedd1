"""Phase timers for host-side profiling (enable with H2O3_PROFILE=1).

Each phase is bracketed by a device synchronize so the attribution is
exact; disabled timers cost nothing.  Complements rocprofv3 kernel traces.
"""
import os
import time
from collections import defaultdict
from contextlib import contextmanager

ENABLED = os.environ.get("H2O3_PROFILE", "0") == "1"
TIMES = defaultdict(float)
COUNTS = defaultdict(int)


def _sync():
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()


@contextmanager
def phase(name):
    if not ENABLED:
        yield
        return
    _sync()
    t = time.perf_counter()
    try:
        yield
    finally:
        _sync()
        TIMES[name] += time.perf_counter() - t
        COUNTS[name] += 1


def report(reset=True):
    out = {k: (round(v * 1000, 3), COUNTS[k]) for k, v in sorted(TIMES.items(), key=lambda kv: -kv[1])}
    if reset:
        TIMES.clear()
        COUNTS.clear()
    return out
