"""MRTask: map over every rank's row shard, reduce across the cloud.

Reference: water/MRTask.java (map(Chunk[]) per chunk on every node,
reduce(MRTask) up a binary tree, postGlobal on the caller).  Here a "map"
is one vectorised call on this rank's device-resident column tensors
(the shard IS the chunk: one contiguous tensor per column), and the
reduce is a single torch.distributed collective on the returned tensors
(sum / min / max), so user code written against this API runs unchanged
on 1..N GPUs.
"""
from __future__ import annotations

from typing import Callable

import torch

from ..parallel import collectives as coll


class MRTask:
    def __init__(self, map_fn: Callable, reduce: str = "sum", post_global: Callable | None = None):
        self.map_fn = map_fn
        self.reduce = reduce
        self.post_global = post_global

    def do_all(self, frame, columns=None):
        cols = columns or list(frame.names)
        tensors = [frame.vec(c).data for c in cols]
        out = self.map_fn(*tensors)
        single = isinstance(out, torch.Tensor)
        outs = [out] if single else list(out)
        for t in outs:
            coll.allreduce_(t, self.reduce)
        res = outs[0] if single else tuple(outs)
        return self.post_global(res) if self.post_global else res


def map_reduce(frame, map_fn, reduce="sum", columns=None):
    return MRTask(map_fn, reduce).do_all(frame, columns)
