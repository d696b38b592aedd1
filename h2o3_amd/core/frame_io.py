"""Native binary frame save/load (reference: `H2OFrame.save` / `h2o.load_frame`,
water/fvec/persist/FramePersist.java).

The reference writes its compressed chunks per node; here a frame is written
as one directory per frame: `frame.json` (names, types, domains, row counts)
plus one raw `.npy` array per column and rank shard (numeric values, enum
codes, epoch-ms times) or a JSON list for host-side string/UUID columns.
Nothing is pickled; loading re-shards rows across the current cloud, so a
frame saved on N ranks can be loaded on M.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from ..parallel import cloud
from ..parallel import collectives as coll
from .vec import T_ENUM, T_STR, T_UUID, Vec

_FORMAT = "h2o3_amd.frame.v1"


def save_frame(frame, path, force=True):
    # rank 0 reads the file system and decides; every rank writes where it
    # says (a rank that looked after another rank's makedirs would pick a
    # different directory)
    d = os.path.join(path, frame.frame_id) if os.path.isdir(path) and not os.path.exists(
        os.path.join(path, "frame.json")) else path
    exists = os.path.exists(os.path.join(d, "frame.json"))
    d, exists = coll.broadcast_object((d, exists))
    if exists and not force:
        raise FileExistsError(f"{d} exists (use force=True)")
    os.makedirs(d, exist_ok=True)
    rank = cloud.rank()
    counts = coll.all_gather_object(frame.nlocal) if cloud.is_distributed() else [frame.nlocal]
    for j, v in enumerate(frame._vecs):
        if v.on_host:
            with open(os.path.join(d, f"c{j}.r{rank}.json"), "w") as f:
                json.dump([None if x is None else str(x) for x in v.data], f)
        else:
            np.save(os.path.join(d, f"c{j}.r{rank}.npy"), v.data.detach().cpu().numpy(), allow_pickle=False)
    if rank == 0:
        meta = {"format": _FORMAT, "frame_id": frame.frame_id, "names": frame.names,
                "types": [v.type for v in frame._vecs], "domains": [v.domain for v in frame._vecs],
                "shards": counts}
        with open(os.path.join(d, "frame.json"), "w") as f:
            json.dump(meta, f)
    cloud.barrier()
    return d


def load_frame(frame_id, path, force=True):
    from .frame import H2OFrame, _local_slice
    d = path
    if not os.path.exists(os.path.join(d, "frame.json")) and frame_id and \
            os.path.exists(os.path.join(path, frame_id, "frame.json")):
        d = os.path.join(path, frame_id)
    with open(os.path.join(d, "frame.json")) as f:
        meta = json.load(f)
    if meta.get("format") != _FORMAT:
        raise ValueError(f"{d} is not a saved h2o3_amd frame")
    shards = meta["shards"]
    n = int(sum(shards))
    s, e = _local_slice(n) if cloud.is_distributed() else (0, n)
    starts = np.cumsum([0] + shards)
    dev = cloud.device()
    vecs = []
    for j, (t, dom) in enumerate(zip(meta["types"], meta["domains"])):
        parts = []
        for r, cnt in enumerate(shards):
            lo, hi = max(s, starts[r]), min(e, starts[r] + cnt)
            if hi <= lo:
                continue
            if t in (T_STR, T_UUID):
                with open(os.path.join(d, f"c{j}.r{r}.json")) as f:
                    parts.append(np.array(json.load(f), dtype=object)[lo - starts[r]: hi - starts[r]])
            else:
                a = np.load(os.path.join(d, f"c{j}.r{r}.npy"), mmap_mode="r", allow_pickle=False)
                parts.append(np.array(a[lo - starts[r]: hi - starts[r]]))
        if t in (T_STR, T_UUID):
            vecs.append(Vec(np.concatenate(parts) if parts else np.array([], dtype=object), t))
        else:
            arr = np.concatenate(parts) if parts else np.zeros(0, dtype=np.float32)
            vecs.append(Vec(torch.from_numpy(arr).to(dev), t, dom if t == T_ENUM else None))
    return H2OFrame.from_vecs(vecs, meta["names"], frame_id=frame_id or meta["frame_id"])
