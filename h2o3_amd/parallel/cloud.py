"""Cloud formation: one process per GPU over torch.distributed.

Replaces the reference's JVM cloud (water/H2O.java, water/Paxos.java,
water/HeartBeatThread.java): instead of multicast/flatfile discovery and a
Paxos-agreed member list, the launcher (torchrun / the bench driver) provides
RANK / WORLD_SIZE / MASTER_ADDR and every rank joins one process group.  The
backend is "nccl" (= RCCL over xGMI) when GPUs are present and "gloo" on CPU.

Every rank holds a contiguous row shard of every Frame; collectives are
issued SPMD by all ranks in the same order (like MRTask's reduce tree).
"""
from __future__ import annotations

import atexit
import datetime
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

_state = {"initialized": False, "device": None, "rank": 0, "world": 1, "local_rank": 0,
          "backend": None, "start": time.time(), "owns_pg": False, "name": None, "failed": False,
          "ctl": None, "healthy": True, "dead": [], "hb": None}


def _mark_failed_hook(prev):
    """sys.excepthook wrapper: an uncaught exception marks this rank as failed,
    so the exit-time teardown does not wait in a barrier for peers that may be
    blocked in a collective this rank will never join."""
    def hook(tp, val, tb):
        _state["failed"] = True
        prev(tp, val, tb)
    return hook


def _env_int(k, d):
    try:
        return int(os.environ.get(k, d))
    except ValueError:
        return d


def init(device: str | None = None, backend: str | None = None, timeout_s: float = 1800.0,
         name: str | None = None):
    """Join (or create) the cloud.  Idempotent."""
    if _state["initialized"]:
        return info()
    world = _env_int("WORLD_SIZE", 1)
    rank = _env_int("RANK", 0)
    local_rank = _env_int("LOCAL_RANK", rank)
    want_gpu = torch.cuda.is_available() and (device is None or str(device).startswith("cuda"))
    if device is None:
        device = f"cuda:{local_rank % max(1, torch.cuda.device_count())}" if want_gpu else "cpu"
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        be = backend or os.environ.get("H2O3_DIST_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
        kw = {}
        if be == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(be, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        _state["owns_pg"] = True
        sys.excepthook = _mark_failed_hook(sys.excepthook)
        atexit.register(_atexit_shutdown)
    if dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
        _state["backend"] = dist.get_backend()
        # control plane: host-side decisions / commands travel on a gloo group
        # (the data plane is RCCL on GPU clouds; a CPU broadcast there would
        # need a device round trip)
        _state["ctl"] = None if dist.get_backend() == "gloo" else dist.new_group(
            backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))
    _state.update(initialized=True, device=dev, rank=rank, world=world, local_rank=local_rank,
                  name=name or f"h2o3_amd_{os.getpid()}", healthy=True, dead=[])
    if world > 1 and dist.is_initialized() and os.environ.get("H2O3_HEARTBEAT", "1") != "0":
        from . import heartbeat
        _state["hb"] = heartbeat.start()
    return info()


def ensure():
    if not _state["initialized"]:
        init()


def device() -> torch.device:
    ensure()
    return _state["device"]


def rank() -> int:
    ensure()
    return _state["rank"]


def world() -> int:
    ensure()
    return _state["world"]


def is_distributed() -> bool:
    ensure()
    return _state["world"] > 1


def is_gpu() -> bool:
    return device().type == "cuda"


def ctl_group():
    """The gloo group for host-side control traffic (None = the default group)."""
    return _state["ctl"]


def agree(values, src: int = 0) -> list:
    """Every rank returns rank `src`'s values (a short list of numbers): the
    per-iteration decisions that depend on one host's clock or on a REST
    cancel request (scoring schedule, max_runtime_secs, job cancel) must be
    taken identically on every rank, or the SPMD collective sequence splits."""
    vals = [float(v) for v in values]
    if not is_distributed():
        return vals
    t = torch.tensor(vals, dtype=torch.float64)
    from . import collectives
    collectives._trace("agree", t)
    dist.broadcast(t, src, group=_state["ctl"])
    return t.tolist()


def broadcast_obj(obj, src: int = 0):
    """Broadcast a picklable host object from `src` on the control group."""
    if not is_distributed():
        return obj
    from . import collectives
    collectives._trace("broadcast_obj")
    lst = [obj]
    dist.broadcast_object_list(lst, src=src, group=_state["ctl"])
    return lst[0]


def healthy() -> bool:
    return bool(_state["healthy"])


def dead_ranks() -> list:
    return list(_state["dead"])


def mark_unhealthy(dead):
    """Heartbeat verdict: ranks that stopped beating (parallel/heartbeat.py)."""
    _state["healthy"] = False
    _state["dead"] = sorted(set(_state["dead"]) | set(dead))


def info() -> dict:
    d = _state["device"]
    props = None
    if d is not None and d.type == "cuda":
        p = torch.cuda.get_device_properties(d)
        props = {"name": p.name, "total_memory_gb": round(p.total_memory / 2**30, 1),
                 "cus": getattr(p, "multi_processor_count", None),
                 "arch": getattr(p, "gcnArchName", None)}
    return {"cloud_name": _state["name"], "rank": _state["rank"], "cloud_size": _state["world"],
            "device": str(d), "backend": _state["backend"], "gpu": props,
            "uptime_s": round(time.time() - _state["start"], 1), "host": socket.gethostname(),
            "healthy": _state["healthy"], "dead_ranks": list(_state["dead"])}


def shutdown(clean: bool = True, barrier_timeout_s: float = 60.0):
    """Tear the owned process group down explicitly (letting interpreter exit
    destroy a live gloo group races its worker threads: std::terminate).

    clean=True: all ranks are finishing together -> rendezvous first (gloo:
    monitored_barrier with a short timeout, so a dead peer is reported instead
    of waiting out the 30-minute collective timeout).  clean=False (this rank
    failed): no barrier -- it could pair with a peer's pending collective --
    just drop the group so the process exits and its peers' collectives fail
    fast on the broken connection."""
    hb = _state.get("hb")
    if hb is not None:
        hb.stop()
        _state["hb"] = None
    if _state["owns_pg"] and dist.is_initialized():
        if clean:
            try:
                if dist.get_backend() == "gloo":
                    dist.monitored_barrier(timeout=datetime.timedelta(seconds=barrier_timeout_s))
                else:
                    barrier()
            except Exception:
                pass
        try:
            dist.destroy_process_group()
        except Exception:
            pass
    _state.update(initialized=False, owns_pg=False, ctl=None)


def _atexit_shutdown():
    shutdown(clean=not _state["failed"])


def barrier():
    if is_distributed():
        from . import collectives
        collectives._trace("barrier")
        if is_gpu() and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device().index])
        else:
            dist.barrier()
