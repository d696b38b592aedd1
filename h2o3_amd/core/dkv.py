"""Distributed key/value store (per-process registry with SPMD-agreed keys).

Reference: water/DKV.java, water/Key.java, water/Lockable.java.  The
reference stores every object under a Key homed on one node and replicates
on read.  Here every rank executes the same program, so a Key names the
rank-local part of an SPMD object (a Frame's row shard, a Model replica);
keys are generated deterministically so all ranks agree without messaging.
"""
from __future__ import annotations

import itertools
import threading
import weakref

_store: dict = {}
_lock = threading.RLock()
_counters: dict = {}


def make_key(prefix: str = "key") -> str:
    from ..parallel import collectives
    collectives._guard_check("make_key")     # a read served off the executor must not advance key counters
    with _lock:
        c = _counters.setdefault(prefix, itertools.count(1))
        k = f"{prefix}_{next(c)}"
    from ..parallel import collectives
    collectives._trace(f"make_key:{k}")     # H2O3_TRACE_COLL: keys must agree across ranks too
    return k


def put(key: str, obj, weak: bool = False):
    with _lock:
        _store[key] = weakref.ref(obj) if weak else obj
    return key


def get(key: str):
    with _lock:
        v = _store.get(key)
    if isinstance(v, weakref.ref):
        v = v()
    return v


def remove(key: str):
    with _lock:
        _store.pop(key, None)


def keys():
    with _lock:
        out = []
        for k, v in list(_store.items()):
            if isinstance(v, weakref.ref) and v() is None:
                _store.pop(k, None)
                continue
            out.append(k)
        return out


def remove_all(retained=()):
    retained = set(retained or ())
    with _lock:
        for k in list(_store.keys()):
            if k not in retained:
                _store.pop(k, None)


def ls():
    return [(k, type(get(k)).__name__) for k in keys()]
