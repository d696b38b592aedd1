"""Heartbeat failure detection for the multi-rank cloud.

Reference: water/HeartBeatThread.java (every node multicasts a heartbeat
each second; a node silent for TIMEOUT = 60 s is suspect and the cloud is
reported unhealthy) and water/H2O.java (a cloud that lost a member cannot
recover and must be restarted).

Here every rank bumps a counter key `h2o3_hb/<rank>` in the rendezvous
TCPStore every `interval` seconds from a daemon thread and reads the peers'
counters.  A peer whose counter has not moved for `suspect_s` seconds of the
reader's own clock (no clock agreement across hosts needed) is declared
dead: the cloud is marked unhealthy (`/3/Cloud` reports it), registered
listeners run (the REST server fails its pending jobs with a clear error),
and -- unless a listener keeps the process alive, as the REST front end
does to report the failure -- the process exits with status 3 instead of
waiting out the 30-minute collective timeout in a collective the dead peer
will never join.  A rank that leaves cleanly (cloud.shutdown) marks its key
as departed first, so orderly teardown is never mistaken for a failure.

Knobs: H2O3_HB_INTERVAL (s, default 5), H2O3_HB_SUSPECT (s, default 60),
H2O3_HEARTBEAT=0 disables it.
"""
from __future__ import annotations

import os
import sys
import threading
import time

import torch.distributed as dist

from ..utils import log as _log

_DEPARTED = 1 << 40
_listeners = []          # callables(dead_ranks) -> bool (True: keep this process alive)


def add_listener(fn):
    _listeners.append(fn)


def remove_listener(fn):
    if fn in _listeners:
        _listeners.remove(fn)


def _store():
    from torch.distributed import distributed_c10d as c10d
    try:
        return c10d._get_default_store()
    except Exception:  # noqa: BLE001 - no default store: connect a client to the rendezvous
        return dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ.get("MASTER_PORT", 29511)),
                             is_master=False)


class Heartbeat:
    def __init__(self, rank, world, interval, suspect_s, store=None, epoch=""):
        self.rank, self.world = rank, world
        # keys are scoped by a per-init epoch agreed by the ranks: a cloud
        # re-initialised on the same rendezvous store must not read the
        # previous session's "departed" counters as its peers' state
        self.epoch = str(epoch)
        self.interval, self.suspect_s = float(interval), float(suspect_s)
        self.store = store if store is not None else _store()
        self._stop = threading.Event()
        self.last = {r: (-1, time.monotonic()) for r in range(world) if r != rank}
        self.dead = []
        self.fired = False
        self.th = threading.Thread(target=self._run, name="h2o3-heartbeat", daemon=True)

    def key(self, r):
        return f"h2o3_hb/{self.epoch}/{r}" if self.epoch else f"h2o3_hb/{r}"

    def _run(self):
        while not self._stop.is_set():
            try:
                self.store.add(self.key(self.rank), 1)
                now = time.monotonic()
                newly = []
                for r, (c, t) in list(self.last.items()):
                    v = self.store.add(self.key(r), 0)
                    if v >= _DEPARTED:
                        self.last.pop(r)                 # left cleanly
                    elif v != c:
                        self.last[r] = (v, now)
                    elif now - t > self.suspect_s and r not in self.dead:
                        newly.append(r)
            except Exception as e:  # noqa: BLE001 - the store host (rank 0 / launcher) is gone
                if self._stop.is_set():
                    return
                newly = [0] if self.rank != 0 and 0 not in self.dead else []
                _log.event("heartbeat_store_error", error=str(e))
            if newly:
                self.dead += newly
                self._fire(newly)
            self._stop.wait(self.interval)

    def _fire(self, newly):
        from . import cloud
        cloud.mark_unhealthy(newly)
        msg = (f"h2o3_amd cloud: rank(s) {sorted(newly)} missed heartbeats for more than {self.suspect_s:g} s "
               f"(HeartBeatThread timeout): cloud unhealthy, rank {self.rank} cannot complete collectives")
        print(msg, file=sys.stderr, flush=True)
        _log.event("cloud_unhealthy", dead=sorted(newly), rank=self.rank)
        keep = False
        for fn in list(_listeners):
            try:
                keep = bool(fn(sorted(newly))) or keep
            except Exception:  # noqa: BLE001 - a listener must not stop the verdict
                pass
        if not keep and os.environ.get("H2O3_HB_EXIT", "1") != "0":
            self.fired = True
            os._exit(3)

    def start(self):
        self.th.start()
        return self

    def stop(self):
        """Clean departure: peers stop watching this rank."""
        if self._stop.is_set():
            return
        self._stop.set()
        try:
            self.store.add(self.key(self.rank), _DEPARTED)
        except Exception:  # noqa: BLE001 - store already gone at teardown
            pass


def start(rank=None, world=None):
    from . import cloud
    interval = float(os.environ.get("H2O3_HB_INTERVAL", 5))
    suspect = float(os.environ.get("H2O3_HB_SUSPECT", 60))
    r = cloud._state["rank"] if rank is None else rank
    w = cloud._state["world"] if world is None else world
    epoch = ""
    if dist.is_initialized():
        r, w = dist.get_rank(), dist.get_world_size()
        # one random epoch id for this init, broadcast from rank 0 over the
        # control plane (gloo) -- every rank calls start() from cloud.init
        obj = [os.urandom(8).hex() if r == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=cloud._state.get("ctl"))
        epoch = obj[0]
    return Heartbeat(r, w, interval, suspect, epoch=epoch).start()
