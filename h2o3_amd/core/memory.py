"""HBM memory manager: a per-rank byte budget for frame columns with LRU
spill of cold Vecs to host memory (pinned when the columns live on a GPU)
and to disk past a host cap, reloaded on touch.

Reference: water/MemoryManager.java:44, 85 (a heap budget; allocations past
it trigger the Cleaner), water/Cleaner.java:12 (a background thread writes
the least-recently-used values to the ice root and frees them; a later get
reloads them).

MI355X design.  A column is one contiguous device tensor (core/vec.py), so
the unit of spill is a whole Vec: its tensor moves to a pinned host buffer
(one DMA) or, once the host tier is past its cap, to a file under the spill
directory (torch.save; reloaded with weights_only=True).  Accounting is by
tensor bytes, LRU order by last touch of Vec.data; spilling happens when a
newly tracked or reloaded Vec pushes the resident bytes over the budget.  The
tree / GLM engines keep their own compact device copies (binned codes,
expanded designs), so cold frame columns can leave HBM while a model trains.
Disabled (zero cost beyond one attribute check) unless a budget is set:
H2O3_HBM_BUDGET (bytes, or with K/M/G suffix) or set_budget().
"""
from __future__ import annotations

import os
import tempfile
import threading
import weakref
from collections import OrderedDict

import torch


def _parse_bytes(s):
    if s is None:
        return None
    s = str(s).strip().upper()
    mult = 1
    for suf, m in (("K", 1 << 10), ("M", 1 << 20), ("G", 1 << 30), ("T", 1 << 40)):
        if s.endswith(suf) or s.endswith(suf + "B"):
            mult = m
            s = s.rstrip("B")[:-1]
            break
    return int(float(s) * mult)


class MemoryManager:
    def __init__(self):
        self.budget = _parse_bytes(os.environ.get("H2O3_HBM_BUDGET"))
        self.host_cap = _parse_bytes(os.environ.get("H2O3_HOST_SPILL_CAP"))
        self.spill_dir = os.environ.get("H2O3_SPILL_DIR")
        self._lru = OrderedDict()     # id(vec) -> weakref(vec)
        self.resident = 0             # bytes of tracked device tensors
        self.host_bytes = 0
        self.spills = 0
        self.reloads = 0
        self.bytes_written = 0
        self._lock = threading.RLock()
        self._ctr = 0

    @property
    def enabled(self):
        return self.budget is not None

    def set_budget(self, budget, host_cap=None, spill_dir=None):
        with self._lock:
            self.budget = _parse_bytes(budget) if budget is not None else None
            self.host_cap = _parse_bytes(host_cap) if host_cap is not None else self.host_cap
            if spill_dir is not None:
                self.spill_dir = spill_dir
            if self.budget is None:
                self._lru.clear()
                self.resident = 0
            else:
                self._evict(None)

    def stats(self):
        return {"budget": self.budget, "resident_bytes": self.resident, "host_bytes": self.host_bytes,
                "tracked": len(self._lru), "spills": self.spills, "reloads": self.reloads,
                "bytes_written": self.bytes_written}

    # ------------------------------------------------------------ tracking
    @staticmethod
    def _nbytes(t):
        return t.numel() * t.element_size()

    def track(self, vec):
        t = vec._d
        if not isinstance(t, torch.Tensor):
            return
        with self._lock:
            key = id(vec)
            if key in self._lru:
                self._lru.move_to_end(key)
                return
            self._lru[key] = weakref.ref(vec, self._dead(key, self._nbytes(t)))
            self.resident += self._nbytes(t)
            self._evict(key)

    def _dead(self, key, nb):
        def cb(_):
            with self._lock:
                if self._lru.pop(key, None) is not None:
                    self.resident -= nb
        return cb

    def untrack(self, vec):
        with self._lock:
            if self._lru.pop(id(vec), None) is not None and isinstance(vec._d, torch.Tensor):
                self.resident -= self._nbytes(vec._d)

    def touch(self, vec):
        with self._lock:
            key = id(vec)
            if key in self._lru:
                self._lru.move_to_end(key)

    # ------------------------------------------------------------ spill / reload
    def _evict(self, protect):
        if self.budget is None or self.resident <= self.budget:
            return
        # hysteresis: evict down to 90% of the budget so a scan over more
        # columns than fit does not spill on every single touch
        target = int(self.budget * 0.9)
        while self.resident > target and self._lru:
            victim = None
            for key, ref in self._lru.items():
                if key == protect:
                    continue
                v = ref()
                if v is None or not isinstance(v._d, torch.Tensor):
                    continue
                victim = (key, v)
                break
            if victim is None:
                return
            key, v = victim
            self._spill(key, v)

    def _spill(self, key, v):
        t = v._d
        nb = self._nbytes(t)
        dev = t.device
        clean = getattr(v, "_clean", None)
        if clean is not None and clean[1] == t._version and clean[0][0] == "disk" and os.path.exists(clean[0][1]):
            # unmodified since its reload: the disk copy is still exact, drop only
            v._sp = clean[0]
            v._d = None
            self._lru.pop(key, None)
            self.resident -= nb
            self.spills += 1
            return
        if clean is not None and clean[0][0] == "disk":
            # reloaded from disk, then modified: that older spill file is stale
            _unlink(clean[0][1])
            try:
                v._clean = None
            except AttributeError:
                pass
        to_disk = dev.type == "cpu" or (self.host_cap is not None and self.host_bytes + nb > self.host_cap)
        if to_disk:
            d = self.spill_dir or os.path.join(tempfile.gettempdir(), f"h2o3_spill_{os.getpid()}")
            os.makedirs(d, exist_ok=True)
            self._ctr += 1
            path = os.path.join(d, f"vec_{self._ctr}.pt")
            # a compact copy: a column may view a larger storage (e.g. a slice of
            # a 2-D host array), and torch.save writes whole storages
            torch.save(t.detach().cpu().clone(), path)
            self.bytes_written += nb
            v._sp = ("disk", path, str(dev), int(t.shape[0]) if t.dim() else 0)
            weakref.finalize(v, _unlink, path)         # the file goes with the Vec
        else:
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=False)
            v._sp = ("host", h, str(dev), int(t.shape[0]) if t.dim() else 0)
            self.host_bytes += nb
            # a Vec collected while spilled returns its host bytes to the cap
            try:
                v._spf = weakref.finalize(v, _host_release, weakref.ref(self), nb)
            except AttributeError:
                pass
        v._d = None
        self._lru.pop(key, None)
        self.resident -= nb
        self.spills += 1

    def reload(self, vec):
        with self._lock:
            sp = vec._sp
            kind, payload, dev = sp[0], sp[1], torch.device(sp[2])
            if kind == "disk":
                t = torch.load(payload, map_location="cpu", weights_only=True).to(dev)
                clean = (sp, t._version)       # the file stays valid until t is modified in place
            else:
                t = payload.to(dev, non_blocking=False)
                fin = getattr(vec, "_spf", None)
                if fin is not None:
                    fin.detach()
                    vec._spf = None
                self.host_bytes -= self._nbytes(payload)
                clean = None
            vec._sp = None
            vec._d = t
            try:
                vec._clean = clean
            except AttributeError:
                pass
            self.reloads += 1
            self.track(vec)
            return t


def _host_release(mref, nb):
    m = mref()
    if m is not None:
        m.host_bytes -= nb


def _unlink(path):
    try:
        os.remove(path)
    except OSError:
        pass


MANAGER = MemoryManager()


def set_budget(budget, host_cap=None, spill_dir=None):
    """Per-rank byte budget for frame columns (None disables the manager)."""
    MANAGER.set_budget(budget, host_cap, spill_dir)


def stats():
    return MANAGER.stats()
