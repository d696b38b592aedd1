"""Jobs: progress / status / cancellation records for long-running work.

Reference: water/Job.java (key, description, status CREATED / RUNNING /
DONE / CANCELLED / FAILED, progress (:206), start on the fork/join pool
(:281), exception), h2o-py h2o/job.py (H2OJob.poll()).

In-process API calls run the work on the caller's thread (every rank runs
the same SPMD program), so the Job is a bookkeeping record the builders
tick.  Behind the REST front end (server/spmd.py) builds run on the cloud's
executor thread: POST returns the RUNNING job at once, `/3/Jobs/{id}`
reads the live progress, and `/3/Jobs/{id}/cancel` sets a flag that the
builder sees at its next iteration (`tick`).  With more than one rank the
flag is rank 0's (the rank that took the cancel request) and every rank
agrees on it in the same tick (cloud.agree), so all ranks stop at the same
tree / iteration and the collective sequence stays aligned.
"""
from __future__ import annotations

import time

from . import dkv


class Job:
    def __init__(self, description="", dest=None, key=None, dest_kind="Model", parent=None):
        self.key = key or dkv.make_key("job")
        self.parent = parent       # enclosing build (CV / grid / AutoML): its cancel stops this one
        self.description = description
        self.dest = dest
        self.dest_kind = dest_kind
        self.status = "CREATED"
        self.progress = 0.0
        self.progress_msg = ""
        self.start_time = None
        self.end_time = None
        self.exception = None
        self.stacktrace = None
        self.warnings = []
        self._cancel = False
        self.spmd = False          # set by the REST executor: cancel agreed across ranks on every tick
        prev = dkv.get(self.key) if key else None
        if isinstance(prev, Job) and prev._cancel:
            self._cancel = True    # a queued (CREATED) build cancelled before it started
        dkv.put(self.key, self)

    def start(self):
        self.status, self.start_time = "RUNNING", time.time()
        return self

    def update(self, progress, msg=None):
        """Local progress update (no cross-rank agreement); raises on cancel
        only in a single-rank cloud or outside the REST executor."""
        self.progress = max(0.0, min(1.0, float(progress)))
        if msg is not None:
            self.progress_msg = msg
        if self.cancel_requested and not self._spmd_any():
            raise JobCancelled(self.key)

    def tick(self, progress, msg=None, extra=()):
        """Per-iteration checkpoint of a builder: progress + cancellation,
        plus optional extra decisions that every rank must take like rank 0
        (returned agreed).  Raises JobCancelled when the job was cancelled."""
        from ..parallel import cloud
        self.progress = max(0.0, min(1.0, float(progress)))
        if msg is not None:
            self.progress_msg = msg
        vals = [1.0 if self.cancel_requested else 0.0] + [float(e) for e in extra]
        self._nticks = getattr(self, "_nticks", 0) + 1
        # SPMD builds agree on the cancel flag at EVERY tick (rank 0's REST
        # thread sets it; the reference checks stop_requested per tree), so a
        # cancel is never delayed by more than one iteration nor dropped
        if (extra or self._spmd_any()) and cloud.is_distributed():
            vals = cloud.agree(vals)
        if vals[0]:
            self._cancel = True
            raise JobCancelled(self.key)
        return vals[1:]

    def done(self):
        if self.status == "CANCELLED":
            return
        self.status, self.progress, self.end_time = "DONE", 1.0, time.time()

    def fail(self, exc):
        if isinstance(exc, JobCancelled) or self.cancel_requested:
            self.status, self.end_time = "CANCELLED", time.time()
            return
        import traceback
        self.status, self.exception, self.end_time = "FAILED", str(exc), time.time()
        self.stacktrace = "".join(traceback.format_exception(type(exc), exc, exc.__traceback__))[-8000:]

    def cancel(self):
        """Request cancellation: the builder stops at its next tick."""
        self._cancel = True
        if self.status in ("CREATED", "RUNNING"):
            self.status = "CANCELLED" if self.status == "CREATED" else self.status
        self.progress_msg = "cancel requested"

    @property
    def cancel_requested(self):
        j = self
        while j is not None:
            if j._cancel:
                return True
            j = j.parent
        return False

    def _spmd_any(self):
        j = self
        while j is not None:
            if j.spmd:
                return True
            j = j.parent
        return False

    @property
    def is_running(self):
        return self.status in ("CREATED", "RUNNING")

    @property
    def run_time(self):
        if self.start_time is None:
            return 0.0
        return (self.end_time or time.time()) - self.start_time

    def poll(self, poll_updates=None):
        while self.is_running:
            time.sleep(0.05)
        return self

    def __repr__(self):
        return f"Job({self.key}, {self.description!r}, {self.status}, {self.progress:.0%})"


class JobCancelled(RuntimeError):
    pass


# The job the current builder reports to (set by the REST executor before a
# build starts, consumed by H2OEstimator.train).
_pending = {"job": None}


def set_pending(job):
    _pending["job"] = job


def take_pending():
    j = _pending["job"]
    _pending["job"] = None
    return j


_stack = []


def current():
    """The innermost running build on this process (None outside builds)."""
    return _stack[-1] if _stack else None


def push(job):
    _stack.append(job)


def pop(job):
    if _stack and _stack[-1] is job:
        _stack.pop()
    elif job in _stack:
        _stack.remove(job)


def jobs():
    return [j for j in (dkv.get(k) for k in dkv.keys()) if isinstance(j, Job)]
