"""Jobs: progress / status / cancellation records for long-running work.

Reference: water/Job.java (key, description, status CREATED / RUNNING /
DONE / CANCELLED / FAILED, progress, start/end time, exception), h2o-py
h2o/job.py (H2OJob.poll()).  Work runs synchronously on the driving
process (every rank executes the same SPMD program), so a Job is a
bookkeeping record that model builders and parsers update; cancel() sets a
flag checked between iterations.
"""
from __future__ import annotations

import time

from . import dkv


class Job:
    def __init__(self, description="", dest=None):
        self.key = dkv.make_key("job")
        self.description = description
        self.dest = dest
        self.status = "CREATED"
        self.progress = 0.0
        self.start_time = None
        self.end_time = None
        self.exception = None
        self._cancel = False
        dkv.put(self.key, self)

    def start(self):
        self.status, self.start_time = "RUNNING", time.time()
        return self

    def update(self, progress):
        self.progress = max(0.0, min(1.0, float(progress)))
        if self._cancel:
            raise JobCancelled(self.key)

    def done(self):
        self.status, self.progress, self.end_time = "DONE", 1.0, time.time()

    def fail(self, exc):
        self.status, self.exception, self.end_time = "FAILED", str(exc), time.time()

    def cancel(self):
        self._cancel = True
        self.status = "CANCELLED"

    @property
    def run_time(self):
        if self.start_time is None:
            return 0.0
        return (self.end_time or time.time()) - self.start_time

    def poll(self, poll_updates=None):
        return self

    def __repr__(self):
        return f"Job({self.key}, {self.description!r}, {self.status}, {self.progress:.0%})"


class JobCancelled(RuntimeError):
    pass


def jobs():
    return [j for j in (dkv.get(k) for k in dkv.keys()) if isinstance(j, Job)]
