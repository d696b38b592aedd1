"""SPMD command loop behind the REST front end: one REST endpoint drives every
GPU of the cloud, and model builds run as asynchronous jobs.

Reference: water/api/RequestServer.java (any node takes a request),
water/api/ModelBuilderHandler.java:19 -> hex/ModelBuilder.java:374
trainModel -> water/Job.java:281 start (the build runs cloud-wide on the
fork/join pool while the request returns the RUNNING job), JobsHandler
(progress / cancel).

MI355X design.  The cloud is one process per GPU (torchrun); every Frame is
an SPMD object (each rank holds its row shard) and every computation issues
the same collectives on every rank.  So a REST request is not "sent to the
node holding the data" -- it is *replayed* on every rank:

* rank 0 serves HTTP (uvicorn) and owns an **executor thread**.  Every
  request that touches frames, models or collectives is turned into a
  picklable command (route, decoded parameters, raw body, a nonce for any
  random names) and queued.  The executor broadcasts the command on the
  cloud's gloo control group and runs the handler; ranks 1..N-1 sit in
  `worker_loop`, receive the same command and run the same handler, so the
  SPMD collective sequence is identical on every rank.  Only rank 0's result
  is sent to the client.
* a model / grid / AutoML build returns a `Deferred`: the executor answers
  the HTTP request with the RUNNING job at once, then runs the build on the
  same thread.  A build request that arrives while another build runs is
  answered at once with a CREATED job whose key / destination rank 0 fixes
  up front (`hint`); it runs when the executor gets to it.  Read-only GETs
  (frames, models, grids, leaderboards, AutoML state) are served on the HTTP
  thread while a build runs, under a guard that refuses any collective
  (parallel/collectives.forbid): a read that would need one (an uncached
  rollup) is queued on the executor like before.  Requests that only read rank-0 state (`/3/Jobs`, `/3/Cloud`,
  metadata, Flow notebook storage) are served by the HTTP thread directly,
  so a client polls live progress and can cancel while the build runs;
  the cancel flag reaches every rank through the per-iteration agreement in
  `Job.tick`.
* while idle the executor broadcasts a no-op every H2O3_SPMD_IDLE_S seconds
  (default 30), so ranks never sit in one collective long enough to hit the
  process-group timeout.
* the heartbeat (parallel/heartbeat.py) marks the cloud unhealthy when a
  rank dies; the executor then fails its running job with a clear error and
  refuses new commands, while rank 0 keeps answering `/3/Cloud` and
  `/3/Jobs` (the reference keeps serving with an unhealthy cloud).
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import json
import os
import queue
import random
import threading
import traceback

from ..parallel import cloud

_rng = random.Random()
_ctx = threading.local()


def seed(nonce):
    _rng.seed(nonce)


def rand_hex(n=16):
    """Random-looking hex id, identical on every rank for one command."""
    return "".join("%x" % _rng.getrandbits(4) for _ in range(n))


def hint(name):
    """A value rank 0 fixed for this command before it was queued (the job
    key / destination of a build accepted while another one runs)."""
    return (getattr(_ctx, "hints", None) or {}).get(name)


def defer_allowed():
    """True inside a top-level REST command that may answer early and keep
    working (a build handler called from a Flow cell runs synchronously)."""
    v = getattr(_ctx, "allow_defer", False)
    _ctx.allow_defer = False
    return v


class Req:
    """The parts of an HTTP request a handler may read, picklable so the
    command replays on every rank."""

    def __init__(self, method="GET", path="", headers=None, body=b"", query=None):
        self.method, self.path = method, path
        self.headers = dict(headers or {})
        self._body = body or b""
        self.query_params = dict(query or {})

    async def body(self):
        return self._body

    async def json(self):
        return json.loads(self._body or b"{}")


class Deferred:
    """A handler's early answer plus the work still to run (a build)."""

    def __init__(self, response, work, job):
        self.response, self.work, self.job = response, work, job

    def run(self):
        from ..core import job as jobmod
        jobmod.push(self.job)
        try:
            self.work()
        except BaseException as e:  # noqa: BLE001 - recorded on the job; the request already returned
            if self.job.is_running:
                self.job.fail(e)
            if not isinstance(e, (jobmod.JobCancelled, Exception)):
                raise
        finally:
            jobmod.pop(self.job)
        if self.job.is_running:
            self.job.done()


class Executor:
    """Rank 0's command thread (see the module docstring)."""

    def __init__(self, run_command):
        self.run_command = run_command          # cmd -> response | Deferred (may raise)
        self.q: queue.Queue = queue.Queue()
        self.idle_s = float(os.environ.get("H2O3_SPMD_IDLE_S", 30))
        self.current = None                     # the Deferred being worked on
        self.stopped = False
        self._th = None
        from ..parallel import heartbeat
        heartbeat.add_listener(self._on_dead)

    def start(self):
        if self._th is None:
            self._th = threading.Thread(target=self._loop, name="h2o3-spmd-executor", daemon=True)
            self._th.start()
        return self

    def busy(self) -> bool:
        """A command (a build) is running or queued on the executor."""
        return self.current is not None or not self.q.empty() or getattr(self, "_running", False)

    def submit(self, cmd) -> concurrent.futures.Future:
        fut: concurrent.futures.Future = concurrent.futures.Future()
        if not cloud.healthy():
            fut.set_exception(RuntimeError(f"cloud unhealthy: rank(s) {cloud.dead_ranks()} stopped responding; "
                                           "restart the cloud"))
            return fut
        if self.stopped:
            fut.set_exception(RuntimeError("the cloud is shut down"))
            return fut
        self.start()
        cmd = dict(cmd, nonce=random.getrandbits(62))
        self.q.put((cmd, fut))
        return fut

    def _on_dead(self, dead):
        d = self.current
        if d is not None and d.job.is_running:
            d.job.fail(RuntimeError(f"cloud unhealthy: rank(s) {dead} missed heartbeats; the job cannot finish"))
        return True        # keep rank 0 alive to report the failure over REST

    def _loop(self):
        _bind_device()
        loop = asyncio.new_event_loop()
        while True:
            try:
                cmd, fut = self.q.get(timeout=self.idle_s)
            except queue.Empty:
                if cloud.is_distributed() and cloud.healthy():
                    cloud.broadcast_obj({"kind": "noop"})
                continue
            if cloud.is_distributed():
                cloud.broadcast_obj(cmd)
            if cmd["kind"] == "stop":
                self.stopped = True
                fut.set_result(None)
                return
            self._running = True
            try:
                execute(cmd, fut, loop, self)
            finally:
                self._running = False


def _bind_device():
    """The current HIP device is per host thread: bind this rank's GPU."""
    dev = cloud.device()
    if dev.type == "cuda":
        import torch
        torch.cuda.set_device(dev)


def execute(cmd, fut, loop, ex=None):
    """Run one command on this rank; fut (rank 0 only) gets the response."""
    seed(cmd.get("nonce", 0))
    _ctx.allow_defer = bool(cmd.get("defer", False))
    _ctx.hints = cmd.get("hints")
    try:
        out = ex.run_command(cmd, loop) if ex is not None else _run_local(cmd, loop)
    except BaseException as e:  # noqa: BLE001 - handed to the HTTP thread
        _ctx.allow_defer = False
        if fut is not None:
            fut.set_exception(e)
        elif not isinstance(e, Exception):
            raise
        else:   # a worker: rank 0 reports the same error to the client; log it here
            import sys
            print(f"[rank {cloud.rank()}] command {cmd.get('method')} {cmd.get('path')} failed: "
                  f"{type(e).__name__}: {e}", file=sys.stderr, flush=True)
        return
    _ctx.allow_defer = False
    if isinstance(out, Deferred):
        if fut is not None:
            fut.set_result(out.response)
        if ex is not None:
            ex.current = out
        try:
            out.run()
        finally:
            if ex is not None:
                ex.current = None
    elif fut is not None:
        fut.set_result(out)


_worker_run = {"fn": None}


def _run_local(cmd, loop):
    return _worker_run["fn"](cmd, loop)


def worker_loop(run_command):
    """Ranks 1..N-1: replay rank 0's commands until it stops the cloud."""
    _bind_device()
    _worker_run["fn"] = run_command
    loop = asyncio.new_event_loop()
    while True:
        cmd = cloud.broadcast_obj(None)
        kind = cmd.get("kind")
        if kind == "noop":
            continue
        if kind == "stop":
            return
        try:
            execute(cmd, None, loop)
        except Exception:  # noqa: BLE001 - rank 0 reports the same error to the client
            traceback.print_exc()
