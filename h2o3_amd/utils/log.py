"""Logging and the event timeline.

Reference: water/util/Log.java (levels TRACE..FATAL, per-node log files,
`h2o.log_and_echo`), water/TimeLine.java (a per-node ring buffer of
timestamped events that the /3/Timeline endpoint snapshots).

One ring buffer per process (rank); `timeline()` gathers every rank's
events (all_gather_object) so rank 0 can show the whole cloud.
"""
from __future__ import annotations

import collections
import logging
import os
import time

from ..parallel import cloud

LEVELS = {"TRACE": 5, "DEBUG": logging.DEBUG, "INFO": logging.INFO, "WARN": logging.WARNING,
          "ERRR": logging.ERROR, "FATAL": logging.CRITICAL}
logging.addLevelName(5, "TRACE")
_log = logging.getLogger("h2o3_amd")
if not _log.handlers:
    h = logging.StreamHandler()
    h.setFormatter(logging.Formatter("%(asctime)s r%(rank)s %(levelname)s: %(message)s"))
    _log.addHandler(h)
    _log.setLevel(os.environ.get("H2O3_LOG_LEVEL", "WARNING").upper() if
                  os.environ.get("H2O3_LOG_LEVEL", "WARNING").upper() in logging._nameToLevel else "WARNING")

_TL = collections.deque(maxlen=int(os.environ.get("H2O3_TIMELINE_SIZE", "4096")))


def log(level: str, msg: str):
    _log.log(LEVELS.get(level.upper(), logging.INFO), msg, extra={"rank": cloud.rank()})


def info(msg):
    log("INFO", msg)


def warn(msg):
    log("WARN", msg)


def event(kind: str, **detail):
    """Record a timeline event (reference TimeLine.record*)."""
    _TL.append({"time_ms": int(time.time() * 1000), "rank": cloud.rank(), "event": kind, **detail})


def timeline(all_ranks: bool = True):
    ev = list(_TL)
    if all_ranks and cloud.is_distributed():
        from ..parallel import collectives as coll
        ev = [e for part in coll.all_gather_object(ev) for e in part]
    return sorted(ev, key=lambda e: e["time_ms"])
