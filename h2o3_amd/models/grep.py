"""Grep (reference: hex/grep/Grep.java + GrepModel.java): regex search over
the raw bytes of a text frame, returning the matches and their byte
offsets.  Python `re` over the host bytes (the reference scans raw chunks
on the CPU as well; no device work would help a regex automaton)."""
from __future__ import annotations

import re

import numpy as np
import pandas as pd

from ..core.frame import H2OFrame
from .base import H2OEstimator

GREP_DEFAULTS = dict(regex="", max_matches=-1)


class H2OGrepModel(H2OEstimator):
    algo = "grep"
    supervised_learning = False
    _defaults = GREP_DEFAULTS

    def _fit(self, spec):
        p = self._parms
        rx = re.compile(p["regex"])
        df = spec.frame.as_data_frame()
        text = "\n".join(",".join("" if v is None else str(v) for v in row) for row in df.itertuples(index=False))
        data = text.encode()
        matches, offsets = [], []
        mm = int(p.get("max_matches", -1))
        for m in rx.finditer(text):
            matches.append(m.group(0))
            offsets.append(len(text[: m.start()].encode()))
            if 0 < mm <= len(matches):
                break
        self._output["matches"] = matches
        self._output["offsets"] = offsets

    def matches(self):
        return self._output["matches"]

    def offsets(self):
        return self._output["offsets"]

    def _score_all(self, spec):
        pass

    def _predict_raw(self, frame):
        raise NotImplementedError
