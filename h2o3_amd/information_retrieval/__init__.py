"""TF-IDF (reference: hex/tfidf/{TfIdfPreprocessorTask, TermFrequencyTask,
DocumentFrequencyTask, InverseDocumentFrequencyTask}.java, h2o-py
h2o/information_retrieval/tf_idf.py).

Words split on whitespace (preprocess=True), optional lower-casing
(case_sensitive=False); TF = count of the word in the document, IDF =
log((#documents + 1) / (document frequency + 1)), output rows
(DocID, Word, TF, IDF, TF-IDF).  Word ids are dictionary-encoded once and
all counting is bincount / unique over integer keys on the device.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

from ..core.frame import H2OFrame
from ..parallel import cloud


def tf_idf(frame, document_id_col, text_col, preprocess=True, case_sensitive=True):
    if not isinstance(frame, H2OFrame):
        raise ValueError("TF-IDF cannot be computed for input of type %s. H2OFrame input is required." % type(frame))
    df = frame.as_data_frame()
    dcol = df.columns[document_id_col] if isinstance(document_id_col, int) else document_id_col
    tcol = df.columns[text_col] if isinstance(text_col, int) else text_col
    docs, words = [], []
    for d, t in zip(df[dcol].values, df[tcol].values):
        if t is None or (isinstance(t, float) and math.isnan(t)):
            continue
        t = str(t)
        if not case_sensitive:
            t = t.lower()
        toks = t.split() if preprocess else [t]
        docs.extend([d] * len(toks))
        words.extend(toks)
    if not words:
        return H2OFrame(pd.DataFrame({"DocID": [], "Word": [], "TF": [], "IDF": [], "TF-IDF": []}))
    dev = cloud.device()
    dvals, dcodes = np.unique(np.asarray(docs), return_inverse=True)
    wvals, wcodes = np.unique(np.asarray(words, dtype=object).astype(str), return_inverse=True)
    dc = torch.as_tensor(dcodes, device=dev)
    wc = torch.as_tensor(wcodes, device=dev)
    W = len(wvals)
    key = dc * W + wc
    uk, tf = torch.unique(key, return_counts=True)
    kd, kw = uk // W, uk % W
    dfreq = torch.bincount(kw, minlength=W).to(torch.float64)
    ndocs = len(dvals)
    idf = torch.log((ndocs + 1.0) / (dfreq + 1.0))
    tfv = tf.to(torch.float64)
    out = pd.DataFrame({"DocID": dvals[kd.cpu().numpy()], "Word": wvals[kw.cpu().numpy()],
                        "TF": tfv.cpu().numpy().astype(np.int64), "IDF": idf[kw].cpu().numpy(),
                        "TF-IDF": (tfv * idf[kw]).cpu().numpy()})
    return H2OFrame(out, column_types={"Word": "string"})
