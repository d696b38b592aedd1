"""Word2Vec (skip-gram, hierarchical softmax).

Reference: hex/word2vec/Word2Vec.java, Word2VecModel.java,
WordVectorTrainer.java, HBWTree.java (Huffman tree over the vocabulary,
skip-gram with hierarchical softmax, sub-sampling of frequent words with
sent_sample_rate, linearly decaying learning rate from
init_learning_rate, min_word_freq vocabulary cut, NA = sentence break;
find_synonyms by cosine similarity, transform with aggregate_method
NONE / AVERAGE, pre_trained vectors import).

MI355X design: the reference trains word-by-word Hogwild threads; here
every epoch's (center, context) pairs are generated on the device at
once and trained in large mini-batches: one gather of the centre vectors,
one gather of all Huffman path nodes [B, L, d], a batched dot, and
scatter-add (index_add_) updates of both embedding tables -- the same
update rule applied to thousands of pairs per kernel instead of one.
"""
from __future__ import annotations

import heapq
import math

import numpy as np
import pandas as pd
import torch

from ..core.frame import H2OFrame
from ..core.vec import T_REAL, T_STR, Vec, make_enum_from_strings
from ..parallel import cloud
from .base import H2OEstimator

_MAX_EXP = 6.0      # WordVectorTrainer.MAX_EXP

W2V_DEFAULTS = dict(vec_size=100, window_size=5, sent_sample_rate=1e-3, norm_model="HSM", epochs=5,
                    min_word_freq=5, init_learning_rate=0.025, word_model="SkipGram", pre_trained=None, seed=-1)


def _huffman(counts):
    """Returns (codes list[list[int]], points list[list[int]]) per word."""
    V = len(counts)
    heap = [(int(c), i) for i, c in enumerate(counts)]
    heapq.heapify(heap)
    parent = {}
    bit = {}
    nxt = V
    while len(heap) > 1:
        c1, a = heapq.heappop(heap)
        c2, b = heapq.heappop(heap)
        parent[a], bit[a] = nxt, 0
        parent[b], bit[b] = nxt, 1
        heapq.heappush(heap, (c1 + c2, nxt))
        nxt += 1
    root = heap[0][1] if heap else 0
    codes, points = [], []
    for i in range(V):
        c, p = [], []
        j = i
        while j != root and j in parent:
            c.append(bit[j])
            p.append(parent[j] - V)
            j = parent[j]
        codes.append(c[::-1])
        points.append(p[::-1])
    return codes, points


class H2OWord2vecEstimator(H2OEstimator):
    _extra_params = ("seed",)   # deterministic sampling (not a reference client argument)
    algo = "word2vec"
    supervised_learning = False
    _defaults = W2V_DEFAULTS

    def train(self, x=None, y=None, training_frame=None, **kw):
        p = self._parms
        if p.get("pre_trained") is not None and training_frame is None:
            self._from_pretrained(p["pre_trained"])
            from ..core import dkv
            dkv.put(self.model_id, self)
            return self
        return super().train(x=x, y=None, training_frame=training_frame, **kw)

    def _from_pretrained(self, fr):
        df = fr.as_data_frame()
        self._vocab = [str(w) for w in df.iloc[:, 0]]
        self._index = {w: i for i, w in enumerate(self._vocab)}
        self._vecs = torch.tensor(df.iloc[:, 1:].values, dtype=torch.float32, device=cloud.device())
        self._parms["vec_size"] = self._vecs.shape[1]

    def _words(self, frame):
        v = frame.vec(frame.names[0])
        if v.type == T_STR:
            return [None if w is None else str(w) for w in v.data]
        if v.domain is not None:
            dom = v.domain
            return [None if c < 0 else dom[c] for c in v.data.cpu().tolist()]
        raise ValueError("Word2Vec needs a single string / categorical column of words")

    def _fit(self, spec):
        p = self._parms
        words = self._words(spec.frame)
        from collections import Counter
        cnt = Counter(w for w in words if w is not None)
        mf = int(p.get("min_word_freq", 5))
        vocab = sorted([w for w, c in cnt.items() if c >= mf], key=lambda w: (-cnt[w], w))
        if not vocab:
            raise ValueError("empty vocabulary (min_word_freq too high?)")
        self._vocab = vocab
        self._index = {w: i for i, w in enumerate(vocab)}
        counts = np.array([cnt[w] for w in vocab], dtype=np.float64)
        V, d = len(vocab), int(p.get("vec_size", 100))
        dev = cloud.device()
        seed = p.get("seed", -1)
        g = torch.Generator(device="cpu").manual_seed(int(seed) if seed not in (-1, None) else 0xC0FFEE)
        syn0 = ((torch.rand((V, d), generator=g) - 0.5) / d).to(dev)
        syn1 = torch.zeros((max(V - 1, 1), d), device=dev)
        codes, points = _huffman(counts)
        L = max(1, max(len(c) for c in codes))
        code_t = torch.full((V, L), -1, dtype=torch.float32)
        pt_t = torch.zeros((V, L), dtype=torch.long)
        for i in range(V):
            n = len(codes[i])
            code_t[i, :n] = torch.tensor(codes[i], dtype=torch.float32)
            pt_t[i, :n] = torch.tensor(points[i], dtype=torch.long)
        code_t, pt_t = code_t.to(dev), pt_t.to(dev)
        # token stream (-1 = sentence break / OOV dropped like the reference)
        ids = np.array([self._index.get(w, -2) if w is not None else -1 for w in words], dtype=np.int64)
        ids = ids[ids != -2]
        tok = torch.as_tensor(ids, device=dev)
        # sentence id per token: breaks at -1
        sent = torch.cumsum((tok == -1).long(), 0)
        keep = tok >= 0
        tok, sent = tok[keep], sent[keep]
        total_words = int(tok.numel())
        ss = float(p.get("sent_sample_rate", 1e-3))
        freq = torch.as_tensor(counts / counts.sum(), dtype=torch.float32, device=dev)
        epochs = int(p.get("epochs", 5))
        lr0 = float(p.get("init_learning_rate", 0.025))
        win = int(p.get("window_size", 5))
        processed = 0
        B = int(min(16384, max(256, 32 * V)))
        wm = str(p.get("word_model") or "SkipGram").lower().replace("_", "")
        if wm not in ("skipgram", "cbow"):
            raise ValueError(f"word_model must be SkipGram or CBOW, got {p.get('word_model')}")
        if str(p.get("norm_model") or "HSM").lower() != "hsm":
            raise ValueError("norm_model: only HSM (hierarchical softmax) is available (Word2Vec.NormModel)")
        cbow = wm == "cbow"
        for ep in range(epochs):
            # frequent-word sub-sampling (word2vec formula)
            if ss > 0:
                f = freq[tok]
                pk = (torch.sqrt(f / ss) + 1) * ss / f
                m = torch.rand(tok.numel(), generator=g).to(dev) < pk
                t_e, s_e = tok[m], sent[m]
            else:
                t_e, s_e = tok, sent
            n = t_e.numel()
            # dynamic window: reduced window b ~ U[0, win)
            red = torch.randint(0, win, (n,), generator=g).to(dev)
            if cbow:
                # CBOW (WordVectorTrainer.CBOW): the mean of the window's input
                # vectors predicts the centre word through the Huffman tree, the
                # hidden error goes back to every window word
                offs = torch.tensor([o for o in range(-win, win + 1) if o != 0], device=dev)
                J = torch.arange(n, device=dev).view(-1, 1) + offs.view(1, -1)
                okm = (J >= 0) & (J < n)
                Jc = J.clamp(0, n - 1)
                okm = okm & (s_e[Jc] == s_e.view(-1, 1)) & (offs.abs().view(1, -1) <= (win - red).view(-1, 1))
                order = torch.randperm(n, generator=g).to(dev)
                for s in range(0, n, B):
                    prog = (processed + s) / max(epochs * total_words, 1)
                    lr = max(lr0 * (1 - prog), lr0 * 1e-4)
                    idx = order[s:s + B]
                    m = okm[idx]
                    bag = m.sum(1)
                    ctxw = t_e[Jc[idx]]                                  # [b, 2w]
                    h = (syn0[ctxw] * m.unsqueeze(2)).sum(1) / bag.clamp_min(1).unsqueeze(1)
                    c = t_e[idx]
                    pts, cds = pt_t[c], code_t[c]
                    S1 = syn1[pts]
                    dot = (S1 * h.unsqueeze(1)).sum(2)
                    valid = (cds >= 0) & (bag > 0).view(-1, 1) & (dot.abs() < _MAX_EXP)
                    gsc = ((1 - cds) - torch.sigmoid(dot)) * lr * valid
                    neu1e = (gsc.unsqueeze(2) * S1).sum(1)
                    pv = pts[valid]
                    c1 = (torch.bincount(pv, minlength=syn1.shape[0]).to(h.dtype) / 8).clamp_min(1)
                    syn1.index_add_(0, pv, (gsc.unsqueeze(2) * h.unsqueeze(1))[valid] / c1[pv].unsqueeze(1))
                    wi = ctxw[m]
                    upd = neu1e.unsqueeze(1).expand(-1, m.shape[1], -1)[m]
                    c0 = (torch.bincount(wi, minlength=syn0.shape[0]).to(h.dtype) / 8).clamp_min(1)
                    syn0.index_add_(0, wi, upd / c0[wi].unsqueeze(1))
                processed += n
                continue
            cen, ctx = [], []
            for off in range(-win, win + 1):
                if off == 0:
                    continue
                j = torch.arange(n, device=dev) + off
                ok = (j >= 0) & (j < n)
                jj = j.clamp(0, n - 1)
                ok = ok & (s_e[jj] == s_e) & (abs(off) <= win - red)
                cen.append(torch.nonzero(ok).view(-1))
                ctx.append(jj[ok])
            ci = torch.cat(cen)
            xi = torch.cat(ctx)
            perm = torch.randperm(ci.numel(), generator=g).to(dev)
            ci, xi = ci[perm], xi[perm]
            npairs = ci.numel()
            for s in range(0, npairs, B):
                # linear decay over all epochs (reference: alpha = init*(1 - progress))
                prog = (processed + s / max(npairs, 1) * n) / max(epochs * total_words, 1)
                lr = max(lr0 * (1 - prog), lr0 * 1e-4)
                c = t_e[ci[s:s + B]]       # input word (skip-gram: predict centre from context vector)
                w_in = t_e[xi[s:s + B]]
                h = syn0[w_in]             # [b, d]
                pts = pt_t[c]              # [b, L]
                cds = code_t[c]
                S1 = syn1[pts]             # [b, L, d]
                dot = (S1 * h.unsqueeze(1)).sum(2)
                # hierarchicalSoftmaxSG skips nodes with |f| >= MAX_EXP (6)
                valid = (cds >= 0) & (dot.abs() < _MAX_EXP)
                f_ = torch.sigmoid(dot)
                gsc = ((1 - cds) - f_) * lr * valid
                neu1e = (gsc.unsqueeze(2) * S1).sum(1)
                # batched Hogwild: rows hit several times in one batch get the
                # sum of at most ~8 of their updates (a plain sum overshoots for frequent words)
                pv = pts[valid]
                c1 = (torch.bincount(pv, minlength=syn1.shape[0]).to(h.dtype) / 8).clamp_min(1)
                syn1.index_add_(0, pv, (gsc.unsqueeze(2) * h.unsqueeze(1))[valid] / c1[pv].unsqueeze(1))
                c0 = (torch.bincount(w_in, minlength=syn0.shape[0]).to(h.dtype) / 8).clamp_min(1)
                syn0.index_add_(0, w_in, neu1e / c0[w_in].unsqueeze(1))
            processed += n
        self._vecs = syn0
        self._output["vocab_size"] = V
        self._output["epochs"] = epochs

    def _score_all(self, spec):
        pass

    def _predict_raw(self, frame):
        raise NotImplementedError("use transform()")

    # ------------------------------------------------------------ API
    def find_synonyms(self, word, count=20):
        if word not in self._index:
            return {}
        V = self._vecs
        nv = V / V.norm(dim=1, keepdim=True).clamp_min(1e-12)
        sims = nv @ nv[self._index[word]]
        sims[self._index[word]] = -2
        top = torch.topk(sims, min(count, V.shape[0] - 1))
        return {self._vocab[int(i)]: float(s) for s, i in zip(top.values.cpu(), top.indices.cpu())}

    def transform(self, words, aggregate_method="NONE"):
        ws = self._words(words)
        d = self._vecs.shape[1]
        agg = str(aggregate_method or "NONE").upper()
        idx = [self._index.get(w, -1) if w is not None else -2 for w in ws]
        V = self._vecs
        if agg == "AVERAGE":
            # one row per NA-terminated word sequence
            def avg(cur):
                ok = [j for j in cur if j >= 0]
                return V[ok].mean(0) if ok else torch.full((d,), float("nan"), device=V.device)
            rows, cur = [], []
            for i in idx:
                if i == -2:
                    rows.append(avg(cur))
                    cur = []
                else:
                    cur.append(i)
            if cur:
                rows.append(avg(cur))
            M = torch.stack(rows) if rows else torch.zeros((0, d), device=V.device)
        else:
            it = torch.as_tensor([max(i, 0) for i in idx], device=V.device)
            M = V[it].clone()
            bad = torch.as_tensor([i < 0 for i in idx], device=V.device)
            M[bad] = float("nan")
        return H2OFrame.from_vecs([Vec(M[:, j].contiguous(), T_REAL) for j in range(d)], [f"C{j + 1}" for j in range(d)])

    def to_frame(self):
        d = self._vecs.shape[1]
        vecs = [make_enum_from_strings(self._vocab)] + [Vec(self._vecs[:, j].contiguous(), T_REAL) for j in range(d)]
        fr = H2OFrame.from_vecs(vecs, ["Word"] + [f"V{j + 1}" for j in range(d)])
        return fr
