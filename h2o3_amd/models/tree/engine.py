"""Level-wise GPU tree growth shared by GBM, DRF, XGBoost and Uplift.

Reference: hex/tree/SharedTree.java (scoreAndBuildTrees / buildLayer),
hex/tree/DTree.java (UndecidedNode/DecidedNode, findBestSplitPoint at
DTree.java:984), hex/tree/ScoreBuildHistogram2.java.

Per tree, per level:
  1. histograms for the *smaller* child of every split (HIP LDS kernel,
     ops/csrc/tree_hist.hip); the larger sibling is parent - smaller
     (histogram subtraction — the reference builds every node from rows);
  2. multi-GPU: reduce_scatter over the feature dim, each rank scores the
     splits of its feature slice, candidates are all_gathered (small);
  3. vectorized split search over [node, feature, threshold, NA-direction]
     (squared-error criterion of the reference, or the second-order gain of
     XGBoost), categorical levels sorted by mean response -> bitset;
  4. stable GPU partition of each split node's row segment.
Leaves end up as contiguous segments of the row permutation, giving the
per-row leaf id for the leaf-value pass without any tree traversal.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from ...ops import tree_ops
from ...parallel import cloud
from ...parallel import collectives as coll
from ...utils.timer import phase

NEG_INF = float("-inf")


@dataclass
class GrowParams:
    criterion: str = "se"          # "se" (H2O GBM/DRF) | "xgb" (second order)
    max_depth: int = 5
    min_rows: float = 10.0         # se: min weighted rows per child; xgb: min_child_weight
    min_split_improvement: float = 1e-5
    reg_lambda: float = 1.0
    reg_alpha: float = 0.0
    gamma: float = 0.0             # xgb min_split_loss
    max_leaves: int = 0            # 0 = unlimited
    monotone: np.ndarray | None = None  # [F] in {-1,0,1}
    col_sample_rate: float = 1.0   # per split (GBM) / mtries fraction
    mtries: int = -1               # DRF: features per node (-1 = all)
    col_sample_rate_change_per_level: float = 1.0
    tree_col_mask: np.ndarray | None = None  # [F] bool, per-tree sampling
    seed: int = 0
    hist_mem_budget: int = 8 << 30
    interaction_sets: list | None = None  # list of sets of feature ids
    leaf_budget_by_gain: bool = False   # max_leaves spent on the highest-gain nodes first (lossguide)
    use_bounds: bool = True        # monotone node bounds clamp (True) or veto (False) splits (GBMModel.java:84)


@dataclass
class Tree:
    """Host-side tree in BFS order (the per-node arrays feed scoring kernels,
    MOJO writer, SHAP and varimp)."""
    feat: list = field(default_factory=list)
    left: list = field(default_factory=list)
    right: list = field(default_factory=list)
    thr: list = field(default_factory=list)        # numeric: x < thr goes left
    na_left: list = field(default_factory=list)
    is_cat: list = field(default_factory=list)
    cat_left: list = field(default_factory=list)   # list of np.uint8 level masks (len = cardinality) or None
    value: list = field(default_factory=list)
    weight: list = field(default_factory=list)     # training cover (sum w or sum h)
    gain: list = field(default_factory=list)
    depth: list = field(default_factory=list)
    split_code: list = field(default_factory=list) # code threshold (numeric) for debugging

    def add_children(self, depth, wl, wr):
        """Append a (left, right) node pair per entry of wl / wr; returns the
        id of the first new node (pairs are consecutive)."""
        k = 2 * len(wl)
        base = len(self.feat)
        w = [0.0] * k
        w[0::2] = [float(x) for x in wl]
        w[1::2] = [float(x) for x in wr]
        self.feat += [-1] * k; self.left += [-1] * k; self.right += [-1] * k; self.thr += [0.0] * k
        self.na_left += [False] * k; self.is_cat += [False] * k; self.cat_left += [None] * k
        self.value += [0.0] * k; self.weight += w; self.gain += [0.0] * k
        self.depth += [depth] * k; self.split_code += [-1] * k
        return base

    def add_node(self, depth, weight):
        self.feat.append(-1); self.left.append(-1); self.right.append(-1); self.thr.append(0.0)
        self.na_left.append(False); self.is_cat.append(False); self.cat_left.append(None)
        self.value.append(0.0); self.weight.append(float(weight)); self.gain.append(0.0)
        self.depth.append(depth); self.split_code.append(-1)
        return len(self.feat) - 1

    @property
    def n_nodes(self):
        return len(self.feat)

    def is_leaf(self, i):
        return self.left[i] < 0

    def leaves(self):
        return np.nonzero(np.asarray(self.left, dtype=np.int64) < 0)[0].tolist()

    def max_depth(self):
        return int(np.max(np.asarray(self.depth))) if len(self.depth) else 0

    def to_arrays(self):
        return {k: np.asarray(getattr(self, k)) for k in ("feat", "left", "right", "thr", "na_left", "is_cat",
                                                          "value", "weight", "gain", "depth")}

    def predict_host(self, X: np.ndarray) -> np.ndarray:
        """Reference traversal on host (X: [n, F] float64, cats as codes)."""
        out = np.empty(X.shape[0])
        for r in range(X.shape[0]):
            i = 0
            while self.left[i] >= 0:
                x = X[r, self.feat[i]]
                if self.is_cat[i]:
                    m = self.cat_left[i]
                    if np.isnan(x) or int(x) >= len(m) or int(x) < 0:
                        go_left = self.na_left[i]
                    else:
                        go_left = bool(m[int(x)])
                elif np.isnan(x):
                    go_left = self.na_left[i]
                else:
                    go_left = x < self.thr[i]
                i = self.left[i] if go_left else self.right[i]
            out[r] = self.value[i]
        return out


class CatMasks:
    """Categorical level masks of a tree's nodes, stored as the per-level
    [k, Bs] uint8 mask matrices the split search produced plus (node, row,
    feature) indices: cat_masks[i] gives node i's level mask (None for a
    non-categorical node) on access.  Building the per-node arrays in the
    level loop cost ~10% of a depth-20 DRF tree's host time (10^4-10^5
    categorical splits per tree)."""

    def __init__(self, n, mats=(), feats=(), part=None, row=None, lvm=None):
        self.n = int(n)
        self.mats = list(mats)
        self.feats = list(feats)
        self.part = np.full(self.n, -1, dtype=np.int32) if part is None else part
        self.row = np.zeros(self.n, dtype=np.int32) if row is None else row
        self.lvm = dict(lvm or {})          # feature -> level index array into the mask row
        self.extra = {}                     # per-node overrides (assignments after construction)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self.n))]
        i = int(i)
        if i < 0:
            i += self.n
        if i in self.extra:
            return self.extra[i]
        p = int(self.part[i])
        if p < 0:
            return None
        r = int(self.row[i])
        return self.mats[p][r][self.lvm[int(self.feats[p][r])]]

    def __setitem__(self, i, v):
        self.extra[int(i)] = v

    def __iter__(self):
        for i in range(self.n):
            yield self[i]


class _TreeBuf:
    """Growable per-node numpy arrays for one tree under construction: the
    level loop records the splits of a whole level with vectorized
    assignments (the per-node Python bookkeeping cost seconds per tree at
    depth 20 / 10^5 nodes); to_tree() hands back the list-based Tree."""

    _FIELDS = (("feat", np.int64, -1), ("left", np.int64, -1), ("right", np.int64, -1), ("thr", np.float64, 0.0),
               ("na_left", bool, False), ("is_cat", bool, False), ("value", np.float64, 0.0),
               ("weight", np.float64, 0.0), ("gain", np.float64, 0.0), ("depth", np.int64, 0),
               ("split_code", np.int64, -1))

    def __init__(self, cap=256):
        self.n = 1                       # the root
        self.cap = cap
        for name, dt, fill in self._FIELDS:
            setattr(self, name, np.full(cap, fill, dtype=dt))
        self.cat_left = {}
        self.cat_parts = []                  # (node ids, features, [k, Bs] mask matrix) per level
        self.cat_lvm = {}

    def _grow(self, need):
        cap = self.cap
        while cap < need:
            cap *= 2
        if cap == self.cap:
            return
        for name, dt, fill in self._FIELDS:
            a = np.full(cap, fill, dtype=dt)
            a[:self.n] = getattr(self, name)[:self.n]
            setattr(self, name, a)
        self.cap = cap

    def add_children(self, depth, wl, wr):
        """(left, right) node pairs for every entry of wl / wr; returns the
        first new id (pairs are consecutive)."""
        k = 2 * len(wl)
        base = self.n
        self._grow(base + k)
        self.weight[base:base + k:2] = wl
        self.weight[base + 1:base + k:2] = wr
        self.depth[base:base + k] = depth
        self.n = base + k
        return base

    def to_tree(self):
        """Tree over numpy per-node arrays (copies; no per-node Python lists:
        the list conversion cost ~5 ms per depth-20 DRF tree).  Index,
        assignment and len() behave like the list form."""
        n = self.n
        t = Tree()
        for name, _, _ in self._FIELDS:
            setattr(t, name, getattr(self, name)[:n].copy())
        cm = CatMasks(n, lvm=self.cat_lvm)
        for nodes, feats, mat in self.cat_parts:
            cm.part[nodes] = len(cm.mats)
            cm.row[nodes] = np.arange(nodes.size, dtype=np.int32)
            cm.mats.append(mat)
            cm.feats.append(feats)
        for i, m in self.cat_left.items():
            cm.extra[i] = m
        t.cat_left = cm
        return t


class TreeGrower:
    """Grows one tree over a BinnedData with a given channel mode."""

    def __init__(self, bd, params: GrowParams):
        self.bd = bd
        self.p = params
        self.dev = bd.codes.device
        n = bd.nrows_local
        self.ridx = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.ridx2 = torch.empty(n, dtype=torch.int32, device=self.dev)
        # position-ordered copies of the two row channels, permuted with ridx
        # (off by default: the extra scattered writes in the partition cost more
        # than the contiguous histogram reads save — A/B in profiles/README.md)
        self.use_payload = False
        self._pay = [torch.empty(n, dtype=torch.float32, device=self.dev) for _ in range(4)] \
            if self.use_payload else [None] * 4
        self.W = cloud.world()
        self.rank = cloud.rank()
        F = bd.F
        self.Fpad = ((F + self.W - 1) // self.W) * self.W
        self.Fl = self.Fpad // self.W
        self.f0 = self.rank * self.Fl
        self.is_cat_t = torch.tensor(bd.is_cat + [False] * (self.Fpad - F), dtype=torch.bool, device=self.dev)
        self.nbins_t = torch.tensor(bd.nbins + [0] * (self.Fpad - F), dtype=torch.int64, device=self.dev)
        mono = params.monotone if params.monotone is not None else np.zeros(F)
        self.mono_t = torch.tensor(list(mono) + [0] * (self.Fpad - F), dtype=torch.float64, device=self.dev)
        self.rng = np.random.RandomState(params.seed & 0x7FFFFFFF)
        if tree_ops.env("H2O3_HIST_BUDGET"):
            params.hist_mem_budget = int(os.environ["H2O3_HIST_BUDGET"])

    # ------------------------------------------------------------------ hist
    def _build_hist(self, ridx, va, vb, mode, starts, counts, need_mask=None):
        if mode == 3:
            # uplift: treatment and control (w, w*y) histograms side by side
            with phase("tree.hist"):
                H1, _ = tree_ops.hist_build(self.bd, ridx, va, vb[0], 0, starts, counts, len(starts),
                                            vmax=self._vmax, posv=False, want_wyy=True)
                H2, _ = tree_ops.hist_build(self.bd, ridx, va, vb[1], 0, starts, counts, len(starts),
                                            vmax=self._vmax, posv=False, want_wyy=True)
            H = torch.cat([H1, H2], -1)
            self._last_wyy = None
            if self.W > 1:
                if self.Fpad > self.bd.F:
                    H = torch.cat([H, torch.zeros((self.Fpad - self.bd.F,) + tuple(H.shape[1:]), dtype=H.dtype,
                                                  device=H.device)], 0)
                H = coll.reduce_scatter_dim0(H)
            return H
        posv = self.use_payload
        if mode == 0 and getattr(self, "_pos1", None) is not None:
            # NaN-masked responses kept in POSITION order (moved by the partition
            # compaction): the histogram reads them coalesced, no row gather
            va, vb, posv = self._pos1[0], None, True
        elif mode == 0 and getattr(self, "_va_eff", None) is not None:
            va, vb = self._va_eff, None   # 0/1 weights folded into NaN-masked responses
        with phase("tree.hist"), phase(f"tree.hist.L{getattr(self, '_level', 0)}"):
            H, wyy = tree_ops.hist_build(self.bd, ridx, va, vb, mode, starts, counts, len(starts), vmax=self._vmax,
                                         posv=posv, want_wyy=True,
                                         unit_w=getattr(self, "_unit_w", False), need_mask=need_mask)
        if self.W > 1:
            H, wyy = self._rs_hist_wyy(H, wyy)
        self._last_wyy = wyy
        return H  # [Fl, n, Bs, C]

    def _rs_hist_wyy(self, H, wyy):
        """Multi-GPU reduce of a level histogram [F, n, Bs, C]: reduce-scatter
        by feature (each rank keeps its Fl features), with the per-node w*y*y
        sums riding along -- every rank's chunk carries a copy of its local
        wyy, so the scattered chunk ends in the global sums: ONE collective
        per level instead of reduce_scatter + all_reduce."""
        W = self.W
        if self.Fpad > self.bd.F:
            H = torch.cat([H, torch.zeros((self.Fpad - self.bd.F,) + tuple(H.shape[1:]), dtype=H.dtype,
                                          device=H.device)], 0)
        if wyy is None:
            return coll.reduce_scatter_dim0(H), None
        n = wyy.numel()
        loc = H.shape[1:]
        buf = torch.cat([H.reshape(W, -1), wyy.to(H.dtype).view(1, n).expand(W, n)], 1)
        out = coll.reduce_scatter_dim0(buf).view(-1)
        chunk = out.numel() - n
        return out[:chunk].view((self.Fl,) + tuple(loc)), out[chunk:]

    def _hist_need(self, cm):
        """Per-node features whose histograms the split search reads: the
        sampled columns plus each rank's first local feature (node totals come
        from H[0]).  None = all (no column sampling / no GPU kernels)."""
        if self.dev.type != "cuda" or getattr(cm, "_all_true", False) or self.p.criterion.startswith("uplift") \
                or tree_ops.env("H2O3_HIST_NEED", "1") == "0":
            return None
        need = cm.to(self.dev, dtype=torch.bool).clone()
        for r in range(self.W):
            if r * self.Fl < self.bd.F:
                need[:, r * self.Fl] = True
        return need

    # ------------------------------------------------------------------ splits
    def _col_sel(self, n_nodes, depth):
        """Per-node sampled columns as a [n, k] int64 tensor of global feature
        ids in ascending order (k random eligible features per node: the k
        smallest of per-(node, feature) uniform keys, on the device when the
        data is -- deep DRF levels have 10^4+ nodes), or None when every
        eligible feature is scored.  Consumes the tree's RNG exactly like the
        mask path so both give the same samples."""
        p = self.p
        F = self.bd.F
        base = np.ones(F, dtype=bool) if p.tree_col_mask is None else p.tree_col_mask.astype(bool)
        rate = p.col_sample_rate * (p.col_sample_rate_change_per_level ** depth)
        k = None
        if p.mtries is not None and p.mtries > 0:
            k = p.mtries
        elif rate < 1.0:
            k = max(1, int(math.floor(rate * base.sum() + 0.5)))
        if k is None or k >= base.sum():
            return None
        elig = np.nonzero(base)[0]
        if self.dev.type == "cuda":
            # one HIP launch: per-node selection sampling, rows come out sorted
            # (was rand + top-k + gather + segmented sort, with a host sync)
            seed = int(self.rng.randint(0, 2 ** 31 - 1))
            el = self.__dict__.setdefault("_elig_dev", {})
            key = elig.tobytes()
            if key not in el:
                el.clear()
                el[key] = self._upload_elig(elig)
            return tree_ops.col_sample(n_nodes, el[key], k, seed)
        keys = self.rng.random_sample((n_nodes, len(elig)))
        sel = np.argpartition(keys, k - 1, axis=1)[:, :k]
        return torch.from_numpy(np.sort(elig[sel], axis=1))

    def _upload_elig(self, elig):
        """The eligible feature ids on the device without a host wait: a
        pageable H2D copy waits for the queued kernels (the look-ahead
        pipeline stalled once per tree, ~1 ms), so the ids go through the
        pinned upload ring (non-blocking) and a stream-ordered device copy
        that outlives the ring slot (the ids are cached for the tree)."""
        return tree_ops._h2d(elig.astype(np.int64), self.dev).clone()

    def _col_mask_allowed(self, allow, depth):
        """Per-node mask under interaction constraints, on the device: the
        branch's allowed features (BranchInteractionConstraints) intersected
        with the per-tree column mask, then column sampling among them
        (DTree.UndecidedNode.scoreCols samples from the columns that still have
        histograms): k smallest of per-(node, feature) uniform keys among each
        node's eligible features -- no per-node host loop."""
        p = self.p
        F = self.bd.F
        dev = allow.device
        base = torch.ones(F, dtype=torch.bool, device=dev) if p.tree_col_mask is None else \
            torch.as_tensor(p.tree_col_mask.astype(bool), device=dev)
        m = allow & base.view(1, -1)
        n = m.shape[0]
        rate = p.col_sample_rate * (p.col_sample_rate_change_per_level ** depth)
        if (p.mtries is not None and p.mtries > 0) or rate < 1.0:
            cnt = m.sum(1)
            if p.mtries is not None and p.mtries > 0:
                k = torch.full_like(cnt, int(p.mtries))
            else:
                k = torch.floor(rate * cnt.to(torch.float64) + 0.5).to(cnt.dtype).clamp(min=1)
            g = torch.Generator(device=dev)
            g.manual_seed(int(self.rng.randint(0, 2 ** 31 - 1)))
            keys = torch.rand((n, F), generator=g, device=dev)
            keys = torch.where(m, keys, torch.full_like(keys, 2.0))
            rank = torch.argsort(torch.argsort(keys, 1), 1)
            m = m & (rank < k.view(-1, 1))
        if self.Fpad > F:
            m = torch.cat([m, torch.zeros((n, self.Fpad - F), dtype=torch.bool, device=dev)], 1)
        m = m.contiguous()
        m._all_true = False
        return m

    def _col_mask(self, n_nodes, depth, sel=None, allow=None):
        """[n, Fpad] bool mask of features eligible per node."""
        p = self.p
        F = self.bd.F
        if allow is not None:
            return self._col_mask_allowed(allow, depth)
        if sel is None:
            sel = self._col_sel(n_nodes, depth)
        if sel is not None:
            m = torch.zeros((n_nodes, self.Fpad), dtype=torch.bool, device=sel.device)
            m.scatter_(1, sel, True)
            m._all_true = False
            return m
        base = np.ones(F, dtype=bool) if p.tree_col_mask is None else p.tree_col_mask.astype(bool)
        m = np.tile(base, (n_nodes, 1))
        all_true = bool(m.all())
        if self.Fpad > F:
            m = np.concatenate([m, np.zeros((n_nodes, self.Fpad - F), dtype=bool)], 1)
        t = torch.from_numpy(m)
        t._all_true = all_true
        return t

    def _interaction_map(self):
        """(allow [F, F] bool: features that may follow a split on f, root [F]
        bool) from GrowParams.interaction_sets, or None."""
        sets = self.p.interaction_sets
        if not sets:
            return None
        F = self.bd.F
        cached = self.__dict__.get("_ics_cache")
        if cached is not None:
            return cached
        allow = np.zeros((F, F), dtype=bool)
        root = np.zeros(F, dtype=bool)
        for st in sets:
            idx = np.asarray(sorted(st), dtype=np.int64)
            root[idx] = True
            for f in idx:
                allow[f, idx] = True
        self._ics_cache = (allow, root)
        return self._ics_cache

    # ------------------------------------------------------------------ monotone node bounds
    def _bnd_dev(self, n):
        """[n, 2] f64 (lo, hi) prediction bounds of the frontier nodes being
        scored, or None when no node is bounded."""
        b = getattr(self, "_bnd", None)
        if b is None:
            return None
        off = getattr(self, "_bnd_off", 0)
        return b[off:off + n]

    def _bound_cost(self, Lb, Rb, lo, hi):
        """(gain penalty of clamping the children's constants into [lo, hi],
        violated?) for left / right channel sums [..., C]."""
        p = self.p
        if p.criterion == "xgb":
            al, ar = Lb[..., 1] + p.reg_lambda, Rb[..., 1] + p.reg_lambda
            pl, pr = -Lb[..., 0] / al, -Rb[..., 0] / ar
            al, ar = 0.5 * al, 0.5 * ar
        else:
            al, ar = Lb[..., 0], Rb[..., 0]
            pl, pr = Lb[..., 1] / al.clamp_min(1e-300), Rb[..., 1] / ar.clamp_min(1e-300)
        cl, cr = torch.minimum(torch.maximum(pl, lo), hi), torch.minimum(torch.maximum(pr, lo), hi)
        viol = (cl != pl) | (cr != pr)
        return al * (cl - pl) ** 2 + ar * (cr - pr) ** 2, viol

    def _bound_winners(self, res):
        """Per-node check of already selected winners (categorical pair
        paths): clamp penalty or veto for splits outside the node bounds."""
        n = res["gain"].shape[0]
        bnd = self._bnd_dev(n)
        if bnd is None:
            return res
        pen, viol = self._bound_cost(res["L"].to(torch.float64), res["R"].to(torch.float64), bnd[:, 0], bnd[:, 1])
        g = res["gain"].to(torch.float64)
        g = torch.where(viol & torch.isfinite(g), g - pen if self.p.use_bounds else torch.full_like(g, NEG_INF), g)
        res = dict(res)
        res["gain"] = g
        return res

    def _child_bounds(self, lo, hi, f_s, cat_s, Lsel, Rsel, mode):
        """Constraints.withNewConstraint for the children of the split nodes:
        bounds at the midpoint of the (clamped) child predictions on
        increasing / decreasing columns, inherited otherwise."""
        p = self.p
        mono = np.asarray(p.monotone, dtype=np.float64)
        c = np.where(cat_s | (f_s >= mono.size), 0.0, mono[np.minimum(f_s, mono.size - 1)])
        if p.criterion == "xgb":
            pl = -Lsel[:, 0] / (Lsel[:, 1] + p.reg_lambda)
            pr = -Rsel[:, 0] / (Rsel[:, 1] + p.reg_lambda)
        else:
            pl = Lsel[:, 1] / np.maximum(Lsel[:, 0], 1e-300)
            pr = Rsel[:, 1] / np.maximum(Rsel[:, 0], 1e-300)
        mid = 0.5 * (np.clip(pl, lo, hi) + np.clip(pr, lo, hi))
        lo_l, hi_l, lo_r, hi_r = lo.copy(), hi.copy(), lo.copy(), hi.copy()
        inc, dec = c > 0, c < 0
        hi_l[inc] = np.minimum(hi[inc], mid[inc])
        lo_r[inc] = np.maximum(lo[inc], mid[inc])
        lo_l[dec] = np.maximum(lo[dec], mid[dec])
        hi_r[dec] = np.minimum(hi[dec], mid[dec])
        return np.stack([lo_l, lo_r], 1).reshape(-1), np.stack([hi_l, hi_r], 1).reshape(-1)

    # ------------------------------------------------------------------ adaptive bins
    _RR_TYPES = ("uniformadaptive", "uniformadaptive", "random", "quantilesglobal")

    def _tree_hist_type(self):
        """Histogram type of the tree being grown: RoundRobin cycles the
        reference's ROUND_ROBIN_CANDIDATES (AUTO counts as UniformAdaptive,
        SharedTreeModel.java:59) tree by tree."""
        ht = getattr(self.bd, "hist_type", "auto")
        if ht == "roundrobin":
            return self._RR_TYPES[(int(self.p.seed) + getattr(self, "_tree_no", 0)) % 4]
        return ht

    def _adapt_hist(self, H):
        """Per-node adaptive binning of the numeric features (reference
        UniformAdaptive / Random, DHistogram.java:366-386, DTree.java:337).  The
        level histogram is on the fixed fine grid of nbins_top_level cells; the
        reference re-bins each (node, column) into
        nb = max(nbins_top_level >> (depth - 1), nbins) uniform bins over the
        parent's observed range (_adapt_range).  Here each run of fine bins that falls into one coarse
        bin is folded into the run's LAST fine bin: every cumulative sum at an
        allowed boundary is unchanged and every other boundary repeats the sums
        of the previous allowed one, so any split search on the folded
        histogram picks only coarse boundaries (ties go to the lower code).
        Random draws the cut subset per (tree, level, node, feature); a
        RoundRobin tree on QuantilesGlobal keeps only the boundaries next to the
        global quantiles.  Categorical features and the NA bin are untouched."""
        ht = self._tree_hist_type()
        if ht not in ("uniformadaptive", "random", "quantilesglobal") or \
                getattr(self.bd, "hist_type", "auto") not in ("uniformadaptive", "random", "roundrobin"):
            return H
        Fl, n, Bs, C = H.shape
        B = Bs - 1
        depth = getattr(self, "_depth", 0)
        # bins per node: nbins_top_level at the root AND its children, halved per
        # level below (the reference fixture's splits, gbm_variable_importance.zip,
        # sit on 1024 / 512 / 256 / 128 cells of the parent's range at depths 1-4)
        nb = max(self.bd.nbins_top >> max(depth - 1, 0), self.bd.nbins_node)
        f0 = self.f0
        isnum = ~self.is_cat_t[f0:f0 + Fl]
        if ht == "uniformadaptive" and nb >= B:
            return H
        dev = H.device
        if ht == "uniformadaptive" and dev.type == "cuda" and C <= 4 and tree_ops.env("H2O3_UA_FOLD") != "torch":
            return self._adapt_hist_dev(H, Fl, n, Bs, C, nb, isnum, depth)
        Hn = H[:, :, :B]
        occ = (Hn != 0).any(-1)                                   # [Fl, n, B]
        idx = torch.arange(B, device=dev)
        first = torch.where(occ, idx, B).amin(-1, keepdim=True)
        last = torch.where(occ, idx, -1).amax(-1, keepdim=True)
        first, last = self._adapt_range(first, last, n, Fl, depth)
        L = (last - first + 1).clamp(min=1)
        inr = (idx >= first) & (idx <= last)
        if ht == "uniformadaptive":
            coarse = torch.div((idx - first).clamp(min=0) * nb, L, rounding_mode="floor")
            nxt = torch.div((idx + 1 - first).clamp(min=0) * nb, L, rounding_mode="floor")
            is_end = inr & ((coarse != nxt) | (idx == last))
            is_end = is_end | (inr & (L <= nb))                   # narrow range: every boundary
        elif ht == "random":
            # per (tree, level, node, feature, bin) uniform draw: keep ~nb - 1 cuts
            key = (torch.arange(Fl, device=dev).view(-1, 1, 1) + f0) * 1000003 + \
                torch.arange(n, device=dev).view(1, -1, 1) * 7919 + idx.view(1, 1, -1) * 104729 + \
                (int(self.p.seed) * 31 + getattr(self, "_tree_no", 0) * 131 + depth * 17)
            key = (key * 0x9E3779B1) & 0xFFFFFFFF
            key = ((key ^ (key >> 15)) * 0x2C1B3C6D) & 0xFFFFFFFF
            u = (key ^ (key >> 12)).to(torch.float64) / 4294967296.0
            pk = ((nb - 1) / (L - 1).clamp(min=1).to(torch.float64))
            is_end = inr & ((u < pk) | (idx == last))
        else:
            qm = self.__dict__.get("_qmask")
            if qm is None:
                qm = torch.zeros((self.Fpad, B), dtype=torch.bool, device=dev)
                for j, qb in enumerate(self.bd.qbounds or []):
                    if qb is not None and len(qb):
                        qm[j, torch.as_tensor(np.minimum(qb, B - 1), device=dev)] = True
                self._qmask = qm
            is_end = inr & (qm[f0:f0 + Fl].view(Fl, 1, B) | (idx == last))
        is_end = is_end | ~isnum.view(Fl, 1, 1)                   # categorical: unchanged
        cs = torch.cumsum(Hn.to(torch.float64), 2)
        E = torch.where(is_end, idx, -1)
        pe_incl = torch.cummax(E, 2).values
        pe = torch.cat([torch.full_like(pe_incl[:, :, :1], -1), pe_incl[:, :, :-1]], 2)
        base = torch.where((pe >= 0).unsqueeze(-1), torch.gather(cs, 2, pe.clamp(min=0).unsqueeze(-1).expand(-1, -1, -1, C)),
                           torch.zeros_like(cs))
        Hf = torch.where(is_end.unsqueeze(-1), cs - base, torch.zeros_like(cs)).to(H.dtype)
        Hf = torch.where(isnum.view(Fl, 1, 1, 1), Hf, Hn)
        return torch.cat([Hf, H[:, :, B:]], 2).contiguous()

    def _adapt_hist_dev(self, H, Fl, n, Bs, C, nb, isnum, depth):
        """UniformAdaptive fold on the device (tree_split.hip ua_range_kernel /
        ua_fold_kernel): the same first / last, parent-range rule and run-end
        folding as the torch chain of _adapt_hist, one wave per (feature,
        node) row, H read twice and written once."""
        import ctypes
        from ...ops import _native
        lib = _native.get_lib("tree_split")
        if lib is None:
            raise RuntimeError("tree_split native library missing (UniformAdaptive fold)")
        if not getattr(lib, "_typed_ua", False):
            cv, ci = ctypes.c_void_p, ctypes.c_int
            lib.h2o_ua_range.argtypes = [cv, ci, ci, ci, cv, cv, cv]
            lib.h2o_ua_fold.argtypes = [cv, ci, ci, ci, ci, cv, cv, ci, cv, cv, cv]
            lib._typed_ua = True
        H = H.contiguous()
        rows = Fl * n
        fl = torch.empty(2 * rows, dtype=torch.int32, device=H.device)
        s = tree_ops._stream()
        rc = lib.h2o_ua_range(ctypes.c_void_p(H.data_ptr()), rows, Bs, C, ctypes.c_void_p(fl.data_ptr()),
                              ctypes.c_void_p(fl.data_ptr() + 4 * rows), s)
        if rc != 0:
            raise RuntimeError(f"h2o_ua_range failed: {rc}")
        first, last = fl[:rows].view(Fl, n, 1).long(), fl[rows:].view(Fl, n, 1).long()
        first, last = self._adapt_range(first, last, n, Fl, depth)
        fr_ = first.to(torch.int32).contiguous()
        la_ = last.to(torch.int32).contiguous()
        isn = isnum.to(torch.uint8).contiguous()
        out = torch.empty_like(H)
        rc = lib.h2o_ua_fold(ctypes.c_void_p(H.data_ptr()), Fl, n, Bs, C, ctypes.c_void_p(fr_.data_ptr()),
                             ctypes.c_void_p(la_.data_ptr()), int(nb), ctypes.c_void_p(isn.data_ptr()),
                             ctypes.c_void_p(out.data_ptr()), s)
        if rc != 0:
            raise RuntimeError(f"h2o_ua_fold failed: {rc}")
        return out

    def _adapt_range(self, first, last, n, Fl, depth):
        """Code range [first, last] ([Fl, n, 1]) each node's coarse bins span.
        The reference bins a child over its PARENT's observed range of each
        column, and the split column over the parent's range cut at the split
        (DTree.java:337-372, nextLevelHistos); at depth 1 the coarse grid is
        then exactly every (1024 >> 1)-th top-level cell.  The node's own
        occupied range is recorded for its children; without a parent record
        (root, chunk / frontier shapes that do not line up) the node's own
        range is used."""
        off = getattr(self, "_bnd_off", 0)
        cur = self.__dict__.get("_rng_cur")
        n_level = off + n if cur is None or off == 0 else max(cur[0].shape[1], off + n)
        if cur is None or off == 0 or cur[0].shape[1] < n_level:
            nf = torch.zeros((Fl, n_level, 1), dtype=first.dtype, device=first.device)
            nl = torch.zeros_like(nf)
            if cur is not None and off > 0:
                k = min(cur[0].shape[1], n_level)
                nf[:, :k], nl[:, :k] = cur[0][:, :k], cur[1][:, :k]
            cur = self._rng_cur = (nf, nl)
        cur[0][:, off:off + n], cur[1][:, off:off + n] = first, last
        par = self.__dict__.get("_adapt_par")
        rp = self.__dict__.get("_rng_par")
        if depth == 0 or par is None or rp is None or rp[0].shape[0] != Fl:
            return first, last
        sids, fs, ts, opts, n_front = par
        if 2 * len(sids) != n_front or off + n > n_front:
            return first, last
        j = np.arange(off, off + n)
        pi = torch.as_tensor(sids[j // 2], device=first.device)
        pf, pl = rp[0][:, pi].clone(), rp[1][:, pi].clone()       # [Fl, n, 1]
        # the split column: left child codes <= t, right child codes > t
        fl = fs[j // 2] - self.f0
        ok = (fl >= 0) & (fl < Fl) & (opts[j // 2] != 2)
        if ok.any():
            jj = np.nonzero(ok)[0]
            side = (j[jj] % 2).astype(bool)
            t = torch.as_tensor(ts[j // 2][jj], device=first.device, dtype=first.dtype)
            fi = torch.as_tensor(fl[jj], device=first.device)
            ji = torch.as_tensor(jj, device=first.device)
            sd = torch.as_tensor(side, device=first.device)
            cf, cl = pf[fi, ji, 0], pl[fi, ji, 0]
            pf[fi, ji, 0] = torch.where(sd, torch.maximum(cf, t + 1), cf)
            pl[fi, ji, 0] = torch.where(sd, cl, torch.minimum(cl, t))
        # empty nodes / columns keep their own (empty) range
        use = (pf <= pl) & (first <= last)
        return torch.where(use, pf, first), torch.where(use, pl, last)

    def _find_splits(self, H, col_mask, node_wyy=None, want_pk=False):
        """Dispatch: fused HIP kernel for numeric features on GPU (categorical
        features, which need a per-node sort of bins, go through the torch path)."""
        H = self._adapt_hist(H)
        if self.dev.type != "cuda" or self.p.criterion.startswith("uplift"):
            Fl_ = H.shape[0]
            cmf = col_mask[:, self.f0:self.f0 + Fl_]
            if not self.p.criterion.startswith("uplift") and cmf.numel() and float(cmf.float().mean()) < 0.5:
                # few eligible features per node (DRF mtries): score only those pairs
                res = self._cat_splits_pairs(H, col_mask, list(range(Fl_)), node_wyy)
                res = self._bound_winners(res)
                res["tot"] = H[0].to(torch.float64).sum(1) if Fl_ > 0 else None
                if self.W > 1:
                    res = self._merge_candidates(res, H.shape[1], H.shape[2], H.shape[3])
                return res
            return self._find_splits_torch(H, col_mask, node_wyy)
        Fl = H.shape[0]
        fsl = slice(self.f0, self.f0 + Fl)
        if getattr(self, "_is_cat_cpu", None) is None:
            self._is_cat_cpu = self.is_cat_t[fsl].cpu()
        is_cat = self._is_cat_cpu
        if bool(is_cat.all()):
            return self._find_splits_torch(H, col_mask, node_wyy)
        if not bool(is_cat.any()):
            # want_pk on a numeric-only frame: every rank takes the packed-record
            # path (split_select2 + one record merge), so the collectives match
            res = self._find_splits_native(H, col_mask, node_wyy,
                                           want_pk=want_pk and not any(self.bd.is_cat))
            if self.W > 1 and "pk" not in res:
                res = self._merge_candidates(res, H.shape[1], H.shape[2], H.shape[3])
            return res
        cm_num = col_mask.clone()
        cm_num[:, fsl] &= ~is_cat.to(cm_num.device).view(1, -1)
        res = self._find_splits_native(H, cm_num, node_wyy)
        if bool(is_cat.any()):
            cat_local = torch.nonzero(is_cat).flatten().tolist()
            rc = self._bound_winners(self._cat_splits_pairs(H, col_mask, cat_local, node_wyy))
            better = rc["gain"] > res["gain"]
            for k in res:
                if res[k] is None or k == "tot":
                    continue
                b = better.view(-1, *([1] * (res[k].dim() - 1))) if res[k].dim() > 1 else better
                res[k] = torch.where(b, rc[k].to(res[k].dtype), res[k])
        if self.W > 1:
            res = self._merge_candidates(res, H.shape[1], H.shape[2], H.shape[3])
        return res

    def _find_splits_native(self, H, col_mask, node_wyy, want_pk=False):
        import ctypes
        from ...ops import _native
        p = self.p
        Fl, n, Bs, C = H.shape
        lib = _native.get_lib("tree_split")
        if not getattr(lib, "_typed", False):
            cv = ctypes.c_void_p
            lib.h2o_split_find.argtypes = [cv, ctypes.c_int, ctypes.c_int, ctypes.c_int, cv, cv, cv] + \
                [ctypes.c_double] * 5 + [ctypes.c_int, cv, cv]
            lib._typed = True
        fsl = slice(self.f0, self.f0 + Fl)
        cm = col_mask[:, fsl]
        if getattr(col_mask, "_all_true", False) and self.f0 + Fl <= self.bd.F:
            # no column sampling: a cached device mask of ones per frontier size
            cache = self.__dict__.setdefault("_ok_cache", {})
            ok = cache.get(n)
            if ok is None:
                ok = cache[n] = torch.ones((n, Fl), dtype=torch.uint8, device=self.dev)
        else:
            ok = cm.to(torch.uint8).contiguous()
            ok = tree_ops._h2d(ok.numpy(), self.dev) if ok.device.type == "cpu" else ok
            if self.f0 + Fl > self.bd.F:
                ok[:, max(0, self.bd.F - self.f0):] = 0
        if getattr(self, "_mono_f32", None) is None:
            self._mono_f32 = self.mono_t[fsl].to(torch.float32).contiguous()
        mono = self._mono_f32
        H = H.contiguous()
        wyy = node_wyy.to(torch.float64).contiguous() if node_wyy is not None else \
            torch.zeros(n, dtype=torch.float64, device=self.dev)
        out = torch.empty((n * Fl, 4), dtype=torch.float64, device=self.dev)
        crit = 1 if p.criterion == "xgb" else 0
        bnd = self._bnd_dev(n)
        if not getattr(lib, "_typed_b", False):
            cv = ctypes.c_void_p
            lib.h2o_split_find_b.argtypes = [cv, ctypes.c_int, ctypes.c_int, ctypes.c_int, cv, cv, cv] + \
                [ctypes.c_double] * 5 + [ctypes.c_int, cv, cv, ctypes.c_int, cv]
            lib._typed_b = True
        rc = lib.h2o_split_find_b(ctypes.c_void_p(H.data_ptr()), Fl, n, Bs, ctypes.c_void_p(wyy.data_ptr()),
                                  ctypes.c_void_p(ok.data_ptr()), ctypes.c_void_p(mono.data_ptr()),
                                  float(p.min_rows), float(p.min_split_improvement), float(p.reg_lambda),
                                  float(p.reg_alpha), float(p.gamma), crit, ctypes.c_void_p(out.data_ptr()),
                                  ctypes.c_void_p(0 if bnd is None else bnd.data_ptr()), int(bool(p.use_bounds)),
                                  tree_ops._stream())
        if rc != 0:
            raise RuntimeError(f"h2o_split_find failed: {rc}")
        if C == 2 and want_pk and (self.W > 1 or self.f0 < self.bd.F):
            # selection + split decision + partition inputs in one kernel; the
            # packed record (12 doubles per node) is what the host fetches
            if not getattr(lib, "_typed_sel2", False):
                cv = ctypes.c_void_p
                lib.h2o_split_select2.argtypes = [cv, cv, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_double, ctypes.c_int, cv, cv, cv, cv]
                lib._typed_sel2 = True
            # 13 fields: split_select2's 12 + the node's NA weight on the chosen column
            pk = torch.empty((n, 13), dtype=torch.float64, device=self.dev)
            mask = torch.empty((n, Bs), dtype=torch.uint8, device=self.dev)
            feat_i = torch.empty(n, dtype=torch.int32, device=self.dev)
            if self.f0 < self.bd.F:
                min_w2 = -1.0 if p.criterion == "xgb" else 2.0 * float(p.min_rows)
                rc = lib.h2o_split_select2(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(H.data_ptr()), Fl, n,
                                           Bs, self.f0, min_w2, 13, ctypes.c_void_p(pk.data_ptr()),
                                           ctypes.c_void_p(mask.data_ptr()), ctypes.c_void_p(feat_i.data_ptr()),
                                           tree_ops._stream())
                if rc != 0:
                    raise RuntimeError(f"h2o_split_select2 failed: {rc}")
            else:
                # a rank holding only padding features: a never-winning record
                pk.zero_()
                pk[:, 0] = NEG_INF
                mask.zero_()
                feat_i.zero_()
            if self.W > 1:
                pk, mask, feat_i = self._merge_records(pk, mask)
            return {"pk": pk, "feat_i32": feat_i, "mask": mask, "gain": pk[:, 0], "feat": pk[:, 1], "t": pk[:, 2],
                    "opt": pk[:, 3], "L": pk[:, 4:6], "R": pk[:, 6:8], "tot": pk[:, 8:10]}
        if C == 2 and self.f0 < self.bd.F:
            # fused per-node selection + mask kernel: few launches, one packed record
            if not getattr(lib, "_typed_sel", False):
                cv = ctypes.c_void_p
                lib.h2o_split_select.argtypes = [cv, cv, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, cv,
                                                 cv, cv]
                lib._typed_sel = True
            pk = torch.empty((n, 10), dtype=torch.float64, device=self.dev)
            mask = torch.empty((n, Bs), dtype=torch.uint8, device=self.dev)
            rc = lib.h2o_split_select(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(H.data_ptr()), Fl, n, Bs,
                                      self.f0, ctypes.c_void_p(pk.data_ptr()), ctypes.c_void_p(mask.data_ptr()),
                                      tree_ops._stream())
            if rc != 0:
                raise RuntimeError(f"h2o_split_select failed: {rc}")
            opt = pk[:, 3].long()
            return {"gain": pk[:, 0], "feat": pk[:, 1].long(), "t": pk[:, 2].long(), "opt": opt,
                    "na_left": opt == 1, "mask": mask, "L": pk[:, 4:6], "R": pk[:, 6:8], "tot": pk[:, 8:10]}
        gain = out[:, 0].view(n, Fl)
        ints = out.view(torch.int32).view(n * Fl, 8)[:, 6:8]
        best, fl = gain.max(1)
        idx = torch.arange(n, device=self.dev) * Fl + fl
        t = ints[idx, 0].long()
        opt = ints[idx, 1].long()
        Lw = out[idx, 1:3]
        T = H[0].sum(1) if self.f0 < self.bd.F else torch.zeros((n, C), dtype=H.dtype, device=H.device)
        B = Bs - 1
        codes = torch.arange(Bs, device=self.dev).view(1, Bs)
        mask = (codes <= t.view(n, 1)) & (codes < B)
        mask = torch.where((opt == 2).view(n, 1), codes < B, mask)
        mask[:, Bs - 1] = opt == 1
        return {"gain": best, "feat": fl + self.f0, "t": t, "opt": opt, "na_left": opt == 1,
                "mask": mask.to(torch.uint8), "L": Lw, "R": T - Lw, "tot": T}

    def _cat_splits_pairs(self, H, col_mask, sub, node_wyy):
        """Categorical splits scored only on the eligible (node, feature) pairs
        (mtries / column sampling usually leave a few per node): levels sorted
        by mean response per pair (DTree.findBestSplitPoint for categoricals),
        prefix sums, the three NA options, best pair per node by a segment
        arg-max (lowest feature on ties).  On the GPU every pair is one
        workgroup of the HIP kernel `cat_pair_kernel` (tree_split.hip); the
        winners' split masks are then rebuilt from their own bins."""
        p = self.p
        Fl, n, Bs, C = H.shape
        B = Bs - 1
        dev = H.device
        sub_t = torch.as_tensor(sub, dtype=torch.long, device=dev)
        gidx = sub_t + self.f0
        cm = col_mask.to(dev)[:, gidx] & (gidx < self.bd.F).view(1, -1)
        nz = torch.nonzero(cm)
        ninf = torch.full((n,), NEG_INF, dtype=torch.float64, device=dev)
        out = {"gain": ninf, "feat": torch.zeros(n, dtype=torch.long, device=dev),
               "t": torch.zeros(n, dtype=torch.long, device=dev), "opt": torch.zeros(n, dtype=torch.long, device=dev),
               "na_left": torch.zeros(n, dtype=torch.bool, device=dev),
               "mask": torch.zeros((n, Bs), dtype=torch.uint8, device=dev),
               "L": torch.zeros((n, C), dtype=torch.float64, device=dev),
               "R": torch.zeros((n, C), dtype=torch.float64, device=dev), "tot": None}
        if nz.shape[0] == 0:
            return out
        node_i, j = nz[:, 0], nz[:, 1]
        pcat = self.is_cat_t[gidx[j]]                              # numeric pairs keep bin order
        mono_p = self.mono_t[gidx[j]]
        if dev.type == "cuda" and C >= 2 and B <= 4096 and H.dtype == torch.float64:
            best, k = self._pairs_native(H, sub_t[j], node_i, pcat, mono_p, node_wyy)
        else:
            st = self._pair_stats(H[sub_t[j], node_i].to(torch.float64), pcat)
            allg = self._pair_gains(st, mono_p.view(-1, 1), node_wyy, node_i)
            best, k = allg.max(1)
        return self._pair_winners(out, best, k, node_i, gidx[j], pcat, lambda wp: H[sub_t[j[wp]], node_i[wp]])

    def _sample_k(self, depth):
        """(k, n_eligible): columns scored per node at this depth."""
        p = self.p
        base_n = self.bd.F if p.tree_col_mask is None else int(np.count_nonzero(p.tree_col_mask))
        rate = p.col_sample_rate * (p.col_sample_rate_change_per_level ** depth)
        if p.mtries is not None and p.mtries > 0:
            k = p.mtries
        elif rate < 1.0:
            k = max(1, int(math.floor(rate * base_n + 0.5)))
        else:
            k = base_n
        return min(k, base_n), base_n

    def _sampled_cols(self, depth):
        """True when the split search at this depth sees a per-node subset
        of the columns (mtries / col_sample_rate(_change_per_level) /
        col_sample_rate_per_tree)."""
        k, ne = self._sample_k(depth)
        return k < self.bd.F

    def _direct_level(self, mode, depth, chunked):
        """Row-direct pair histograms for this level (tree_ops.pair_hist):
        column-sampled splits where at most a quarter of the features are
        scored per node (DRF's sqrt(F) mtries) or the level histogram would
        need node batching (H2O3_PAIR_DIRECT=auto); at every sampled level
        (=1); never (=0).  Measured on the DRF config (10M x 500, 100
        categoricals of cardinality 1000): 995 ms/tree with level histograms,
        ~500 ms/tree with pair histograms at every sampled level."""
        env = tree_ops.env("H2O3_PAIR_DIRECT", "auto")
        if env == "0" or mode not in (0, 1) or self.p.criterion.startswith("uplift") or \
                not self._sampled_cols(depth):
            return False
        if self.dev.type == "cuda" and self.bd.codes_col is None:
            return False
        k, _ = self._sample_k(depth)
        return env == "1" or chunked or 4 * k <= self.bd.F

    def _flush_masks(self, tb):
        """Collect the categorical mask rows of the previous level from the
        pinned staging buffer into the tree (waits on the copy's event: by the
        time the next level's record arrived it has completed)."""
        pend = self.__dict__.get("_mask_pend")
        if pend is None:
            return
        nodes, feats, shape, ev = pend
        ev.synchronize()
        n = int(np.prod(shape))
        tb.cat_parts.append((nodes, feats, self._mask_stage[:n].numpy().reshape(shape).copy()))
        self._mask_pend = None

    def _narrow_bins(self):
        """Per-feature code counts [F] int32 on the device when the pair path
        may bound its work by each feature's bins (histograms wider than 256
        bins: H2O3_PAIR_NARROW), else None."""
        if self.dev.type != "cuda" or self.bd.Bs - 1 <= 256 or tree_ops.env("H2O3_PAIR_NARROW", "1") != "1":
            return None
        if getattr(self, "_nbins_t", None) is None:
            nb = np.minimum(np.asarray(self.bd.nbins[:self.bd.F], dtype=np.int64), self.bd.Bs - 1)
            self._nbins_t = torch.as_tensor(nb.astype(np.int32), device=self.dev)
        return self._nbins_t

    def _all_levels_direct(self, mode):
        """True when every level of the tree takes the device pair path (a
        fixed per-node column sample of at most a quarter of the features),
        so no level-histogram kernel ever reads the response by row."""
        p = self.p
        if mode != 0 or self.dev.type != "cuda" or self.bd.codes_col is None or p.criterion.startswith("uplift"):
            return False
        if tree_ops.env("H2O3_PAIR_DIRECT", "auto") == "0":
            return False
        if not (p.mtries is not None and p.mtries > 0) or p.col_sample_rate_change_per_level != 1.0:
            return False
        k, _ = self._sample_k(0)
        return k < self.bd.F and 4 * k <= self.bd.F

    def _pair_direct_splits(self, ridx, va, vb, mode, f_st, f_ct, cm):
        """Best split of every frontier node from row-direct histograms of its
        sampled (node, feature) pairs only: pair histograms built from the rows
        (HIP `pair_hist_kernel`), scored per pair (`cat_pair_kernel`: numeric
        bin order or categorical levels sorted by mean response, three NA
        options), per-node winner + mask (_pair_winners).  Pairs are processed
        in node batches under hist_mem_budget.  Every rank sums the pair
        histograms (all-reduce) and scores all pairs, so no candidate merge."""
        p = self.p
        bd, dev = self.bd, self.dev
        F, Bs, C = bd.F, bd.Bs, 2
        n = len(f_st)
        posv = False
        if mode == 0 and getattr(self, "_pos1", None) is not None:
            va, vb, posv = self._pos1[0], None, True
        elif mode == 0 and getattr(self, "_va_eff", None) is not None:
            va, vb = self._va_eff, None
        st = np.asarray(f_st, dtype=np.int64)
        ct = np.asarray(f_ct, dtype=np.int64)
        nz = torch.nonzero(cm[:, :F]).cpu().numpy()           # node-major pairs
        pn_all, pf_all = nz[:, 0].astype(np.int64), nz[:, 1].astype(np.int64)
        per_pairs = max(1, int(p.hist_mem_budget // (Bs * C * 8)))
        cum = np.cumsum(np.bincount(pn_all, minlength=n))     # pairs of nodes [0, i]
        parts = []
        a = 0
        while a < n:
            base = int(cum[a - 1]) if a > 0 else 0
            b = min(n, max(a + 1, int(np.searchsorted(cum, base + per_pairs, side="right"))))
            lo, hi = base, int(cum[b - 1])
            parts.append(self._pair_direct_part(ridx, va, vb, mode, posv, st[a:b], ct[a:b], pn_all[lo:hi] - a,
                                                pf_all[lo:hi]))
            a = b
        if len(parts) == 1:
            return parts[0]
        return {k: torch.cat([q[k] for q in parts], 0) for k in parts[0]}

    def _pair_direct_dev(self, ridx, va, vb, mode, f_st, f_ct, sel):
        """Device-resident version of _pair_direct_splits: pairs from the
        [n, k] column sample on the device, pair histograms
        (pair_hist_kernel), per-pair scoring (cat_pair_kernel) and the
        per-node winner / record / mask (pair_select_kernel) -- the level's
        split record comes out in the packed form of split_select2, so the
        async partition and the single host transfer of the level apply."""
        import ctypes
        from ...ops import _native
        p = self.p
        bd, dev = self.bd, self.dev
        Bs = bd.Bs
        if sel is None:
            # no per-node sampling (only the per-tree column mask): every eligible feature
            base = np.ones(bd.F, dtype=bool) if p.tree_col_mask is None else p.tree_col_mask.astype(bool)
            elig = torch.as_tensor(np.nonzero(base)[0], device=dev)
            sel = elig.view(1, -1).expand(len(f_st), -1)
        n, k = sel.shape
        posv = False
        if mode == 0 and getattr(self, "_pos1", None) is not None:
            va, vb, posv = self._pos1[0], None, True
        elif mode == 0 and getattr(self, "_va_eff", None) is not None:
            va, vb = self._va_eff, None
        lib = _native.get_lib("tree_split")
        if not getattr(lib, "_typed_psel", False):
            cv, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
            lib.h2o_pair_select.argtypes = [cv, ci, ci, ci, cv, cv, cv, ci, cd, ci, cv, cv, cv, cv]
            lib._typed_psel = True
        if getattr(self, "_fcat_u8", None) is None:
            self._fcat_u8 = self.is_cat_t[:bd.F].to(torch.uint8).contiguous()
        st = np.asarray(f_st, dtype=np.int64)
        ct = np.asarray(f_ct, dtype=np.int64)
        per = max(1, int(p.hist_mem_budget // (k * Bs * 2 * 8)))
        pk = torch.empty((n, 13), dtype=torch.float64, device=dev)
        mask = torch.empty((n, Bs), dtype=torch.uint8, device=dev)
        feat_i = torch.empty(n, dtype=torch.int32, device=dev)
        min_w2 = -1.0 if p.criterion == "xgb" else 2.0 * float(p.min_rows)
        for a in range(0, n, per):
            b = min(n, a + per)
            sl = sel[a:b]
            with phase("tree.hist"), phase("tree.hist.pairs"):
                Hp, wyy_n, pfeat = tree_ops.pair_hist_dev(bd, ridx, va, vb, mode, st[a:b], ct[a:b], sl, self._vmax,
                                                          posv=posv, fbins=self._narrow_bins())
            nb = b - a
            if self.W > 1:
                # node-sharded reduction: every rank receives the summed pair
                # histograms of 1/W of the nodes, packed at each feature's own
                # width (sparse at deep levels: _pair_exchange), scores and
                # selects those nodes, and only the small per-node records are
                # all-gathered
                W = self.W
                npad = -(-nb // W) * W
                wv = wyy_n if wyy_n is not None else torch.zeros(nb, dtype=torch.float64, device=dev)
                nl = npad // W
                lo = self.rank * nl
                pn_all = torch.arange(nb, device=dev).repeat_interleave(k)
                Hmine = self._pair_exchange(Hp.view(nb * k, Bs, 2), pfeat.long(), pn_all, nb, full=False)
                if npad > nb:
                    wv = torch.cat([wv, torch.zeros(npad - nb, dtype=wv.dtype, device=dev)], 0)
                    pfeat = torch.cat([pfeat, torch.zeros((npad - nb) * k, dtype=pfeat.dtype, device=dev)], 0)
                Hl = torch.zeros((nl * k, Bs, 2), dtype=Hp.dtype, device=dev)
                Hl[:Hmine.shape[0]] = Hmine
                wl = coll.reduce_scatter_dim0(wv.contiguous()) if wyy_n is not None else None
                del Hp, Hmine
                pk_l = torch.empty((nl, 13), dtype=torch.float64, device=dev)
                mask_l = torch.empty((nl, Bs), dtype=torch.uint8, device=dev)
                feat_l = torch.empty(nl, dtype=torch.int32, device=dev)
                self._pair_score_select(lib, Hl, nl, k, pfeat[lo * k:(lo + nl) * k].contiguous(), wl, min_w2,
                                        pk_l, mask_l, feat_l)
                pk[a:b] = coll.all_gather_dim0(pk_l)[:nb]
                mask[a:b] = coll.all_gather_dim0(mask_l)[:nb]
                feat_i[a:b] = coll.all_gather_dim0(feat_l)[:nb]
                continue
            self._pair_score_select(lib, Hp, nb, k, pfeat, wyy_n, min_w2, pk[a:b], mask[a:b], feat_i[a:b])
            del Hp
        return {"pk": pk, "feat_i32": feat_i, "mask": mask, "gain": pk[:, 0], "feat": pk[:, 1].long(),
                "t": pk[:, 2].long(), "opt": pk[:, 3].long(), "L": pk[:, 4:6], "R": pk[:, 6:8], "tot": pk[:, 8:10],
                "naw": pk[:, 12]}

    # ------------------------------------------------------------------ multi-GPU pair exchange
    def _pair_exchange(self, Hp, pf, pn, n, full):
        """Sum the (node, feature) pair histograms of every rank without
        shipping empty bins.  Hp: [P, Bs, C] dense rows of node-major pairs
        (pair p belongs to node pn[p], feature pf[p]); node q is owned by rank
        q // ceil(n / W).

        Each pair row is packed at its feature's OWN width (bins + NA: <= 256
        for the numeric columns, the cardinality for a categorical) instead of
        the frame-wide stride Bs, the packed rows of every owner are laid out
        back to back, and the level is summed either by ONE reduce-scatter of
        the packed [W, Lmax] buffer or -- when the bins that are non-zero on
        the busiest rank cost less than half of that (deep levels: nodes of a
        few dozen rows fill a few bins of each 1000-level histogram) -- by ONE
        all_to_all of (position, value) pairs summed by the owner.  Returns the
        owner's dense [P_own, Bs, C] rows (pairs of its nodes, in order), or
        with full=True every pair's summed dense row (packed all-gather).
        Reference: hex/tree/DHistogram.java:366 -- the reference ships
        per-node histograms of nbins = 20 numeric bins."""
        W, r = self.W, self.rank
        dev = Hp.device
        P, Bs, C = Hp.shape
        nl = -(-n // W)
        if getattr(self, "_pw_t", None) is None or self._pw_t.device != dev:
            nb = np.minimum(np.asarray(self.bd.nbins[:self.bd.F], dtype=np.int64), Bs - 1) + 1
            self._pw_t = torch.as_tensor(nb, device=dev)
        w = self._pw_t[pf]
        owner = torch.div(pn, nl, rounding_mode="floor")
        cw = torch.cumsum(w, 0)
        start = cw - w
        E = int(cw[-1]) if P else 0
        own_cnt = torch.bincount(owner, minlength=W)
        own_first = torch.cumsum(own_cnt, 0) - own_cnt                  # first pair of each owner
        ch_start = torch.where(own_cnt > 0, start[own_first.clamp(max=max(P - 1, 0))] if P else own_cnt,
                               torch.zeros_like(own_cnt))
        Lq = torch.zeros(W, dtype=torch.int64, device=dev).index_add_(0, owner, w)
        Lh = Lq.tolist()
        Lmax = max(1, max(Lh))
        # element index arrays in int32 when they fit (a deep DRF level holds
        # 1e8 packed bins: 4 bytes instead of 8 per bin and array)
        it = torch.int32 if P * Bs < 2 ** 31 and E < 2 ** 31 else torch.int64
        pe = torch.repeat_interleave(torch.arange(P, device=dev, dtype=it), w)   # element -> pair
        j = torch.arange(E, device=dev, dtype=it) - start.to(it)[pe]            # element -> packed bin
        dense_idx = pe * Bs + torch.where(j == w.to(it)[pe] - 1, torch.full_like(j, Bs - 1), j)
        oe = owner.to(it)[pe]
        pos = start.to(it)[pe] + j - ch_start.to(it)[oe]                      # position in its owner's chunk
        del pe, j
        vals = Hp.reshape(P * Bs, C)[dense_idx]                          # [E, C]
        nzm = (vals != 0).any(1)
        nnz = int(nzm.sum())
        # lossless integer transport: unweighted / bootstrap-count classification
        # histograms hold whole numbers (w = counts, wy = class counts); when every
        # rank's values are integers below 2^27 the level ships int32 (a sum of
        # 8 ranks stays exact), half the bytes of f64
        big = float(vals.abs().max()) if vals.numel() else 0.0
        not_int = 0.0 if big < 2.0 ** 27 else 1.0
        step_ = 1 << 24
        for a_ in range(0, vals.shape[0] if not_int == 0.0 else 0, step_):
            v_ = vals[a_:a_ + step_]
            if bool((v_ != torch.round(v_)).any()):
                not_int = 1.0
                break
        stat = torch.tensor([float(nnz), not_int], dtype=torch.float64, device=dev)
        coll.allreduce_(stat, "max")
        ints = float(stat[1]) == 0.0
        vb_ = 4 if ints else 8
        dense_b = W * Lmax * C * vb_
        tdt = torch.int32 if ints else Hp.dtype
        if float(stat[0]) * (4 + vb_ * C) < dense_b:
            # sparse: (position, value) of the non-zero bins to their owner, when
            # that ships fewer bytes than the dense reduce-scatter
            from ...core.dist_munge import exchange
            from ...core.vec import T_INT, T_REAL, Vec
            vsend = vals[nzm].to(tdt).contiguous()
            got = exchange([Vec(pos[nzm].to(torch.int32), T_INT), Vec(vsend, T_INT if ints else T_REAL)], oe[nzm])
            chunk = torch.zeros((Lmax, C), dtype=Hp.dtype, device=dev).index_add_(
                0, got[0].data.long(), got[1].data.to(Hp.dtype))
        else:
            buf = torch.zeros((W, Lmax, C), dtype=tdt, device=dev)
            buf[oe, pos] = vals.to(tdt)
            chunk = coll.reduce_scatter_dim0(buf.view(W * Lmax, C)).to(Hp.dtype)
        if full:
            allc = coll.all_gather_dim0(chunk.to(tdt)).view(W, Lmax, C).to(Hp.dtype)
            out = torch.zeros((P * Bs, C), dtype=Hp.dtype, device=dev)
            out[dense_idx] = allc[oe, pos]
            return out.view(P, Bs, C)
        mine = oe == r
        p0 = int(own_first[r]) if P else 0
        Pr = int(own_cnt[r])
        out = torch.zeros((max(Pr, 0) * Bs, C), dtype=Hp.dtype, device=dev)
        out[dense_idx[mine] - p0 * Bs] = chunk[pos[mine]]
        return out.view(Pr, Bs, C)

    def _pair_score_select(self, lib, Hp, n, k, pfeat, wyy_n, min_w2, pk, mask, feat_i):
        """Score the n*k pairs of Hp (cat_pair_kernel) and write the n nodes'
        records / masks / features (pair_select_kernel) into the given
        contiguous output views."""
        import ctypes
        p = self.p
        dev = self.dev
        Bs = self.bd.Bs
        P = n * k
        if n <= 0:
            return
        fl = pfeat.long()
        nb_t = self._narrow_bins()
        best_k = self._pairs_native(Hp.view(1, P, Bs, 2), torch.zeros(P, dtype=torch.long, device=dev),
                                    torch.arange(P, device=dev), self.is_cat_t[fl], self.mono_t[fl],
                                    wyy_n.repeat_interleave(k) if wyy_n is not None else None, raw=True,
                                    pbins=nb_t[fl] if nb_t is not None else None)
        if nb_t is not None:
            if not getattr(lib, "_typed_psel2", False):
                cv, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
                lib.h2o_pair_select2.argtypes = [cv, ci, ci, ci, cv, cv, cv, ci, cd, ci, cv, cv, cv, cv, cv]
                lib._typed_psel2 = True
            rc = lib.h2o_pair_select2(ctypes.c_void_p(Hp.data_ptr()), n, Bs, k, ctypes.c_void_p(best_k.data_ptr()),
                                      ctypes.c_void_p(pfeat.data_ptr()), ctypes.c_void_p(self._fcat_u8.data_ptr()),
                                      1 if p.criterion == "xgb" else 0, min_w2, pk.stride(0), ctypes.c_void_p(pk.data_ptr()),
                                      ctypes.c_void_p(mask.data_ptr()), ctypes.c_void_p(feat_i.data_ptr()),
                                      ctypes.c_void_p(nb_t.data_ptr()), tree_ops._stream())
        else:
            rc = lib.h2o_pair_select(ctypes.c_void_p(Hp.data_ptr()), n, Bs, k, ctypes.c_void_p(best_k.data_ptr()),
                                     ctypes.c_void_p(pfeat.data_ptr()), ctypes.c_void_p(self._fcat_u8.data_ptr()),
                                     1 if p.criterion == "xgb" else 0, min_w2, pk.stride(0), ctypes.c_void_p(pk.data_ptr()),
                                     ctypes.c_void_p(mask.data_ptr()), ctypes.c_void_p(feat_i.data_ptr()),
                                     tree_ops._stream())
        if rc != 0:
            raise RuntimeError(f"h2o_pair_select failed: {rc}")

    def _pair_direct_part(self, ridx, va, vb, mode, posv, st, ct, pn, pf):
        p = self.p
        dev = self.dev
        n = st.size
        Bs, C = self.bd.Bs, 2
        out = {"gain": torch.full((n,), NEG_INF, dtype=torch.float64, device=dev),
               "feat": torch.zeros(n, dtype=torch.long, device=dev),
               "t": torch.zeros(n, dtype=torch.long, device=dev), "opt": torch.zeros(n, dtype=torch.long, device=dev),
               "na_left": torch.zeros(n, dtype=torch.bool, device=dev),
               "mask": torch.zeros((n, Bs), dtype=torch.uint8, device=dev),
               "L": torch.zeros((n, C), dtype=torch.float64, device=dev),
               "R": torch.zeros((n, C), dtype=torch.float64, device=dev),
               "tot": torch.zeros((n, C), dtype=torch.float64, device=dev),
               "naw": torch.zeros(n, dtype=torch.float64, device=dev)}
        with phase("tree.hist"), phase("tree.hist.pairs"):
            Hp, wyy_n = tree_ops.pair_hist(self.bd, ridx, va, vb, mode, st, ct, pn, pf, vmax=self._vmax, posv=posv,
                                           want_wyy=mode == 0)
        if self.W > 1:
            if pn.size:
                Hp = self._pair_exchange(Hp, tree_ops._h2d(pf, dev), tree_ops._h2d(pn, dev), n, full=True)
            if wyy_n is not None:
                coll.allreduce_(wyy_n)
        P = pn.size
        if P == 0:
            return out
        pn_t = tree_ops._h2d(pn, dev)
        first = np.ones(P, dtype=bool)
        first[1:] = pn[1:] != pn[:-1]
        fi = np.nonzero(first)[0]
        out["tot"] = out["tot"].index_put((pn_t[tree_ops._h2d(fi, dev)],),
                                          Hp[tree_ops._h2d(fi, dev)].sum(1))
        fglob = tree_ops._h2d(pf, dev)
        pcat = self.is_cat_t[fglob]
        mono_p = self.mono_t[fglob]
        wyy_p = wyy_n[pn_t] if wyy_n is not None else None
        ar = torch.arange(P, device=dev)
        if dev.type == "cuda" and Bs - 1 <= 4096:
            best, k = self._pairs_native(Hp.view(1, P, Bs, C), torch.zeros(P, dtype=torch.long, device=dev), ar,
                                         pcat, mono_p, wyy_p)
        else:
            stt = self._pair_stats(Hp, pcat)
            allg = self._pair_gains(stt, mono_p.view(-1, 1), wyy_p, ar)
            best, k = allg.max(1)
        return self._pair_winners(out, best, k, pn_t, fglob, pcat, lambda wp: Hp[wp])

    def _pair_winners(self, out, best, k, node_i, fglob, pcat, hist_of):
        """Per-node winner among scored (node, feature) pairs (largest gain,
        lowest pair index on ties) and its split record: threshold / NA option
        from k, left statistics and the go-left code mask rebuilt from the
        winner's own bins (hist_of(wp) -> [len(wp), Bs, C])."""
        p = self.p
        n = out["gain"].shape[0]
        dev = best.device
        P = best.numel()
        ninf = torch.full((n,), NEG_INF, dtype=torch.float64, device=dev)
        B = self.bd.Bs - 1
        Bs = self.bd.Bs
        xgb = p.criterion == "xgb"
        node_best = ninf.clone().scatter_reduce(0, node_i, best, reduce="amax", include_self=True)
        cand = torch.where((best == node_best[node_i]) & torch.isfinite(best), torch.arange(P, device=dev),
                           torch.full((P,), P, device=dev))
        win = torch.full((n,), P, dtype=torch.long, device=dev).scatter_reduce(0, node_i, cand, reduce="amin",
                                                                              include_self=True)
        has = win < P
        if not bool(has.any()):
            return out
        nodes = torch.nonzero(has).flatten()
        wp = win[nodes]
        # the winners' sorted order / prefix sums, from their own bins only
        st = self._pair_stats(hist_of(wp).to(torch.float64), pcat[wp])
        h, order, L, totnn, na, T = st["h"], st["order"], st["L"], st["totnn"], st["na"], st["T"]
        nt = B - 1
        kk = k[wp]
        opt = torch.where(kk < nt, torch.zeros_like(kk), torch.where(kk < 2 * nt, torch.ones_like(kk),
                                                                     torch.full_like(kk, 2)))
        t = torch.where(opt == 0, kk, torch.where(opt == 1, kk - nt, torch.zeros_like(kk)))
        na_left = opt == 1
        ar = torch.arange(wp.numel(), device=dev)
        Lw = torch.where((opt == 2).view(-1, 1), totnn,
                         L[ar, t.clamp(max=nt - 1)] + torch.where(na_left.view(-1, 1), na, torch.zeros_like(na)))
        rank = torch.empty_like(order)
        rank.scatter_(1, order, torch.arange(B, device=dev).view(1, B).expand(order.shape[0], B))
        in_left = rank <= t.view(-1, 1)
        bw = h[:, :B, 1] if xgb else h[:, :B, 0]
        empty = (bw <= 0) & pcat[wp].view(-1, 1)     # empty categorical levels follow the NAs
        in_left = torch.where(empty, na_left.view(-1, 1).expand_as(in_left), in_left)
        in_left = torch.where((opt == 2).view(-1, 1), ~empty | na_left.view(-1, 1), in_left)
        mask = torch.cat([in_left, na_left.view(-1, 1).expand(-1, Bs - B)], 1).to(torch.uint8)
        out["gain"] = out["gain"].index_put((nodes,), best[wp])
        out["feat"] = out["feat"].index_put((nodes,), fglob[wp])
        out["t"] = out["t"].index_put((nodes,), t)
        out["opt"] = out["opt"].index_put((nodes,), opt)
        out["na_left"] = out["na_left"].index_put((nodes,), na_left)
        out["mask"] = out["mask"].index_put((nodes,), mask)
        out["L"] = out["L"].index_put((nodes,), Lw)
        out["R"] = out["R"].index_put((nodes,), T - Lw)
        if "naw" in out:
            out["naw"] = out["naw"].index_put((nodes,), na[:, 0].to(out["naw"].dtype))
        return out

    def _pair_stats(self, h, pcat):
        """Sorted order and prefix sums of pair histograms h [P, Bs, C] f64."""
        B = h.shape[1] - 1
        dev = h.device
        bins, na = h[:, :B], h[:, B]
        if self.p.criterion == "xgb":
            key = torch.where(bins[..., 1] > 0, bins[..., 0] / bins[..., 1].clamp_min(1e-300),
                              torch.full_like(bins[..., 0], float("inf")))
        else:
            key = torch.where(bins[..., 0] > 0, bins[..., 1] / bins[..., 0].clamp_min(1e-300),
                              torch.full_like(bins[..., 0], float("inf")))
        key = torch.where(pcat.view(-1, 1), key, torch.arange(B, device=dev, dtype=key.dtype).view(1, B))
        order = torch.argsort(key, dim=1, stable=True)             # [P, B]
        bs_ = torch.gather(bins, 1, order.unsqueeze(-1).expand(-1, -1, h.shape[2]))
        cum = torch.cumsum(bs_, 1)
        totnn = cum[:, -1]
        L = cum[:, :-1]
        return {"h": h, "na": na, "order": order, "L": L, "totnn": totnn, "R": totnn.unsqueeze(1) - L,
                "T": totnn + na}

    def _pair_gains(self, st, mono, node_wyy, node_i):
        """[P, 2(B-1)+1] gains of every threshold x NA option (torch path)."""
        p = self.p
        xgb = p.criterion == "xgb"
        L, R, totnn, na, T = st["L"], st["R"], st["totnn"], st["na"], st["T"]
        naE = na.unsqueeze(1)
        P = L.shape[0]

        def score(S):
            if xgb:
                g, hh = S[..., 0], S[..., 1]
                if p.reg_alpha > 0:
                    g = torch.sign(g) * torch.clamp(g.abs() - p.reg_alpha, min=0)
                return g * g / (hh + p.reg_lambda)
            w, wy = S[..., 0], S[..., 1]
            return torch.where(w > 0, wy * wy / w.clamp_min(1e-300), torch.zeros_like(w))

        sT = score(T).unsqueeze(1)

        def gain_of(LL, RR):
            g = score(LL) + score(RR) - sT
            if xgb:
                g = 0.5 * g - p.gamma
                ok = (LL[..., 1] >= max(p.min_rows, 1e-12)) & (RR[..., 1] >= max(p.min_rows, 1e-12))
            else:
                wl, wr = LL[..., 0], RR[..., 0]
                ok = (wl >= p.min_rows) & (wr >= p.min_rows) & (wl > 0) & (wr > 0)
                pl = (LL[..., 1] / wl.clamp_min(1e-300))
                pr = (RR[..., 1] / wr.clamp_min(1e-300))
                ok &= pl.to(torch.float32) != pr.to(torch.float32)
            if xgb:
                pl = -LL[..., 0] / (LL[..., 1] + p.reg_lambda)
                pr = -RR[..., 0] / (RR[..., 1] + p.reg_lambda)
            ok &= ~((mono > 0) & (pl > pr)) & ~((mono < 0) & (pl < pr))
            return torch.where(ok, g, torch.full_like(g, NEG_INF))

        gA = gain_of(L, R + naE)
        gB = gain_of(L + naE, R)
        gC = gain_of(totnn.unsqueeze(1), naE)
        has_na = ((na[..., 1] > 0) | (na[..., 0] != 0)) if xgb else (na[..., 0] > 0)
        gB = torch.where(has_na.unsqueeze(1), gB, torch.full_like(gB, NEG_INF))
        gC = torch.where(has_na.unsqueeze(1), gC, torch.full_like(gC, NEG_INF))
        allg = torch.cat([gA, gB, gC], 1)                          # [P, 2(B-1)+1]
        if xgb:
            return torch.where(allg > 0, allg, torch.full_like(allg, NEG_INF))
        wyy = node_wyy.to(torch.float64)[node_i].view(-1, 1) if node_wyy is not None else \
            torch.zeros((P, 1), dtype=torch.float64, device=L.device)
        se_before = (wyy - score(T).unsqueeze(1)).clamp_min(0)
        return torch.where((allg > se_before * p.min_split_improvement) & (se_before > 0), allg,
                           torch.full_like(allg, NEG_INF))

    def _pairs_native(self, H, fslot, node_i, pcat, mono_p, node_wyy, raw=False, pbins=None):
        """(best gain, k) per pair from the HIP pair kernel.  pbins (bins of each
        pair's feature): pairs of narrow (< 256-bin) features are scored by the
        256-wide kernel instance, the rest at the full histogram width."""
        import ctypes
        from ...ops import _native
        p = self.p
        Fl, n, Bs, C = H.shape
        lib = _native.get_lib("tree_split")
        if not getattr(lib, "_typed_pairs", False):
            cv, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
            lib.h2o_cat_pairs.argtypes = [cv, ci, ci, ci, ci, cv, cv, cv, cv, cv, cd, cd, cd, cd, cd, ci, cv, cv]
            lib._typed_pairs = True
        H = H.contiguous()
        P = fslot.numel()
        pf = fslot.to(torch.int32).contiguous()
        pn = node_i.to(torch.int32).contiguous()
        pc = pcat.to(torch.uint8).contiguous()
        pm = mono_p.to(torch.float32).contiguous()
        wyy = node_wyy.to(torch.float64).contiguous() if node_wyy is not None else None
        res = torch.empty((P, 2), dtype=torch.float64, device=H.device)

        def ptr(t):
            return ctypes.c_void_p(0 if t is None else t.data_ptr())
        if pbins is not None and Bs - 1 > 256 and tree_ops.env("H2O3_PAIR_NARROW", "1") == "1":
            if not getattr(lib, "_typed_pairs2", False):
                cv, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
                lib.h2o_cat_pairs2.argtypes = [cv, ci, ci, ci, ci, cv, cv, cv, cv, cv, cd, cd, cd, cd, cd, ci, cv,
                                               cv, ci, cv, cv]
                lib._typed_pairs2 = True
            lists = torch.empty(2 * P + 2, dtype=torch.int32, device=H.device)
            pb = pbins.to(torch.int32).contiguous()
            rc = lib.h2o_cat_pairs2(ptr(H), n, Bs, C, P, ptr(pf), ptr(pn), ptr(pc), ptr(pm), ptr(wyy),
                                    float(p.min_rows), float(p.min_split_improvement), float(p.reg_lambda),
                                    float(p.reg_alpha), float(p.gamma), 1 if p.criterion == "xgb" else 0, ptr(res),
                                    ptr(pb), 255, ptr(lists), tree_ops._stream())
            if rc != 0:
                raise RuntimeError(f"h2o_cat_pairs2 failed: {rc}")
            return res if raw else (res[:, 0].contiguous(), res[:, 1].to(torch.long))
        rc = lib.h2o_cat_pairs(ptr(H), n, Bs, C, P, ptr(pf), ptr(pn), ptr(pc), ptr(pm), ptr(wyy),
                               float(p.min_rows), float(p.min_split_improvement), float(p.reg_lambda),
                               float(p.reg_alpha), float(p.gamma), 1 if p.criterion == "xgb" else 0, ptr(res),
                               tree_ops._stream())
        if rc != 0:
            raise RuntimeError(f"h2o_cat_pairs failed: {rc}")
        if raw:
            return res
        return res[:, 0].contiguous(), res[:, 1].to(torch.long)

    def _find_splits_torch(self, H, col_mask, node_wyy=None, merge=True, sub=None):
        """H: [Fl, n, Bs, C] (local feature slice).  Returns dict of per-node
        tensors on device: gain, feat, na_left, mask[n, Bs], stats L/R [n,C],
        tot [n,C].  sub: local feature indices to score (e.g. the categorical
        ones); large frontiers are scored in node chunks to bound memory."""
        Fl0, n0, Bs0, C0 = H.shape
        if sub is not None:
            sub_t = torch.as_tensor(sub, dtype=torch.long, device=H.device)
            gidx = sub_t + self.f0
            H = H.index_select(0, sub_t)
        else:
            gidx = torch.arange(self.f0, self.f0 + Fl0, device=H.device)
        Fs = H.shape[0]
        # chunk the frontier: ~12 live [nc, Fs, Bs, C] float64 temporaries <= ~3 GB
        nc = max(1, int(3e9 // max(1, 12 * Fs * Bs0 * C0 * 8)))
        if n0 > nc:
            parts = [self._find_splits_torch_core(H[:, i:i + nc], col_mask[i:i + nc], gidx,
                                                  None if node_wyy is None else node_wyy[i:i + nc])
                     for i in range(0, n0, nc)]
            res = {k: (torch.cat([q[k] for q in parts], 0) if parts[0][k] is not None else None) for k in parts[0]}
        else:
            res = self._find_splits_torch_core(H, col_mask, gidx, node_wyy)
        if self.W > 1 and merge:
            res = self._merge_candidates(res, n0, Bs0, C0)
        return res

    def _find_splits_torch_core(self, H, col_mask, gidx, node_wyy=None):
        p = self.p
        Fl, n, Bs, C = H.shape
        B = Bs - 1
        h = H.permute(1, 0, 2, 3).to(torch.float64)       # [n, Fl, Bs, C]
        bins = h[:, :, :B]
        na = h[:, :, B]                                    # [n, Fl, C]
        is_cat = self.is_cat_t[gidx]
        order = None
        uplift = p.criterion.startswith("uplift")
        if bool(is_cat.any()):
            if uplift:
                pt = bins[..., 1] / bins[..., 0].clamp_min(1e-300)
                pc = bins[..., 3] / bins[..., 2].clamp_min(1e-300)
                key = torch.where((bins[..., 0] + bins[..., 2]) > 0, pt - pc,
                                  torch.full_like(bins[..., 0], float("inf")))
            elif p.criterion == "xgb":
                key = torch.where(bins[..., 1] > 0, bins[..., 0] / bins[..., 1].clamp_min(1e-300),
                                  torch.full_like(bins[..., 0], float("inf")))
            else:
                key = torch.where(bins[..., 0] > 0, bins[..., 1] / bins[..., 0].clamp_min(1e-300),
                                  torch.full_like(bins[..., 0], float("inf")))
            ar = torch.arange(B, device=h.device).view(1, 1, B).expand(n, Fl, B)
            key = torch.where(is_cat.view(1, Fl, 1), key, ar.to(key.dtype))
            order = torch.argsort(key, dim=2, stable=True)             # [n, Fl, B]
            bins = torch.gather(bins, 2, order.unsqueeze(-1).expand(-1, -1, -1, C))
        cum = torch.cumsum(bins, 2)
        totnn = cum[:, :, -1]                              # [n, Fl, C] non-NA totals
        L = cum[:, :, :-1]                                 # [n, Fl, B-1, C]
        R = totnn.unsqueeze(2) - L
        T = totnn + na                                     # [n, Fl, C] all rows
        naE = na.unsqueeze(2)
        # option 0: NA right, option 1: NA left, option 2: NA vs rest
        LA, RA = L, R + naE
        LB, RB = L + naE, R
        LC, RC = totnn.unsqueeze(2), naE

        def diverg(S):
            # uplift divergence between treatment and control response rates
            wt, wc = S[..., 0], S[..., 2]
            pt = (S[..., 1] / wt.clamp_min(1e-300)).clamp(1e-6, 1 - 1e-6)
            pc = (S[..., 3] / wc.clamp_min(1e-300)).clamp(1e-6, 1 - 1e-6)
            if p.criterion == "uplift_kl":
                d = pt * torch.log(pt / pc) + (1 - pt) * torch.log((1 - pt) / (1 - pc))
            elif p.criterion == "uplift_chisquared":
                d = (pt - pc) ** 2 / pc + ((1 - pt) - (1 - pc)) ** 2 / (1 - pc)
            else:  # euclidean
                d = (pt - pc) ** 2 + ((1 - pt) - (1 - pc)) ** 2
            return torch.where((wt > 0) & (wc > 0), d, torch.zeros_like(d))

        def score(S):
            if uplift:
                return diverg(S)
            if p.criterion == "xgb":
                g, hh = S[..., 0], S[..., 1]
                if p.reg_alpha > 0:
                    g = torch.sign(g) * torch.clamp(g.abs() - p.reg_alpha, min=0)
                return g * g / (hh + p.reg_lambda)
            w, wy = S[..., 0], S[..., 1]
            return torch.where(w > 0, wy * wy / w.clamp_min(1e-300), torch.zeros_like(w))

        sT = score(T).unsqueeze(2)                         # [n, Fl, 1]

        def gain_of(LL, RR):
            if uplift:
                nl = LL[..., 0] + LL[..., 2]
                nr = RR[..., 0] + RR[..., 2]
                nt = (nl + nr).clamp_min(1e-300)
                g = (nl / nt) * diverg(LL) + (nr / nt) * diverg(RR) - sT
                ok = (nl >= p.min_rows) & (nr >= p.min_rows) & (LL[..., 0] > 0) & (LL[..., 2] > 0) & \
                    (RR[..., 0] > 0) & (RR[..., 2] > 0)
                return torch.where(ok, g, torch.full_like(g, NEG_INF))
            g = score(LL) + score(RR) - sT
            if p.criterion == "xgb":
                g = 0.5 * g - p.gamma
                wl, wr = LL[..., 1], RR[..., 1]
                ok = (wl >= max(p.min_rows, 1e-12)) & (wr >= max(p.min_rows, 1e-12))
                predl = -LL[..., 0] / (wl + p.reg_lambda)
                predr = -RR[..., 0] / (wr + p.reg_lambda)
            else:
                wl, wr = LL[..., 0], RR[..., 0]
                ok = (wl >= p.min_rows) & (wr >= p.min_rows) & (wl > 0) & (wr > 0)
                predl = LL[..., 1] / wl.clamp_min(1e-300)
                predr = RR[..., 1] / wr.clamp_min(1e-300)
                ok &= predl.to(torch.float32) != predr.to(torch.float32)
            mono = self.mono_t[gidx].view(1, Fl, 1)
            ok &= ~((mono > 0) & (predl > predr)) & ~((mono < 0) & (predl < predr))
            return torch.where(ok, g, torch.full_like(g, NEG_INF))

        gA = gain_of(LA, RA)
        gB = gain_of(LB, RB)
        has_na = (na[..., 0] > 0) if p.criterion != "xgb" else ((na[..., 1] > 0) | (na[..., 0] != 0))
        if uplift:
            has_na = (na[..., 0] + na[..., 2]) > 0
        gB = torch.where(has_na.unsqueeze(2), gB, torch.full_like(gB, NEG_INF))
        gC = gain_of(LC, RC)
        gC = torch.where(has_na.unsqueeze(2), gC, torch.full_like(gC, NEG_INF))
        # feature eligibility (column sampling, padding, interaction constraints)
        cm = col_mask.to(h.device)[:, gidx] & (gidx < self.bd.F).view(1, -1)
        allg = torch.cat([gA, gB, gC], 2)                  # [n, Fl, 2(B-1)+1]
        allg = torch.where(cm.unsqueeze(2), allg, torch.full_like(allg, NEG_INF))
        # min split improvement (relative to the node's squared error)
        if uplift:
            allg = torch.where(allg > 1e-12, allg, torch.full_like(allg, NEG_INF))
        elif p.criterion != "xgb":
            wyy_tot = node_wyy.view(-1, 1).to(T.dtype) if node_wyy is not None else torch.zeros_like(T[..., 0])
            se_before = (wyy_tot - score(T)).clamp_min(0).unsqueeze(2)
            allg = torch.where(allg > se_before * p.min_split_improvement, allg, torch.full_like(allg, NEG_INF))
            allg = torch.where(se_before > 0, allg, torch.full_like(allg, NEG_INF))
        else:
            allg = torch.where(allg > 0, allg, torch.full_like(allg, NEG_INF))
        K = allg.shape[2]
        bnd = self._bnd_dev(n)
        if bnd is not None and not uplift and Fl > 0:
            # monotone node bounds on each column's best split (DTree.java:1386-1445)
            bk = allg.argmax(2)                                        # [n, Fl]
            gk = allg.gather(2, bk.unsqueeze(2)).squeeze(2)
            LL_all = torch.cat([LA, LB, LC.expand(-1, -1, 1, -1)], 2)
            RR_all = torch.cat([RA, RB, RC.expand(-1, -1, 1, -1)], 2)
            ix = bk.view(n, Fl, 1, 1).expand(-1, -1, 1, C)
            Lb, Rb = LL_all.gather(2, ix).squeeze(2), RR_all.gather(2, ix).squeeze(2)
            pen, viol = self._bound_cost(Lb, Rb, bnd[:, 0].view(n, 1), bnd[:, 1].view(n, 1))
            gk = torch.where(viol & torch.isfinite(gk),
                             gk - pen if p.use_bounds else torch.full_like(gk, NEG_INF), gk)
            allg = torch.full_like(allg, NEG_INF).scatter_(2, bk.unsqueeze(2), gk.unsqueeze(2))
        flat = allg.reshape(n, Fl * K)
        best, arg = flat.max(1)
        fl = arg // K
        k = arg % K
        nt = B - 1
        opt = torch.where(k < nt, torch.zeros_like(k), torch.where(k < 2 * nt, torch.ones_like(k), torch.full_like(k, 2)))
        t = torch.where(opt == 0, k, torch.where(opt == 1, k - nt, torch.zeros_like(k)))
        na_left = opt == 1
        ar_n = torch.arange(n, device=h.device)
        # stats of the winning split
        Lw = torch.where((opt == 2).view(n, 1), totnn[ar_n, fl],
                         L[ar_n, fl, t.clamp(max=nt - 1)] + torch.where(na_left.view(n, 1), na[ar_n, fl], torch.zeros_like(na[ar_n, fl])))
        Tw = T[ar_n, fl]
        Rw = Tw - Lw
        # go-left masks over codes
        codes = torch.arange(Bs, device=h.device).view(1, Bs)
        cat_best = is_cat[fl]
        mask_num = (codes <= t.view(n, 1)) & (codes < B)
        mask_num = torch.where((opt == 2).view(n, 1), codes < B, mask_num)
        if order is not None:
            ordw = order[ar_n, fl]                                     # [n, B]
            rank = torch.empty_like(ordw)
            rank.scatter_(1, ordw, torch.arange(B, device=h.device).view(1, B).expand(n, B))
            in_left = rank <= t.view(n, 1)
            bins_w = h[ar_n, fl, :B, 0] if p.criterion != "xgb" else h[ar_n, fl, :B, 1]
            if uplift:
                bins_w = h[ar_n, fl, :B, 0] + h[ar_n, fl, :B, 2]
            empty = bins_w <= 0
            in_left = torch.where(empty, na_left.view(n, 1).expand(n, B), in_left)
            in_left = torch.where((opt == 2).view(n, 1), ~empty | na_left.view(n, 1), in_left)
            mask_cat = torch.cat([in_left, torch.zeros((n, Bs - B), dtype=torch.bool, device=h.device)], 1)
            mask = torch.where(cat_best.view(n, 1), mask_cat, mask_num)
        else:
            mask = mask_num
        mask = mask.clone()
        mask[:, Bs - 1] = na_left
        res = {"gain": best, "feat": gidx[fl], "t": t, "opt": opt, "na_left": na_left,
               "mask": mask.to(torch.uint8), "L": Lw, "R": Rw, "tot": T[:, 0] if Fl > 0 else None}
        return res

    def _merge_records(self, pk, mask):
        """Multi-GPU merge of the per-rank packed split records (split_select2
        over each rank's feature slice): two all-gathers (records, go-left
        masks as bytes), the highest gain wins per node, ties to the lowest
        rank (= lowest feature).  Node totals are global on every rank (the
        histograms were reduce-scattered), so the winner's record is complete."""
        W = self.W
        n, Bs = mask.shape
        # ONE all-gather: the record's bytes and the mask bytes side by side
        rb = pk.shape[1] * 8
        buf = torch.cat([pk.contiguous().view(torch.uint8).view(n, rb), mask.contiguous()], 1)
        g = coll.all_gather_dim0(buf).view(W, n, rb + Bs)
        gains = g[:, :, :8].contiguous().view(torch.float64).view(W, n)
        best_r = torch.argmax(gains, 0)
        ar = torch.arange(n, device=pk.device)
        win = g[best_r, ar]
        pk_w = win[:, :rb].contiguous().view(torch.float64).view(n, -1)
        mask_w = win[:, rb:].contiguous()
        return pk_w, mask_w, pk_w[:, 1].to(torch.int32)

    def _merge_candidates(self, res, n, Bs, C):
        W = self.W
        packed = torch.cat([res["gain"].view(n, 1), res["feat"].to(torch.float64).view(n, 1),
                            res["t"].to(torch.float64).view(n, 1), res["opt"].to(torch.float64).view(n, 1),
                            res["L"], res["R"], res["tot"], res["mask"].to(torch.float64)], 1)
        g = coll.all_gather_dim0(packed.contiguous()).view(W, n, -1)
        gains = g[:, :, 0]
        # deterministic tie-break: lowest rank (= lowest feature) wins
        best_r = torch.argmax(gains, 0)
        sel = g[best_r, torch.arange(n, device=g.device)]
        off = 4
        out = {"gain": sel[:, 0], "feat": sel[:, 1].long(), "t": sel[:, 2].long(), "opt": sel[:, 3].long()}
        out["na_left"] = out["opt"] == 1
        out["L"] = sel[:, off:off + C]
        out["R"] = sel[:, off + C:off + 2 * C]
        out["tot"] = g[0, :, off + 2 * C:off + 3 * C]   # rank 0 holds feature 0
        out["mask"] = sel[:, off + 3 * C:].to(torch.uint8)
        return out

    # ------------------------------------------------------------------ grow
    def pos_payload_ok(self):
        """True when grow() keeps the 0/1-weighted mode-0 response as a
        position-ordered NaN-masked payload (quad histogram kernels)."""
        return self.dev.type == "cuda" and not self.use_payload and self.bd.code_bytes == 1 and \
            self.bd.Bs <= 256 and self.bd.Fp % 16 == 0 and tree_ops.env("H2O3_HIST_KERNEL", "quad") == "quad" \
            and tree_ops.env("H2O3_POSV", "1") == "1" and tree_ops.env("H2O3_PART", "ballot") == "ballot"

    def grow(self, va, vb, mode, tree_node_hook=None, want_nid=True, vmax=None, unit_w=None, va_scratch=False):
        """Grow one tree (environment switches read once per tree); see _grow."""
        with tree_ops.env_scope():
            return self._grow(va, vb, mode, tree_node_hook=tree_node_hook, want_nid=want_nid, vmax=vmax,
                              unit_w=unit_w, va_scratch=va_scratch)

    def _grow(self, va, vb, mode, tree_node_hook=None, want_nid=True, vmax=None, unit_w=None, va_scratch=False):
        """Grow one tree.  Returns (Tree, nid[N] leaf index per local row,
        leaf_nodes list (tree node ids, indexed by nid), leaf_tot [n_leaves, C]).
        vmax / unit_w: caller-known bounds (max |channel| for the fixed-point
        histogram scale, 0/1 row weights) that spare the two device syncs at
        the start of the tree."""
        bd, p = self.bd, self.p
        N = bd.nrows_local
        C = tree_ops.channels(mode)
        self._tree_no = getattr(self, "_tree_no", -1) + 1
        self._adaptive = getattr(bd, "hist_type", "auto") in ("uniformadaptive", "random", "roundrobin")
        self._stream_obj = torch.cuda.current_stream() if self.dev.type == "cuda" else None
        if not (self.dev.type == "cuda" and tree_ops.iota_i32(self.ridx)):
            torch.arange(N, dtype=torch.int32, device=self.dev, out=self.ridx)
        if self.dev.type != "cuda":
            self._vmax = None
        else:
            self._vmax = list(vmax) if vmax is not None else tree_ops.channel_max(va, vb, mode)
        # 0/1 row weights (unweighted data, row sampling) -> packed histogram atomics
        self._unit_w = mode == 0 and self.dev.type == "cuda" and (
            vb is None or (bool(unit_w) if unit_w is not None else bool(((vb == 0) | (vb == 1)).all())))
        self._va_eff = None
        quad = self.bd.code_bytes == 1 and self.bd.Bs <= 256 and self.bd.Fp % 16 == 0 and \
            tree_ops.env("H2O3_HIST_KERNEL", "quad") == "quad"
        # every level on the row-direct pair path (DRF's mtries << F): the
        # pair kernels read the position-ordered payload at any histogram width
        all_direct = self._all_levels_direct(mode) and tree_ops.env("H2O3_DRF_POSV", "1") == "1"
        if self._unit_w and not self.use_payload and (quad or all_direct):
            self._va_eff = torch.where(vb > 0, va, torch.full_like(va, float("nan"))) if vb is not None else va
        self._pos1 = None
        self._mask_pend = None
        if self._va_eff is not None and tree_ops.env("H2O3_POSV", "1") == "1" and \
                tree_ops.env("H2O3_PART", "ballot") == "ballot":
            # va_scratch: the caller hands over va (a NaN-masked residual it
            # will not read again) as the root payload -- no copy
            p0 = self._va_eff.clone() if (self._va_eff is va and not va_scratch) else self._va_eff
            self._pos1 = [p0, torch.empty_like(p0)]   # root: position order == row order
        ridx, ridx2 = self.ridx, self.ridx2
        self._la = None
        pa, pb, pa2, pb2 = self._pay
        if self.use_payload:
            pa.copy_(va)
            if vb is not None:
                pb.copy_(vb)
            else:
                pb.fill_(1.0)
            va, vb = pa, pb   # position order == row order while ridx is the identity
        tb = _TreeBuf()
        # frontier as arrays (all nodes of a level share the depth): node ids,
        # row segments [st, st + ct) of ridx, channel totals from the parent's
        # split record (used when the last level builds no histograms)
        f_id = np.zeros(1, dtype=np.int64)
        f_st = np.zeros(1, dtype=np.int64)
        f_ct = np.full(1, N, dtype=np.int64)
        f_tot = None
        depth = 0
        H_prev = None
        wyy_prev, wyy_level = None, None
        # (build slot, derived slot, parent slot) of the node pairs of this level
        p_build = p_der = p_par = None
        leaf_parts = []    # per level: (node ids, starts, counts, totals [k, C])
        level = 0
        async_part = self.dev.type == "cuda" and not p.max_leaves and not self.use_payload and \
            tree_ops.env("H2O3_ASYNC_PART", "1") == "1" and tree_ops.env("H2O3_PART", "ballot") == "ballot"
        is_cat_np = np.asarray(bd.is_cat, dtype=bool)
        # interaction constraints (GlobalInteractionConstraints /
        # BranchInteractionConstraints): the features each frontier node may
        # still split on; the root may use every feature named in a set
        ics = self._interaction_map()
        f_allow = torch.as_tensor(ics[1][None, :].copy(), device=self.dev) if ics is not None else None
        ics_t = torch.as_tensor(ics[0], device=self.dev) if ics is not None else None
        cutmat = self._cut_matrix()
        # monotone node prediction bounds (Constraints._min / _max), per frontier node
        mono_b = p.monotone is not None and bool(np.any(np.asarray(p.monotone) != 0))
        f_lo = np.full(1, -np.inf) if mono_b else None
        f_hi = np.full(1, np.inf) if mono_b else None
        self._bnd, self._bnd_off = None, 0

        coll._TAG.append("tree.L0")
        ntag = len(coll._TAG)
        while f_id.size:
            self._level = level
            coll._TAG[ntag - 1] = f"tree.L{level}"       # collective bytes per level (coll.bytes_report)
            n_front = int(f_id.size)
            can_split = depth < p.max_depth
            C_ = tree_ops.channels(mode)
            level_bytes = self.Fpad * n_front * bd.Bs * C_ * 8
            prev_bytes = 0 if H_prev is None else H_prev.numel() * 8
            chunked = can_split and (level_bytes + prev_bytes) > p.hist_mem_budget and n_front > 1
            self._depth = depth
            # parent records for the per-node adaptive ranges (_adapt_range)
            nxt = self.__dict__.get("_adapt_next")
            self._adapt_par = None if (depth == 0 or nxt is None) else nxt + (n_front,)
            self._rng_par = None if depth == 0 else self.__dict__.get("_rng_cur")
            self._rng_cur = None
            self._adapt_next = None
            direct = can_split and f_allow is None and not self._adaptive and not mono_b and \
                self._direct_level(mode, depth, chunked)
            if mono_b and bool(np.isfinite(f_lo).any() | np.isfinite(f_hi).any()):
                self._bnd = torch.as_tensor(np.stack([f_lo, f_hi], 1), dtype=torch.float64, device=self.dev)
            else:
                self._bnd = None
            self._bnd_off = 0
            chunked = chunked or direct
            la, self._la = self._la, None
            if la is not None and (chunked or not can_split or la[0].shape[1] < n_front):
                la = None   # defensive: the look-ahead only matches a full next level
            if la is not None:
                # this level's histograms were built on the device before the
                # host read the previous level's decisions (_lookahead)
                H = la[0][:, :n_front].contiguous()
                wyy_level = la[1][:n_front] if la[1] is not None else None
                if tree_ops.env("H2O3_LA_CHECK") == "1":
                    self._la_check(la, p_build, p_der, p_par)
            elif chunked:
                # frontier too wide for one level of histograms, or column-sampled
                # levels on the pair path: no parent level kept (no subtraction)
                H, H_prev, wyy_level = None, None, None
            elif not can_split and level > 0:
                # last level: no histograms needed, leaf totals come from the parent split stats
                H = None
            elif level == 0 or H_prev is None:
                H = self._build_hist(ridx, va, vb, mode, f_st, f_ct)
                wyy_level = self._last_wyy
            else:
                Hb = self._build_hist(ridx, va, vb, mode, f_st[p_build], f_ct[p_build])
            if la is not None:
                pass
            elif level > 0 and H_prev is not None and (can_split or level == 0) and self.dev.type == "cuda":
                # copy + parent-minus-built subtraction in one kernel
                clamp = {0: 0b1, 1: 0b0}.get(mode, (1 << tree_ops.channels(mode)) - 1)
                wb = self._last_wyy if mode == 0 else None
                H, wyy_n = tree_ops.hist_sibling(Hb, H_prev, p_build, p_der, p_par, n_front, clamp,
                                                 wyy_b=wb, wyy_prev=wyy_prev if wb is not None else None)
                if wyy_n is not None:
                    wyy_level = wyy_n
                del Hb
            elif level > 0 and H_prev is not None and can_split:
                H = torch.empty((Hb.shape[0], n_front) + tuple(Hb.shape[2:]), dtype=Hb.dtype, device=Hb.device)
                bs = torch.as_tensor(p_build, device=Hb.device)
                ds = torch.as_tensor(p_der, device=Hb.device)
                ps = torch.as_tensor(p_par, device=Hb.device)
                H[:, bs] = Hb
                H[:, ds] = (H_prev[:, ps] - Hb).clamp_min_(0) if mode != 1 else (H_prev[:, ps] - Hb)
                if mode == 0 and self._last_wyy is not None:
                    wyy_level = torch.empty(n_front, dtype=torch.float64, device=Hb.device)
                    wyy_level[bs] = self._last_wyy
                    wyy_level[ds] = wyy_prev[ps] - self._last_wyy
                if mode == 0:
                    # only w / wyy are non-negative; wy may be negative
                    H[:, ds, :, 1] = H_prev[:, ps, :, 1] - Hb[:, :, :, 1]
                del Hb
            nleft_pre = None
            ok_h = None
            naw_h = None
            if can_split:
                sel = self._col_sel(n_front, depth) if direct else None
                cm = None if (direct and self.dev.type == "cuda") else self._col_mask(n_front, depth, sel=sel,
                                                                                      allow=f_allow)
                # node totals of w*y*y (only the total enters the SE split test),
                # fused into the histogram kernel; derived siblings by subtraction
                node_wyy = wyy_level if mode == 0 else None
                with phase("tree.split"):
                    if direct and self.dev.type == "cuda":
                        sp = self._pair_direct_dev(ridx, va, vb, mode, f_st, f_ct, sel)
                    elif direct:
                        sp = self._pair_direct_splits(ridx, va, vb, mode, f_st, f_ct, cm)
                    elif chunked:
                        per = max(1, int(p.hist_mem_budget // max(1, self.Fpad * bd.Bs * C_ * 8)))
                        parts = []
                        need = self._hist_need(cm)
                        for a in range(0, n_front, per):
                            Hc = self._build_hist(ridx, va, vb, mode, f_st[a:a + per], f_ct[a:a + per],
                                                  need_mask=None if need is None else need[a:a + per])
                            wyy_c = self._last_wyy if mode == 0 else None
                            self._bnd_off = a
                            parts.append(self._find_splits(Hc, cm[a:a + per], wyy_c, want_pk=False))
                            del Hc
                        self._bnd_off = 0
                        sp = {k: (torch.cat([q[k] for q in parts], 0) if parts[0].get(k) is not None else None)
                              for k in parts[0]}
                    else:
                        sp = self._find_splits(H, cm, node_wyy, want_pk=async_part)
                nn_ = n_front
                if async_part and "pk" in sp:
                    pkd = sp["pk"]
                    with phase("tree.partition"):
                        # no ridx2 <- ridx copy: every frontier segment is rewritten (non-splitting
                        # nodes in place), earlier leaves are identical in both buffers already
                        pay = (self._pos1[0], None, self._pos1[1], None) if self._pos1 is not None else None
                        tree_ops.partition_async(bd, ridx, ridx2, sp["feat_i32"], sp["mask"], f_st, f_ct,
                                                 payload=pay, pk=pkd, pk_col=11)
                    # the record's copy is queued BEFORE the look-ahead kernels, so
                    # the host gets it while the GPU builds the next level
                    pk_h = self._d2h_async(pkd)
                    self._maybe_lookahead(pkd, (10, 11, 4 + (mode == 1), 6 + (mode == 1)), f_st, f_ct, mode, va,
                                          vb, ridx2, H, wyy_level, depth, level_bytes, chunked)
                    pk = self._d2h_wait(pk_h)
                    self._flush_masks(tb)
                    ok_h = pk[:, 10] > 0
                    nleft_pre = pk[:, 11].astype(np.int64)
                    naw_h = pk[:, 12] if pk.shape[1] > 12 else None
                cols = [] if nleft_pre is not None else [
                    sp["gain"].view(nn_, 1).to(torch.float64), sp["feat"].view(nn_, 1).to(torch.float64),
                    sp["t"].view(nn_, 1).to(torch.float64), sp["opt"].view(nn_, 1).to(torch.float64),
                    sp["L"].to(torch.float64), sp["R"].to(torch.float64), sp["tot"].to(torch.float64)]
                naw_d = sp["naw"].to(torch.float64) if (cols and sp.get("naw") is not None) else None
                if naw_d is None and cols and H is not None and self.W == 1 and mode == 0 and H.shape[1] == nn_:
                    # the winner's NA-bin weight per node (per-node NA direction rule below)
                    fi = sp["feat"].to(torch.int64).clamp(0, H.shape[0] - 1)
                    naw_d = H[fi, torch.arange(nn_, device=H.device), H.shape[2] - 1, 0].to(torch.float64)
                if async_part and nleft_pre is None:
                    # split decision + partition of the whole frontier on the device: no
                    # host round trip between the split search and the row partition
                    tot_d = sp["tot"].to(torch.float64)
                    w_d = (tot_d[:, 0] if mode != 1 else tot_d[:, 1]) + (tot_d[:, 2] if mode == 3 else 0.0)
                    ok_d = torch.isfinite(sp["gain"].to(torch.float64))
                    if p.criterion != "xgb":
                        ok_d &= w_d >= 2 * p.min_rows
                    feat_all = torch.where(ok_d, sp["feat"].to(torch.int64),
                                           torch.zeros_like(sp["feat"].to(torch.int64)))
                    mask_all = torch.where(ok_d.view(-1, 1), sp["mask"].to(torch.uint8),
                                           torch.ones_like(sp["mask"], dtype=torch.uint8))
                    with phase("tree.partition"):
                        pay = (self._pos1[0], None, self._pos1[1], None) if self._pos1 is not None else None
                        nleft_d = tree_ops.partition_async(bd, ridx, ridx2, feat_all, mask_all, f_st, f_ct,
                                                           payload=pay)
                    cols += [ok_d.view(nn_, 1).to(torch.float64), nleft_d.view(nn_, 1).to(torch.float64)]
                # ONE device->host transfer of every per-node scalar of the level
                if cols:
                    if naw_d is not None:
                        cols.append(naw_d.view(nn_, 1))      # last column
                    rec = torch.cat(cols, 1)
                    pk_h = self._d2h_async(rec)
                    if async_part:
                        self._maybe_lookahead(rec, (4 + 3 * C, 5 + 3 * C, 4 + (mode == 1), 4 + C + (mode == 1)),
                                              f_st, f_ct, mode, va, vb, ridx2, H, wyy_level, depth, level_bytes,
                                              chunked)
                    pk = self._d2h_wait(pk_h)
                    self._flush_masks(tb)
                    if async_part:
                        ok_h = pk[:, 4 + 3 * C] > 0
                        nleft_pre = pk[:, 5 + 3 * C].astype(np.int64)
                    naw_h = pk[:, -1] if naw_d is not None else None
                gains = pk[:, 0]
                feats = pk[:, 1].astype(np.int64)
                t_a = pk[:, 2].astype(np.int64)
                opt_a = pk[:, 3].astype(np.int64)
                Ls = pk[:, 4:4 + C]
                Rs = pk[:, 4 + C:4 + 2 * C]
                tots = pk[:, 4 + 2 * C:4 + 3 * C]
            else:
                # totals only
                tots = self._totals(H).numpy() if H is not None else f_tot
                gains = None
            tots = np.asarray(tots, dtype=np.float64)
            w_a = (tots[:, 0] if mode != 1 else tots[:, 1]) + (tots[:, 2] if mode == 3 else 0.0)
            tb.weight[f_id] = w_a
            if ok_h is not None:
                ok = np.asarray(ok_h, dtype=bool).copy()
            elif can_split and gains is not None:
                ok = np.isfinite(gains)
                if p.criterion != "xgb":
                    ok &= w_a >= 2 * p.min_rows
            else:
                ok = np.zeros(n_front, dtype=bool)
            if p.max_leaves:
                # leaf budget, node by node in frontier order (the leaves of this
                # level counted as they are decided); lossguide spends it on the
                # largest loss reductions first (XGBoost's best-first expansion
                # order among the nodes of a level)
                n_leaves = sum(part[0].size for part in leaf_parts)
                n_split = 0
                order = range(n_front)
                if p.leaf_budget_by_gain and gains is not None:
                    order = np.argsort(-np.where(ok, gains, -np.inf), kind="stable")
                for i in order:
                    if ok[i] and (n_leaves + n_front + n_split + 1) > p.max_leaves:
                        ok[i] = False
                    if ok[i]:
                        n_split += 1
                    else:
                        n_leaves += 1
            lf = ~ok
            if lf.any():
                leaf_parts.append((f_id[lf], f_st[lf], f_ct[lf], tots[lf]))
            sids = np.nonzero(ok)[0]
            if sids.size == 0:
                if nleft_pre is not None:
                    ridx, ridx2 = ridx2, ridx   # the (identity) partition already ran
                    if self._pos1 is not None:
                        self._pos1.reverse()
                break
            # record the splits in the tree (vectorized over the level)
            k = int(sids.size)
            nid_s = f_id[sids]
            f_s = feats[sids]
            opt_s = opt_a[sids]
            t_s = t_a[sids]
            Lsel, Rsel = Ls[sids], Rs[sids]
            wl_a = (Lsel[:, 0] if mode != 1 else Lsel[:, 1]) + (Lsel[:, 2] if mode == 3 else 0.0)
            wr_a = (Rsel[:, 0] if mode != 1 else Rsel[:, 1]) + (Rsel[:, 2] if mode == 3 else 0.0)
            build_left = wl_a <= wr_a
            first = tb.add_children(depth + 1, Lsel[:, 0], Rsel[:, 0])
            lid = first + 2 * np.arange(k, dtype=np.int64)
            tb.feat[nid_s] = f_s
            tb.gain[nid_s] = gains[sids]
            na_s = opt_s == 1
            hn = getattr(self.bd, "has_na", None)
            if p.criterion != "xgb" and (naw_h is not None or (hn is not None and len(hn) == self.bd.F)):
                # no NA weight reached THIS node on the split column: NAs of later
                # data go to the heavier child (DTree.java:1475-1478 decides per
                # node, nasplit == None); without the node's NA weight (chunked /
                # pair / multi-rank torch paths) the training-wide flag stands in
                no_na = (np.asarray(naw_h)[sids] == 0) if naw_h is not None else ~np.asarray(hn, dtype=bool)[f_s]
                free = no_na & (opt_s != 2) & ~is_cat_np[f_s]
                na_s = np.where(free, wl_a > wr_a, na_s)
            tb.na_left[nid_s] = na_s
            if self._adaptive:
                self._adapt_next = (sids.copy(), np.asarray(f_s).copy(), np.asarray(t_s).copy(),
                                    np.asarray(opt_s).copy())
            tb.left[nid_s] = lid
            tb.right[nid_s] = lid + 1
            cat_s = is_cat_np[f_s]
            num = ~cat_s
            if num.any():
                tb.thr[nid_s[num]] = np.where(opt_s[num] == 2, np.inf, cutmat[f_s[num], np.minimum(t_s[num],
                                                                                                   cutmat.shape[1] - 1)])
                tb.split_code[nid_s[num]] = t_s[num]
            all_split = k == n_front
            masks = None
            if cat_s.any() or nleft_pre is None:
                masks = sp["mask"] if all_split else sp["mask"][tree_ops._h2d(sids, sp["mask"].device)]
            if cat_s.any():
                # only the categorical splits' mask rows cross to the host (one gather + copy)
                cj = np.nonzero(cat_s)[0]
                mk = masks[tree_ops._h2d(cj, masks.device)] if cj.size < k else masks
                masks_h = None
                if mk.is_cuda and tree_ops.env("H2O3_ASYNC_MASKS", "1") == "1":
                    # asynchronous copy into a pinned staging buffer: the rows are
                    # collected after the next level's record arrives (the GPU has
                    # long finished the copy by then) instead of a blocking .cpu()
                    self._flush_masks(tb)
                    need = mk.numel()
                    st_buf = self.__dict__.get("_mask_stage")
                    if st_buf is None or st_buf.numel() < need:
                        st_buf = self._mask_stage = torch.empty(max(need, 1 << 20), dtype=torch.uint8,
                                                                pin_memory=True)
                    st_buf[:need].view(mk.shape).copy_(mk, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
                else:
                    masks_h = mk.cpu().numpy()
                tb.is_cat[nid_s[cj]] = True
                tb.thr[nid_s[cj]] = np.nan
                fcj = f_s[cj]
                for f in np.unique(fcj).tolist():
                    if f not in tb.cat_lvm:
                        # level -> code of the mask row (grouped high-cardinality levels share a code)
                        card = bd.cat_card[f]
                        tb.cat_lvm[f] = np.arange(card) if (bd.cat_group[f] == 1 and card <= bd.Bs - 1) else \
                            np.minimum(np.arange(card) // bd.cat_group[f], bd.Bs - 2)
                if masks_h is not None:
                    tb.cat_parts.append((nid_s[cj].astype(np.int64), fcj.astype(np.int64), masks_h))
                else:
                    self._mask_pend = (nid_s[cj].astype(np.int64), fcj.astype(np.int64), tuple(mk.shape), ev)
            st_s, ct_s = f_st[sids], f_ct[sids]
            # partition
            if nleft_pre is not None:
                nleft = nleft_pre[sids]
                if self._pos1 is not None:
                    self._pos1.reverse()
            else:
                with phase("tree.partition"):
                    ridx2.copy_(ridx)
                    if self.use_payload:
                        pa2.copy_(pa)
                        pb2.copy_(pb)
                    pay = (pa, pb, pa2, pb2) if self.use_payload else None
                    if self._pos1 is not None:
                        pay = (self._pos1[0], None, self._pos1[1], None)
                    nleft = np.asarray(tree_ops.partition(bd, ridx, ridx2, f_s, masks, st_s, ct_s, payload=pay),
                                       dtype=np.int64)
                    if self._pos1 is not None:
                        self._pos1.reverse()
            ridx, ridx2 = ridx2, ridx
            if self.use_payload:
                pa, pa2, pb, pb2 = pa2, pa, pb2, pb
                va, vb = pa, pb
            # next frontier: (left, right) of every split node, in order
            f_id = np.stack([lid, lid + 1], 1).reshape(-1)
            f_st = np.stack([st_s, st_s + nleft], 1).reshape(-1)
            f_ct = np.stack([nleft, ct_s - nleft], 1).reshape(-1)
            f_tot = np.stack([Lsel, Rsel], 1).reshape(2 * k, -1)
            if f_allow is not None:
                # nextLevelInteractionConstraints: branch set ∩ the split feature's set
                ca = f_allow[tree_ops._h2d(sids, self.dev)] & ics_t[tree_ops._h2d(f_s, self.dev)]
                f_allow = torch.repeat_interleave(ca, 2, dim=0)
            if mono_b:
                f_lo, f_hi = self._child_bounds(f_lo[sids], f_hi[sids], f_s, cat_s, np.asarray(Lsel, dtype=np.float64),
                                                np.asarray(Rsel, dtype=np.float64), mode)
            jj = 2 * np.arange(k, dtype=np.int64)
            p_build = jj + (~build_left)
            p_der = jj + build_left
            # parent hists for the next level (only split nodes)
            if H is None:
                H_prev, wyy_prev = None, None   # chunked level: next level builds from rows
                p_par = np.arange(k, dtype=np.int64)
            elif self.dev.type == "cuda":
                # the sibling kernel indexes the parent level directly: keep the
                # whole level and point the pairs at their parents' slots
                H_prev = H
                wyy_prev = wyy_level if mode == 0 else None
                p_par = sids.astype(np.int64)
            else:
                sid = torch.as_tensor(sids, device=H.device)
                H_prev = H[:, sid]
                wyy_prev = wyy_level[sid] if (mode == 0 and wyy_level is not None) else None
                p_par = np.arange(k, dtype=np.int64)
            depth += 1
            level += 1
        del coll._TAG[ntag - 1:]
        self._flush_masks(tb)
        tree = tb.to_tree()
        if leaf_parts:
            leaf_ids = np.concatenate([q[0] for q in leaf_parts])
            leaf_st = np.concatenate([q[1] for q in leaf_parts])
            leaf_ct = np.concatenate([q[2] for q in leaf_parts])
            leaf_tot_np = np.concatenate([q[3] for q in leaf_parts], 0)
        else:
            leaf_ids = leaf_st = leaf_ct = np.zeros(0, dtype=np.int64)
            leaf_tot_np = np.zeros((0, C))
        leaves = leaf_ids.tolist()
        lids = list(range(len(leaves)))
        nid = None
        if want_nid:
            with phase("tree.nid"):
                nid = tree_ops.fill_nid(ridx, np.arange(len(leaves), dtype=np.int64), leaf_st, leaf_ct, N)
        self.ridx, self.ridx2 = ridx, ridx2
        self._pay = [pa, pb, pa2, pb2]
        self.last_segs = (lids, leaf_st.tolist(), leaf_ct.tolist())
        leaf_tot_t = torch.from_numpy(np.ascontiguousarray(leaf_tot_np, dtype=np.float64))
        return tree, nid, leaves, leaf_tot_t

    def _d2h_async(self, t):
        """Queue a device->host copy of t into a reusable pinned slot; returns
        (host view, event).  CPU tensors pass through."""
        if t.device.type != "cuda":
            return (t, None, 0)
        ring = self.__dict__.setdefault("_d2h_ring", [None, None])
        k = self.__dict__.get("_d2h_k", 0)
        self._d2h_k = k ^ 1
        buf = ring[k]
        if buf is None or buf.numel() < t.numel():
            buf = ring[k] = torch.empty(max(t.numel(), 4096), dtype=t.dtype, pin_memory=True)
        h = buf[:t.numel()].view(t.shape)
        h.copy_(t, non_blocking=True)
        # one reusable event per slot, recorded on the stream cached by grow()
        evs = self.__dict__.setdefault("_d2h_ev", [None, None])
        if evs[k] is None:
            evs[k] = torch.cuda.Event()
        st = getattr(self, "_stream_obj", None)
        evs[k].record(st if st is not None else torch.cuda.current_stream())
        # uploads staged after this record (the look-ahead) are NOT covered
        return (h, evs[k], tree_ops.upload_mark())

    @staticmethod
    def _d2h_wait(hev):
        h, ev = hev[0], hev[1]
        if ev is not None:
            ev.synchronize()
            tree_ops.host_synced(hev[2])   # every upload queued before the record has completed
        return h.numpy().copy()

    def _maybe_lookahead(self, rec, cols, f_st, f_ct, mode, va, vb, ridx_next, H, wyy_level, depth, level_bytes,
                         chunked):
        """Launch the NEXT level's histograms now (device-built work list,
        tree_ops.hist_build_dev + hist_sibling_dev), before the host syncs on
        this level's split record: the host bookkeeping of this level then runs
        while the GPU builds the next level's histograms.  Only for a full next
        level (every node may split) that fits the histogram budget; else the
        next level is built after the sync as before."""
        self._la = None
        p = self.p
        if tree_ops.env("H2O3_LOOKAHEAD", "1") != "1" or self.dev.type != "cuda" or chunked or H is None or \
                depth + 1 >= p.max_depth or mode not in (0, 1) or p.max_leaves:
            return
        if 2 * level_bytes + H.numel() * 8 > p.hist_mem_budget:
            return
        posv = False
        va_n, vb_n = va, vb
        if mode == 0 and getattr(self, "_pos1", None) is not None:
            va_n, vb_n, posv = self._pos1[1], None, True     # the payload the partition just moved
        elif mode == 0 and getattr(self, "_va_eff", None) is not None:
            va_n, vb_n = self._va_eff, None
        with phase("tree.hist"), phase("tree.hist.lookahead"):
            r = tree_ops.hist_build_dev(self.bd, ridx_next, va_n, vb_n, mode, rec, cols, f_st, f_ct, self._vmax,
                                        posv=posv, unit_w=getattr(self, "_unit_w", False))
            if r is None:
                return
            Hb, wyy_b, slots, cnts = r
            if self.W > 1:
                Hb, wyy_b = self._rs_hist_wyy(Hb, wyy_b)
            clamp = {0: 0b1, 1: 0b0}.get(mode, (1 << tree_ops.channels(mode)) - 1)
            Hn, wyy_n = tree_ops.hist_sibling_dev(Hb, H, slots, cnts, clamp, wyy_b=wyy_b if mode == 0 else None,
                                                  wyy_prev=wyy_level if mode == 0 else None)
        self._la = (Hn, wyy_n, slots, cnts)

    def _la_check(self, la, p_build, p_der, p_par):
        """Debug (H2O3_LA_CHECK=1): the device-built pair slots equal the host's."""
        slots, cnts = la[2].cpu().numpy(), la[3].cpu().numpy()
        nb = len(p_build)
        assert int(cnts[0]) == nb, (int(cnts[0]), nb)
        nl = len(slots) // 3
        assert np.array_equal(slots[:nb], p_build) and np.array_equal(slots[nl:nl + nb], p_der) and \
            np.array_equal(slots[2 * nl:2 * nl + nb], p_par)

    def _cut_matrix(self):
        """[F, max_cuts + 1] numeric split values by (feature, threshold code):
        cuts[f][t], +inf past the last cut (BinnedData.split_value)."""
        cm = getattr(self, "_cutmat", None)
        if cm is None:
            bd = self.bd
            w = 1 + max([len(c) for c in bd.cuts if c is not None] or [0])
            cm = np.full((bd.F, w), np.inf)
            for f, c in enumerate(bd.cuts):
                if c is not None and len(c):
                    cm[f, :len(c)] = c
            self._cutmat = cm
        return cm

    def _totals(self, H):
        """Per-node channel totals [n, C] (global), from feature 0."""
        Fl, n, Bs, C = H.shape
        t = H[0].to(torch.float64).sum(1) if Fl > 0 else torch.zeros((n, C), dtype=torch.float64, device=H.device)
        if self.W > 1:
            t = coll.all_gather_dim0(t.contiguous()).view(self.W, n, C)[0]
        return t.cpu()
