"""Device-resident GBM tree: the whole level loop of one tree as a fixed
kernel sequence, captured once as a hipGraph and replayed per tree.

Reference: hex/tree/SharedTree.java:481-516 (scoreAndBuildTrees -> one
buildLayer per level), hex/tree/gbm/GBM.java:464 (buildNextKTrees) and the
GammaPass leaf values (GBM.java:1286).

The level loop of `engine.TreeGrower` reads every level's split decisions on
the host (one device->host round trip per level) and sizes its launches from
them.  Here nothing crosses to the host inside a tree:

* the frontier of level d is a heap of 2^d slots; slot i's children are slots
  2i and 2i+1 of level d+1 and absent nodes carry a zero row count;
* one f64 record row per heap node (ops/csrc/tree_hist.hip, DT_RS fields:
  split record of split_select2, left count, row segment, leaf value) is the
  only tree state; every work list (lighter-child histogram chunks, partition
  chunks, leaf chunks) is built from it on the device (dt_items_kernel) and
  every launch grid is a fixed capacity with early-exiting workgroups;
* so the sequence -- residual, root histogram, per level (child histograms by
  subtraction, split search, ballot partition, next-level segments), leaf
  gamma sums, leaf values, per-row leaf-value scatter -- is static: one
  hipGraph replay per tree on one rank, stream-ordered RCCL collectives
  (histogram reduce-scatter, split-record all-gather, leaf-sum all-reduce)
  between the same kernels on several ranks;
* the tree comes back as ONE [2^(D+1) - 1, 16] f64 record copied
  asynchronously to pinned memory and decoded on the host when the forest is
  next read.

Row sampling (sample_rate, sample_rate_per_class) enters as the residual
pass's 0/1 weight buffer (NaN residual = out-of-sample row, as in the level
loop); per-node column sampling (col_sample_rate, its change per level) as
a device kernel that builds each level's eligibility mask from the parent
records with the level loop's per-node samples (dt_colmask_kernel), seeds
drawn per tree from the grower's generator exactly as the level loop draws
them.

Scope (everything else takes the level loop of engine.py): bernoulli /
gaussian GBM, K = 1, 0/1 row weights, numeric features with one-byte codes
on the bin-major histogram kernel, no monotone or interaction constraints,
no adaptive histogram types, max_depth <= 11.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from ...ops import tree_ops
from ...ops.tree_ops import _ptr, _stream
from ...parallel import cloud
from ...parallel import collectives as coll
from ...utils import graphs
from .engine import _TreeBuf

RS = 16
(GAIN, FEAT, T, OPT, L0, L1, R0, R1, T0, T1, OK, NL, NAW, ST, CT, VAL) = range(16)
MAX_DEPTH = 11
_cv, _ci, _cll, _cd, _cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_double, ctypes.c_float


def _libs():
    from ...ops import _native
    lh = tree_ops._lib()
    ls = _native.get_lib("tree_split")
    if not getattr(lh, "_typed_dt", False):
        lh.h2o_dt_items.argtypes = [_ci, _cv, _ci, _ci, _ci, _ci, _ci, _cv, _cv, _cv, _cv]
        lh.h2o_dt_offsets.argtypes = [_cv, _cv, _cv, _cv, _ci, _cv, _cv, _cv, _cv]
        lh.h2o_dt_sibling.argtypes = [_cv, _cv, _cv, _ci, _ci, _ci, _ci, _ci, _ci, _cv, _cv, _cv, _cv, _cv]
        lh.h2o_dt_leaf_vals.argtypes = [_cv, _cv, _ci, _ci, _cv, _cd, _cv, _cv]
        lh.h2o_dt_root.argtypes = [_cv, _cll, _cv]
        lh.h2o_part_flags_dev.argtypes = [_cv, _ci, _cll, _cll, _cv, _cv, _cv, _ci, _cv, _cv, _ci, _cv, _cv, _cv, _cv]
        lh.h2o_part_compact_dev.argtypes = [_cv, _cv, _cv, _ci, _cv, _cv, _cv, _cv, _cv, _cv, _cv, _cv]
        lh.h2o_leaf_pos_dev.argtypes = [_cv, _cv, _ci, _ci, _cv, _cv, _cv]
        lh.h2o_leaf_scatter_dev.argtypes = [_cv, _cv, _ci, _cv, _cv, _cv, _cv]
        lh.h2o_hist_bm.argtypes = [_cv, _ci, _cv, _cv, _cv, _cv, _ci, _ci, _ci, _ci, _cf, _cf, _cv, _ci, _ci, _cv,
                                   _ci, _cll, _ci, _cv, _cv, _cv, _cv]
        lh.h2o_gbm_grad.argtypes = [_cv, _cv, _cv, _ci, _cll, _cv, _cv, _cv]
        lh.h2o_iota_i32.argtypes = [_cv, _cll, _cv]
        lh.h2o_dt_colmask.argtypes = [_ci, _cv, _cv, _cv, _cv, _cv, _ci, _ci, _cv, _cv]
        lh._typed_dt = True
    if not getattr(ls, "_typed_dt", False):
        ls.h2o_split_find_b.argtypes = [_cv, _ci, _ci, _ci, _cv, _cv, _cv] + [_cd] * 5 + [_ci, _cv, _cv, _ci, _cv]
        ls.h2o_split_select2.argtypes = [_cv, _cv, _ci, _ci, _ci, _ci, _cd, _ci, _cv, _cv, _cv, _cv]
        ls._typed_dt = True
    return lh, ls


def _ck(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: error {rc}")


def supported(drv) -> str | None:
    """None when the GBM driver's configuration runs on the device-resident
    tree, else the reason it does not (the engine's level loop then runs)."""
    if os.environ.get("H2O3_DEV_TREE", "1") != "1":
        return "disabled (H2O3_DEV_TREE=0)"
    bd, gp, p = drv.bd, drv.gp, drv.est._parms
    if drv.dev.type != "cuda":
        return "no GPU"
    if drv.K != 1 or drv.dist.family not in ("bernoulli", "gaussian") or drv.dist.link not in ("logit", "identity"):
        return "distribution"
    if drv.mono_on or drv.noise_bw != 0 or gp.interaction_sets:
        return "constraints / prediction noise"
    if not drv._base_unit:
        return "row weights other than 0/1"
    if any(bd.is_cat) or bd.code_bytes != 1 or bd.Bs > 256 or bd.Bs % 4 or bd.Fp % 16:
        return "categorical features / wide codes"
    if getattr(bd, "hist_type", "auto") in ("uniformadaptive", "random", "roundrobin"):
        return "adaptive histogram type"
    if gp.max_depth > MAX_DEPTH or gp.max_depth < 1:
        return "max_depth"
    if (gp.mtries or -1) > 0:
        return "mtries"
    if gp.max_leaves:
        return "max_leaves"
    if tree_ops.bm_groups(bd.F, bd.Fp, bd.Bs, True) is None:
        return "histogram layout"
    if drv.offset is not None or getattr(drv.dist, "huber_delta", None) is not None:
        return "offset"
    if not drv.grower.pos_payload_ok():
        return "payload path"
    return None


class DevTreeGBM:
    """Static buffers + the per-tree kernel sequence of one GBM driver."""

    def __init__(self, drv):
        self.drv = drv
        bd, gp = drv.bd, drv.gp
        self.bd, self.gp = bd, gp
        self.lh, self.ls = _libs()
        g = drv.grower
        self.W, self.rank = g.W, g.rank
        self.F, self.Fl, self.Fpad, self.f0 = bd.F, g.Fl, g.Fpad, g.f0
        self.N = N = bd.nrows_local
        self.D = D = int(gp.max_depth)
        self.nh = (1 << (D + 1)) - 1
        self.Bs = Bs = bd.Bs
        self.C = C = 2
        self.bern = drv.dist.family == "bernoulli"
        self.maxabs = float(drv.est._parms.get("max_abs_leafnode_pred", 1.79e308))
        dev = drv.dev
        self.dev = dev
        # histogram layout and fixed-point scales (static: the chunk sizes follow
        # from N exactly as the level loop's do for a full frontier)
        self.pack = tree_ops.env("H2O3_HIST_PACK", "1") == "1"
        n_fg, G = tree_ops.bm_groups(bd.F, bd.Fp, Bs, self.pack)
        self.n_fg, self.G = n_fg, G
        self.chunk_r = tree_ops.hist_chunk(N, n_fg)
        self.chunk_c = tree_ops.hist_chunk((N + 1) // 2, n_fg)
        if self.pack and max(self.chunk_r, self.chunk_c) >= (1 << 23):
            raise RuntimeError("devtree: histogram chunk too large for the packed path")
        self.chunk_p = tree_ops._part_chunk(N)
        self.chunk_l = 65536
        # bernoulli residuals with 0/1 weights lie in (-1, 1): static bound;
        # gaussian: the bound is refreshed per tree (one host read per tree)
        self.vmax = [1.0, 1.0]
        self._scales()
        # capacities of the device-built work lists
        n_lvl_max = 1 << (D - 1) if D >= 1 else 1
        self.cap_r = 1 + N // self.chunk_r + 1
        self.cap_c = n_lvl_max + ((N + 1) // 2) // self.chunk_c + 2
        self.cap_p = (1 << D) + N // self.chunk_p + 1
        self.cap_l = self.nh + N // self.chunk_l + 1
        cap_h = max(self.cap_r, self.cap_c)
        i32, f64 = torch.int32, torch.float64
        self.rec = torch.zeros(self.nh * RS, dtype=f64, device=dev)
        self.sums = torch.zeros(self.nh * 2, dtype=f64, device=dev)
        self.vals = torch.zeros(self.nh, dtype=torch.float32, device=dev)
        self.lr_t = torch.zeros(1, dtype=torch.float32, device=dev)
        self.ridx = [g.ridx, g.ridx2]
        self.pos = [torch.empty(N, dtype=torch.float32, device=dev) for _ in range(2)]
        self.dbuf = torch.zeros(N, dtype=torch.float32, device=dev)
        lvl = self.Fl * n_lvl_max * Bs * C
        self.Hbuf = [torch.zeros(lvl, dtype=f64, device=dev) for _ in range(2)]
        self.wyybuf = [torch.zeros(n_lvl_max, dtype=f64, device=dev) for _ in range(2)]
        npar_max = max(1, n_lvl_max // 2)
        # local (all-feature) histogram of the built children, + per-pair w*y*y
        self.Hb = torch.zeros(bd.F * npar_max * Bs * C + npar_max, dtype=f64, device=dev)
        self.Hroot = torch.zeros(bd.F * Bs * C + 1, dtype=f64, device=dev)
        self.hwork = torch.zeros(cap_h * 4, dtype=i32, device=dev)
        self.pwork = torch.zeros(self.cap_p * 4, dtype=i32, device=dev)
        self.fbase = torch.zeros(self.cap_p, dtype=i32, device=dev)
        self.lwork = torch.zeros(self.cap_l * 4, dtype=i32, device=dev)
        self.counts = torch.zeros(2, dtype=i32, device=dev)
        self.cnt = torch.zeros(self.cap_p, dtype=i32, device=dev)
        self.loff = torch.zeros(self.cap_p, dtype=i32, device=dev)
        self.roff = torch.zeros(self.cap_p, dtype=i32, device=dev)
        self.flags = torch.zeros(N // 64 + self.cap_p + 1, dtype=torch.int64, device=dev)
        self.part = tree_ops.bm_part(cap_h, n_fg, Bs, G, self.pack, dev)
        self.split_out = torch.zeros(n_lvl_max * max(self.Fl, 1) * 4, dtype=f64, device=dev)
        self.mask = torch.zeros(n_lvl_max * Bs, dtype=torch.uint8, device=dev)
        self.feat_i = torch.zeros(n_lvl_max, dtype=i32, device=dev)
        self.okm = torch.ones((n_lvl_max, max(self.Fl, 1)), dtype=torch.uint8, device=dev)
        if self.f0 + self.Fl > self.F:
            self.okm[:, max(0, self.F - self.f0):] = 0
        self._okm_col = None
        self.mono = torch.zeros(max(self.Fl, 1), dtype=torch.float32, device=dev)
        if bd.codes_col is not None:
            self.pcodes, self.prs, self.pfs = bd.codes_col, 1, bd.nrows_local
        else:
            self.pcodes, self.prs, self.pfs = bd.codes, bd.Fp, 1
        self.cutmat = g._cut_matrix()
        # row sampling: the residual pass reads a static 0/1 weight buffer
        self.sampled = not drv._unit_weights
        self.wbuf = torch.ones(N, dtype=torch.float32, device=dev) if self.sampled else None
        # per-node column sampling: per-tree eligible ids / count and per-level
        # (k, seed) in device buffers read by dt_colmask_kernel
        self.colsamp = gp.col_sample_rate < 1.0 or gp.col_sample_rate_change_per_level != 1.0
        if self.colsamp:
            self.cs_elig = torch.zeros(max(self.F, 1), dtype=torch.int64, device=dev)
            self.cs_m = torch.zeros(1, dtype=torch.int32, device=dev)
            self.cs_k = torch.zeros(max(D, 1), dtype=torch.int32, device=dev)
            self.cs_seed = torch.zeros(max(D, 1), dtype=torch.int64, device=dev)
        self.graph = None
        self._hv = [None, None]
        self._k = 0

    # ---------------------------------------------------------------- scales
    def _scales(self):
        vm = self.vmax
        self.s_r = [tree_ops.fixed_point_scale(m, self.chunk_r) for m in vm]
        self.s_c = [tree_ops.fixed_point_scale(m, self.chunk_c) for m in vm]
        self.bq_r = self.bq_c = -1
        if self.pack:
            self.s_r[1], self.bq_r = tree_ops._pack_scale(vm[1], self.chunk_r)
            self.s_c[1], self.bq_c = tree_ops._pack_scale(vm[1], self.chunk_c)

    def set_tree_cols(self, mask):
        """Per-tree column sample (col_sample_rate_per_tree): the split kernels'
        [n, Fl] eligibility mask, rewritten outside the captured graph."""
        key = None if mask is None else mask.tobytes()
        if key == self._okm_col:
            return
        self._okm_col = key
        m = np.ones(self.Fpad, dtype=np.uint8)
        if mask is not None:
            m[:self.F] = np.asarray(mask, dtype=np.uint8)
        m[self.F:] = 0
        row = self._upload([m[self.f0:self.f0 + self.Fl].copy()])[0]
        self.okm.copy_(row.view(1, -1).expand_as(self.okm))

    def _upload(self, arrays):
        """Per-tree host inputs to the device without a host/GPU sync: packed
        into a pinned staging slot (two slots, each reused only after its
        previous copy completed), ONE non-blocking copy into a device staging
        buffer, returned as device views (8-byte aligned) for stream-ordered
        device copies.  A pageable torch.as_tensor here waited for the GPU
        every tree (1.8 ms per tree in an AutoML GBM step)."""
        offs, n = [], 0
        for a in arrays:
            offs.append(n)
            n += (a.nbytes + 7) & ~7
        n = max(n, 8)
        if getattr(self, "_stg", None) is None or self._stg[0].numel() < n:
            self._stg = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
            self._stg_ev = [None, None]
            self._dstg = torch.empty(n, dtype=torch.uint8, device=self.dev)
            self._stg_i = 0
        i = self._stg_i
        self._stg_i ^= 1
        if self._stg_ev[i] is not None:
            self._stg_ev[i].synchronize()
        buf = self._stg[i].numpy()
        for a, o in zip(arrays, offs):
            buf[o:o + a.nbytes] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        # the device staging buffer is consumed by the copies below in stream
        # order before the next upload overwrites it
        self._dstg[:n].copy_(self._stg[i][:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._stg_ev[i] = ev
        out = []
        for a, o in zip(arrays, offs):
            out.append(self._dstg[o:o + a.nbytes].view(torch.from_numpy(a[:0]).dtype)
                       if a.nbytes else torch.empty(0, dtype=torch.from_numpy(a[:0]).dtype, device=self.dev))
        return out

    # ---------------------------------------------------------------- sequence
    def _rec_lvl(self, d):
        off = (1 << d) - 1
        return self.rec[off * RS:]

    def _hist(self, d, cur):
        """Level d's histogram [Fl, 2^d, Bs, C] (+ w*y*y [2^d]) into buffer d % 2."""
        lh = self.lh
        bd, Bs, C = self.bd, self.Bs, self.C
        n = 1 << d
        H = self.Hbuf[d % 2][:self.Fl * n * Bs * C]
        wyy = self.wyybuf[d % 2][:n]
        s = _stream()
        if d == 0:
            _ck(lh.h2o_dt_items(0, _ptr(self.rec), 1, self.D, 0, self.chunk_r, self.cap_r, _ptr(self.hwork), None,
                                _ptr(self.counts), s), "dt_items(root)")
            nh = bd.F * Bs * C
            buf = self.Hroot
            buf.zero_()
            _ck(lh.h2o_hist_bm(_ptr(bd.codes), bd.Fp, _ptr(self.ridx[cur]), _ptr(self.pos[cur]), None,
                               _ptr(self.hwork), self.cap_r, bd.F, 0, Bs, self.s_r[0], self.s_r[1], _ptr(buf), 1, 0,
                               _ptr(buf[nh:]), 1, self.bq_r, self.G, None, _ptr(self.counts), _ptr(self.part), s),
                "hist_bm(root)")
            Hl, wl = buf[:nh].view(bd.F, 1, Bs, C), buf[nh:]
            if self.W > 1:
                Hl, wl = self.drv.grower._rs_hist_wyy(Hl, wl)
            H.view(self.Fl, 1, Bs, C).copy_(Hl)
            wyy.copy_(wl)
            return H, wyy
        npar = n // 2
        rp = self._rec_lvl(d - 1)
        _ck(lh.h2o_dt_items(1, _ptr(rp), npar, self.D, 0, self.chunk_c, self.cap_c, _ptr(self.hwork), None,
                            _ptr(self.counts), s), "dt_items(child)")
        nhb = bd.F * npar * Bs * C
        buf = self.Hb[:nhb + npar]
        buf.zero_()
        _ck(lh.h2o_hist_bm(_ptr(bd.codes), bd.Fp, _ptr(self.ridx[cur]), _ptr(self.pos[cur]), None, _ptr(self.hwork),
                           self.cap_c, bd.F, 0, Bs, self.s_c[0], self.s_c[1], _ptr(buf), npar, 0, _ptr(buf[nhb:]), 1,
                           self.bq_c, self.G, None, _ptr(self.counts), _ptr(self.part), s), "hist_bm(child)")
        Hb, wb = buf[:nhb].view(bd.F, npar, Bs, C), buf[nhb:]
        if self.W > 1:
            Hb, wb = self.drv.grower._rs_hist_wyy(Hb, wb)
            Hb, wb = Hb.contiguous(), wb.contiguous()
        Hp = self.Hbuf[(d - 1) % 2]
        wp = self.wyybuf[(d - 1) % 2]
        _ck(lh.h2o_dt_sibling(_ptr(Hb), _ptr(Hp), _ptr(rp), npar, self.Fl, Bs * C, C, 0b1, 0, _ptr(H), _ptr(wb),
                              _ptr(wp), _ptr(wyy), _stream()), "dt_sibling")
        return H, wyy

    def _merge(self, recl, n):
        """Multi-rank: per node, the highest-gain record of the ranks' feature
        slices (ties to the lowest rank = lowest feature) with its go-left mask;
        stream-ordered all-gather, no host sync."""
        W, Bs = self.W, self.Bs
        rows = recl[:n * RS].view(n, RS)
        rb = 13 * 8
        buf = torch.cat([rows[:, :13].contiguous().view(torch.uint8).view(n, rb), self.mask[:n * Bs].view(n, Bs)], 1)
        g = coll.all_gather_dim0(buf).view(W, n, rb + Bs)
        gains = g[:, :, :8].contiguous().view(torch.float64).view(W, n)
        best = torch.argmax(gains, 0)
        win = g[best, torch.arange(n, device=buf.device)]
        pk = win[:, :rb].contiguous().view(torch.float64).view(n, 13)
        rows[:, :13].copy_(pk)
        self.mask[:n * Bs].view(n, Bs).copy_(win[:, rb:])
        okf = pk[:, OK] > 0
        self.feat_i[:n].copy_(torch.where(okf, pk[:, FEAT], torch.zeros_like(pk[:, FEAT])).to(torch.int32))

    def _level(self, d, cur):
        """Split search + partition of level d; returns the new current buffer."""
        lh, ls, gp = self.lh, self.ls, self.gp
        n = 1 << d
        Bs = self.Bs
        H, wyy = self._hist(d, cur)
        recl = self._rec_lvl(d)
        s = _stream()
        if self.colsamp:
            rp = self._rec_lvl(d - 1) if d > 0 else None
            _ck(lh.h2o_dt_colmask(d, _ptr(rp), _ptr(self.cs_elig), _ptr(self.cs_m), _ptr(self.cs_k),
                                  _ptr(self.cs_seed), self.f0, self.Fl, _ptr(self.okm), s), "dt_colmask")
        _ck(ls.h2o_split_find_b(_ptr(H), self.Fl, n, Bs, _ptr(wyy), _ptr(self.okm), _ptr(self.mono),
                                float(gp.min_rows), float(gp.min_split_improvement), float(gp.reg_lambda),
                                float(gp.reg_alpha), float(gp.gamma), 0, _ptr(self.split_out), None, 0, s),
            "split_find")
        _ck(ls.h2o_split_select2(_ptr(self.split_out), _ptr(H), self.Fl, n, Bs, self.f0, 2.0 * float(gp.min_rows), RS,
                                 _ptr(recl), _ptr(self.mask), _ptr(self.feat_i), s), "split_select2")
        if self.W > 1:
            self._merge(recl, n)
        s = _stream()
        _ck(lh.h2o_dt_items(0, _ptr(recl), n, self.D, 0, self.chunk_p, self.cap_p, _ptr(self.pwork), _ptr(self.fbase),
                            _ptr(self.counts), s), "dt_items(part)")
        _ck(lh.h2o_part_flags_dev(_ptr(self.pcodes), 1, self.prs, self.pfs, _ptr(self.ridx[cur]), _ptr(self.pwork),
                                  _ptr(self.fbase), self.cap_p, _ptr(self.feat_i), _ptr(self.mask), Bs,
                                  _ptr(self.flags), _ptr(self.cnt), _ptr(self.counts), s), "part_flags_dev")
        _ck(lh.h2o_dt_offsets(_ptr(self.cnt), _ptr(self.pwork), _ptr(self.counts), _ptr(recl), n,
                              _ptr(self._rec_lvl(d + 1)), _ptr(self.loff), _ptr(self.roff), s), "dt_offsets")
        nxt = cur ^ 1
        _ck(lh.h2o_part_compact_dev(_ptr(self.ridx[cur]), _ptr(self.pwork), _ptr(self.fbase), self.cap_p,
                                    _ptr(self.flags), _ptr(self.loff), _ptr(self.roff), _ptr(self.ridx[nxt]),
                                    _ptr(self.pos[cur]), _ptr(self.pos[nxt]), _ptr(self.counts), s),
            "part_compact_dev")
        return nxt

    def _sequence(self):
        """One tree: residual -> levels -> leaf values -> per-row scatter."""
        lh, drv = self.lh, self.drv
        s = _stream()
        y = drv.yb if self.bern else torch.nan_to_num(drv.yf)
        if not hasattr(self, "_y"):
            self._y = y.contiguous().to(torch.float32)
        f = drv._f[:, 0]
        _ck(lh.h2o_gbm_grad(_ptr(self._y), _ptr(f), _ptr(self.wbuf) if self.sampled else None,
                            1 if self.bern else 0, self.N, _ptr(self.pos[0]), _ptr(self.dbuf), s), "gbm_grad")
        _ck(lh.h2o_iota_i32(_ptr(self.ridx[0]), self.N, s), "iota")
        self.rec.zero_()
        self.sums.zero_()
        _ck(lh.h2o_dt_root(_ptr(self.rec), self.N, _stream()), "dt_root")
        cur = 0
        for d in range(self.D):
            cur = self._level(d, cur)
        s = _stream()
        _ck(lh.h2o_dt_items(2, _ptr(self.rec), self.nh, self.D, 0, self.chunk_l, self.cap_l, _ptr(self.lwork), None,
                            _ptr(self.counts), s), "dt_items(leaf)")
        _ck(lh.h2o_leaf_pos_dev(_ptr(self.pos[cur]), _ptr(self.lwork), self.cap_l, 1 if self.bern else 0,
                                _ptr(self.sums), _ptr(self.counts), s), "leaf_pos_dev")
        if self.W > 1:
            coll.allreduce_(self.sums)
        s = _stream()
        _ck(lh.h2o_dt_leaf_vals(_ptr(self.rec), _ptr(self.sums), self.nh, self.D, _ptr(self.lr_t), self.maxabs,
                                _ptr(self.vals), s), "dt_leaf_vals")
        _ck(lh.h2o_leaf_scatter_dev(_ptr(self.ridx[cur]), _ptr(self.lwork), self.cap_l, _ptr(self.vals),
                                    _ptr(self.dbuf), _ptr(self.counts), s), "leaf_scatter_dev")
        self.cur = cur

    def set_col_sampling(self, tree_mask):
        """Per-tree inputs of dt_colmask_kernel: the eligible features (the
        per-tree column sample) and, per level, k and the seed -- drawn from
        the grower's generator in the level loop's order (engine._col_sel:
        one draw per splitting level that samples)."""
        if not self.colsamp:
            return
        g, gp, F, D = self.drv.grower, self.gp, self.F, self.D
        base = np.ones(F, dtype=bool) if tree_mask is None else np.asarray(tree_mask, dtype=bool)
        elig = np.nonzero(base)[0]
        m = int(elig.size)
        ks = np.zeros(D, dtype=np.int32)
        seeds = np.zeros(D, dtype=np.int64)
        for d in range(D):
            rate = gp.col_sample_rate * (gp.col_sample_rate_change_per_level ** d)
            k = max(1, int(np.floor(rate * m + 0.5))) if rate < 1.0 else m
            if k >= m:
                ks[d] = m
            else:
                ks[d] = k
                seeds[d] = int(g.rng.randint(0, 2 ** 31 - 1))
        e = np.zeros(max(F, 1), dtype=np.int64)
        e[:m] = elig
        de, dm, dk, dsd = self._upload([e, np.array([m], dtype=np.int32), ks, seeds])
        self.cs_elig.copy_(de)
        self.cs_m.copy_(dm)
        self.cs_k.copy_(dk)
        self.cs_seed.copy_(dsd)

    def run(self, lr, pending, w=None):
        """Grow one tree; `pending`: the previous tree's scatter (dbuf) has not
        been folded into f yet; `w`: this tree's 0/1 row weights (row
        sampling).  Returns (host record view, event)."""
        if not pending:
            self.dbuf.zero_()
        if self.sampled:
            self.wbuf.copy_(w)
        self.lr_t.fill_(float(lr))
        if not self.bern:
            # gaussian: per-tree residual bound for the fixed-point scales (the
            # one host read of the tree); no graph (the scales are launch args)
            f = self.drv._f[:, 0]
            z = (torch.nan_to_num(self.drv.yf) - (f + self.dbuf))
            self.vmax = [1.0, float(z.abs().max())]
            self._scales()
            self._sequence()
        elif self.W == 1 and os.environ.get("H2O3_DEV_TREE_GRAPH", "1") == "1":
            if self.graph is None:
                # first tree eagerly (kernel attributes, lazy library state),
                # then capture the sequence for every later tree: capture only
                # records, so f / dbuf / the record of this tree are untouched
                self._sequence()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with graphs.capture(g):
                    self._sequence()
                self.graph = g
            else:
                self.graph.replay()
        else:
            self._sequence()
        return self._copy_out()

    def _copy_out(self):
        k = self._k
        self._k ^= 1
        h = self._hv[k]
        if h is None:
            h = self._hv[k] = torch.empty(self.nh * RS, dtype=torch.float64, pin_memory=True)
        h.copy_(self.rec, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return h, ev

    # ---------------------------------------------------------------- host tree
    def decode(self, rec_h, criterion="se"):
        """Tree (BFS node order of the level loop) from the heap record."""
        D, nh = self.D, self.nh
        R = np.asarray(rec_h, dtype=np.float64).reshape(nh, RS)
        lv = np.floor(np.log2(np.arange(nh) + 1)).astype(np.int64)
        ok = R[:, OK] > 0
        exists = np.zeros(nh, dtype=bool)
        exists[0] = True
        for d in range(1, D + 1):
            a, b = (1 << d) - 1, (1 << (d + 1)) - 1
            par = (np.arange(a, b) - 1) >> 1
            exists[a:b] = exists[par] & ok[par]
        split = exists & ok & (lv < D)
        ids = np.nonzero(exists)[0]
        bfs = np.full(nh, -1, dtype=np.int64)
        bfs[ids] = np.arange(ids.size)
        n = ids.size
        tb = _TreeBuf(cap=max(n, 1))
        tb.n = n
        par = np.maximum((ids - 1) >> 1, 0)
        is_left = (ids % 2) == 1
        w_own = R[ids, T0]
        w_par = np.where(is_left, R[par, L0], R[par, R0])
        tb.weight[:n] = np.where(lv[ids] < D, w_own, w_par)
        tb.depth[:n] = lv[ids]
        sp = split[ids]
        hs = ids[sp]
        bi = bfs[hs]
        f = R[hs, FEAT].astype(np.int64)
        t = R[hs, T].astype(np.int64)
        opt = R[hs, OPT].astype(np.int64)
        tb.feat[bi] = f
        tb.left[bi] = bfs[2 * hs + 1]
        tb.right[bi] = bfs[2 * hs + 2]
        tb.gain[bi] = R[hs, GAIN]
        tb.split_code[bi] = t
        cm = self.cutmat
        tb.thr[bi] = np.where(opt == 2, np.inf, cm[f, np.minimum(t, cm.shape[1] - 1)])
        na = opt == 1
        if criterion != "xgb":
            # no NA weight reached this node on the split column: NAs of later
            # data go to the heavier child (DTree.java:1475-1478)
            free = (R[hs, NAW] == 0) & (opt != 2)
            na = np.where(free, R[hs, L0] > R[hs, R0], na)
        tb.na_left[bi] = na
        lf = ~sp
        tb.value[bfs[ids[lf]]] = R[ids[lf], VAL]
        return tb.to_tree()
