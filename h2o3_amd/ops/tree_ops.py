"""Python entry points for the tree-engine kernels (HIP on GPU, torch on CPU).

`hist_build`, `partition` and `fill_nid` dispatch to libtree_hist.so on a
GPU device; the torch implementations below are the fp32 references used
on CPU and by the numerics tests.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch

from . import _native

_LDS_BUDGET = 80 * 1024   # bytes of LDS histogram per workgroup (2+ WG / CU)
_c_void = ctypes.c_void_p
_c_int = ctypes.c_int
_c_ll = ctypes.c_longlong



# Upload sequence numbers: every staged upload gets the next number; the
# host learns that all uploads numbered below `_synced_upto` have completed
# when it waits on an event recorded after them on the same stream
# (host_synced(mark) with mark = upload_mark() taken at the record), so a
# staging slot is rewritten without a stream sync once its upload is below
# the mark -- no per-upload event record / query.
_upload_seq = 0
_synced_upto = 0


def upload_mark():
    """Sequence number of the next upload: record it together with an event;
    every upload before it is complete once the event is."""
    return _upload_seq


def host_synced(mark=None):
    """Tell the upload ring that every copy queued before `mark` (an
    upload_mark() taken when the waited-on event was recorded) has completed;
    mark=None: the caller drained the whole stream."""
    global _synced_upto
    m = _upload_seq if mark is None else mark
    if m > _synced_upto:
        _synced_upto = m


class _PinnedRing:
    """Reusable staging for the small per-level host->device uploads (work
    items, per-chunk metadata, column masks): pinned host slots and device
    slots, both reused.  A copy from a pinned slot is truly asynchronous; a
    slot is only rewritten once its previous upload is known complete
    (sequence number below the synced mark), else the host synchronises
    first, so no pending copy ever reads overwritten bytes.  Device slots are
    consumed by kernels queued after the copy on the same stream, and a later
    copy into the slot is queued behind them: stream order keeps them intact.
    A returned device tensor ALIASES its slot: it must be consumed (by work
    queued on the stream) before len(ring) further uploads.  (Per-upload
    events and device allocations cost ~30 us of host time per upload.)"""

    def __init__(self, n=16):
        self.bufs = [None] * n
        self.dbufs = [None] * n
        self.seq = [-1] * n
        self.i = 0

    def upload(self, a: np.ndarray, dev):
        global _upload_seq
        k = self.i
        self.i = (self.i + 1) % len(self.bufs)
        if self.seq[k] >= _synced_upto:
            torch.cuda.current_stream(dev).synchronize()
            host_synced()
        nb = max(a.nbytes, 8)
        buf = self.bufs[k]
        if buf is None or buf.numel() < nb:
            cap = max(nb, 1 << 16)
            buf = self.bufs[k] = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
            self.dbufs[k] = torch.empty(cap, dtype=torch.uint8, device=dev)
        dbuf = self.dbufs[k]
        if dbuf.device != torch.device(dev) if not isinstance(dev, torch.device) else dbuf.device != dev:
            dbuf = self.dbufs[k] = torch.empty(buf.numel(), dtype=torch.uint8, device=dev)
        tdt = torch.from_numpy(a[:0]).dtype
        stage = buf[:a.nbytes].view(tdt).view(a.shape)
        stage.numpy()[...] = a
        out = dbuf[:a.nbytes].view(tdt).view(a.shape)
        out.copy_(stage, non_blocking=True)
        self.seq[k] = _upload_seq
        _upload_seq += 1
        return out


_ring = None


def _h2d(a, dev):
    """Small host array -> device without a stream sync, staged through a
    reusable pinned ring (one pinned allocation per slot, not per call)."""
    a = np.ascontiguousarray(a)
    if dev.type != "cuda":
        return torch.from_numpy(a)
    global _ring
    if _ring is None:
        _ring = _PinnedRing()
    return _ring.upload(a, dev)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


# Environment switches read on the per-level hot path: inside a tree build
# (env_scope) each key is read once per tree, elsewhere every call reads
# os.environ (tests flip switches between direct kernel calls).
_ENV_CACHE = None


def env(key, default=None):
    c = _ENV_CACHE
    if c is None:
        return os.environ.get(key, default)
    k = (key, default)
    v = c.get(k, c)
    if v is c:
        v = c[k] = os.environ.get(key, default)
    return v


class env_scope:
    """Cache environment switches for the duration of one tree build."""

    def __enter__(self):
        global _ENV_CACHE
        self._prev = _ENV_CACHE
        _ENV_CACHE = {}
        return self

    def __exit__(self, *exc):
        global _ENV_CACHE
        _ENV_CACHE = self._prev
        return False


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_get_device = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """Current HIP stream as a ctypes pointer (the raw C getters: ~10x cheaper
    than torch.cuda.current_stream(), called for every kernel launch)."""
    if _raw_stream is not None and _get_device is not None:
        return ctypes.c_void_p(_raw_stream(_get_device()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _lib():
    lib = _native.get_lib("tree_hist")
    if lib is not None and not getattr(lib, "_typed", False):
        lib.h2o_hist_build.argtypes = [_c_void, _c_int, _c_int, _c_void, _c_void, _c_void, _c_void, _c_int,
                                       _c_int, _c_int, _c_int, ctypes.c_float, ctypes.c_float, _c_void, _c_int, _c_int,
                                       _c_int, _c_void, _c_int, _c_void, _c_void]
        lib.h2o_hist_quad3.argtypes = [_c_void, _c_int, _c_void, _c_void, _c_void, _c_void, _c_int, _c_int, _c_int,
                                       _c_int, ctypes.c_float, ctypes.c_float, _c_void, _c_int, _c_int, _c_int,
                                       _c_void, _c_int, _c_ll, _c_int, _c_void, _c_void]
        lib.h2o_hist_bm.argtypes = [_c_void, _c_int, _c_void, _c_void, _c_void, _c_void, _c_int, _c_int, _c_int,
                                    _c_int, ctypes.c_float, ctypes.c_float, _c_void, _c_int, _c_int, _c_void, _c_int,
                                    _c_ll, _c_int, _c_void, _c_void, _c_void, _c_void]
        lib.h2o_hist_build_pk.argtypes = [_c_void, _c_int, _c_int, _c_void, _c_void, _c_void, _c_void, _c_int,
                                          _c_int, _c_int, _c_int, ctypes.c_float, _c_ll, _c_void, _c_int, _c_int,
                                          _c_void, _c_int, _c_void, _c_void]
        lib.h2o_part_flags.argtypes = [_c_void, _c_int, _c_ll, _c_ll, _c_void, _c_void, _c_void, _c_int, _c_void,
                                       _c_void, _c_int, _c_void, _c_void, _c_void]
        lib.h2o_part_compact.argtypes = [_c_void, _c_void, _c_void, _c_int, _c_void, _c_void, _c_void, _c_void,
                                         _c_void, _c_void, _c_void]
        lib.h2o_part_count.argtypes = [_c_void, _c_int, _c_ll, _c_ll, _c_void, _c_void, _c_int, _c_void,
                                       _c_void, _c_int, _c_void, _c_void]
        lib.h2o_part_scatter.argtypes = [_c_void, _c_int, _c_ll, _c_ll, _c_void, _c_void, _c_int, _c_void,
                                         _c_void, _c_int, _c_void, _c_void, _c_void, _c_void, _c_void, _c_void,
                                         _c_void, _c_void]
        lib.h2o_fill_nid.argtypes = [_c_void, _c_void, _c_int, _c_void, _c_void]
        lib._typed = True
    return lib


def channels(mode: int) -> int:
    """Histogram channels: 0 (w, w*y), 1 (g, h), 2 (w), 3 uplift (wt, wt*y, wc, wc*y)."""
    return 1 if mode == 2 else (4 if mode == 3 else 2)


def feature_group(F: int, Bs: int, mode: int, budget: int = _LDS_BUDGET) -> int:
    """Features per workgroup (= lanes per row in the wave mapping).

    Minimises wave-instructions per row, ~ n_groups / floor(64 / FGL), under
    the LDS budget; ties go to fewer groups (less re-reading of row data)."""
    import os
    if env("H2O3_HIST_FGL"):
        return max(1, min(64, int(os.environ["H2O3_HIST_FGL"]), F))
    C = channels(mode)
    fmax = max(1, min(64, budget // (Bs * C * 8)))
    best = None
    for ng in range(1, F + 1):
        fgl = -(-F // ng)
        if fgl > fmax:
            continue
        # wave-instructions per row + re-read of the row payload per group
        cost = ng / (64 // fgl) + 0.05 * ng
        key = (round(cost, 6), ng)
        if best is None or key < best[0]:
            best = (key, fgl)
        if fgl == 1:
            break
    return best[1] if best else 1


def quad_groups(F: int, Fp: int, Bs: int, pack: bool, budget: int = _LDS_BUDGET):
    """(n_fg, fgw) of the grouped-lane histogram kernel: the FEWEST feature
    groups whose LDS histogram (fgw x (Bs + 1) x channels x 8 B) fits the
    per-workgroup budget (2 workgroups per CU), widths a multiple of 4 and at
    most 64, all in one launch (the kernel's cost is per group pass over the
    rows: scripts/hist_fsweep_mb.py).  F = 100, 256 bins, packed -> 3 x 36."""
    CL = 1 if pack else 2
    fmax = max(4, min(64, (budget // ((Bs * CL + CL) * 8)) // 4 * 4))
    fmax = int(env("H2O3_HIST_FGW", fmax))
    n_fg = -(-F // fmax)
    while True:
        fgw = -(-(-(-F // n_fg)) // 4) * 4
        if n_fg * fgw <= Fp or fgw <= 4:
            return n_fg, fgw
        n_fg += 1


def bm_groups(F: int, Fp: int, Bs: int, one_channel: bool):
    """(n_fg, G) of the bank-conflict-free bin-major kernel (hist_bm_kernel):
    G in {64, 32, 16} features per group (G <= 32 with two LDS channels), the
    FEWEST groups whose code dwords stay inside the Fp-byte row and whose LDS
    histogram (Bs x G x channels x 8 B) fits 160 KB; None when no width fits
    (the grouped-lane kernel then runs).  F = 100 (Fp 128), 256 bins: packed
    -> 2 x 64 (128 KB), two channels -> 4 x 32."""
    if env("H2O3_HIST_BM", "1") != "1" or Bs > 256 or Bs % 4 or Fp % 4:
        return None
    cl = 1 if one_channel else 2
    best = None
    for G in (64, 32, 16):
        if cl == 2 and G == 64:
            continue
        n_fg = -(-F // G)
        if n_fg * G > Fp or Bs * G * cl * 8 > 160 * 1024:
            continue
        if best is None or n_fg < best[0]:
            best = (n_fg, G)
    return best


def bm_part(n_items, n_fg, Bs, G, one_channel, dev):
    """Scratch of the two-pass flush of hist_bm_kernel: one u64 partial image
    [Bs][G * channels] per (work item, group); None = f64 atomic flush
    (H2O3_HIST_BM_RED=0)."""
    if env("H2O3_HIST_BM_RED", "1") != "1":
        return None
    cl = 1 if one_channel else 2
    return torch.empty(int(n_items) * n_fg * Bs * G * cl, dtype=torch.int64, device=dev)


def make_work(starts, counts, slots, chunk):
    """Chunk node segments into (slot, start, count, chunk_id) work items
    (host, vectorized) -> int32 numpy array [n_items, 4]."""
    st = np.asarray(starts, dtype=np.int64).reshape(-1)
    ct = np.asarray(counts, dtype=np.int64).reshape(-1)
    sl = np.asarray(list(slots), dtype=np.int64).reshape(-1)
    m = ct > 0
    st, ct, sl = st[m], ct[m], sl[m]
    if st.size == 0:
        return np.zeros((0, 4), dtype=np.int32)
    nch = (ct + chunk - 1) // chunk
    rep = np.repeat(np.arange(st.size), nch)
    k = np.arange(int(nch.sum())) - np.repeat(np.cumsum(nch) - nch, nch)
    p = st[rep] + k * chunk
    c = np.minimum(chunk, st[rep] + ct[rep] - p)
    return np.stack([sl[rep], p, c, k], 1).astype(np.int32)


def channel_max(va, vb, mode):
    """Max |value| per histogram channel (host floats, one device sync)."""
    if mode == 3:
        a, b = channel_max(va, vb[0], 0), channel_max(va, vb[1], 0)
        return [max(a[0], b[0]), max(a[1], b[1])]
    if mode == 0:
        w = vb if vb is not None else None
        # NaN responses are zero-weight rows (NaN-masked payloads): not part of the bound
        m1 = torch.nan_to_num(va.abs() * (w.abs() if w is not None else 1), nan=0.0).max() if va.numel() \
            else va.new_zeros(())
        m0 = w.abs().max() if (w is not None and w.numel()) else va.new_ones(())
    elif mode == 1:
        m0, m1 = va.abs().max(), vb.abs().max()
    else:
        m0 = vb.abs().max() if vb is not None else va.new_ones(())
        m1 = m0
    t = torch.stack([m0.float(), m1.float()]).cpu().tolist()
    return [x if x == x else 0.0 for x in t]


def fixed_point_scale(maxv, nmax):
    """Power-of-two scale S so that nmax values of magnitude <= maxv sum
    below 2^62 in int64 (exact fixed-point histogram accumulation)."""
    import math
    if not maxv or maxv <= 0 or not math.isfinite(maxv):
        return 1.0
    k = math.floor(math.log2(2.0 ** 62 / (maxv * max(nmax, 1))))
    return float(2.0 ** max(min(k, 100), -100))


def _pack_scale(vmax, chunk):
    """(s1, bq) of the packed 40-bit response field: chunk * (2*bq + 1) < 2^40."""
    vm = max(float(vmax), 1e-30)
    k = math.floor(math.log2((2.0 ** 40 - 2 * chunk) / (2.0 * chunk * vm * 1.0001)))
    s1 = 2.0 ** k
    return s1, int(math.ceil(vm * s1))


# Rows per histogram workgroup: every workgroup zeroes and flushes a full
# feature-group histogram (fixed cost), so chunks aim at ~128K rows while
# keeping >= 512 workgroups to fill the chip (scripts/hist_bm_mb.py with the
# two-pass flush of the bin-major kernel: 100M-row root 3.69 -> 3.35 ms,
# 12.5M-row root 0.59 -> 0.47 ms vs 64K rows, deeper levels unchanged).
_PK_BUDGET = 152 * 1024     # packed wide-code histogram: one 512-thread workgroup per CU
_HIST_CHUNK_ROWS = 131072
_HIST_MIN_BLOCKS = 512


def hist_chunk(total, n_fg, target_blocks=None):
    """Rows per work item for `total` rows over n_fg feature groups."""
    tb = env("H2O3_HIST_TB", target_blocks)
    if tb is not None:
        n_chunks = max(1, int(tb) // n_fg)
    else:
        rows = int(env("H2O3_HIST_CHUNK", _HIST_CHUNK_ROWS))
        n_chunks = max(-(-_HIST_MIN_BLOCKS // n_fg), -(-total // rows))
    return max(2048, -(-total // n_chunks))


def hist_build(bd, ridx, va, vb, mode, starts, counts, n_slots, use_native=None, target_blocks=None, vmax=None,
               want_wyy=False, posv=False, unit_w=False, need_mask=None):
    """Histograms of the row segments [starts[i], starts[i]+counts[i]) of
    ridx into slot i.  Returns hist [F, n_slots, Bs, C] float64 (and, with
    want_wyy in mode 0, the per-slot sum of w*y*y).  posv: va/vb are stored
    in position (row-permutation) order instead of row order.
    need_mask: optional [n_slots, >=F] bool tensor of the features that will be
    scored per slot (DRF mtries); feature groups with no needed feature are
    skipped by the kernels and their histogram entries stay zero."""
    C = channels(mode)
    dev = ridx.device
    nh = bd.F * n_slots * bd.Bs * C
    if want_wyy and mode == 0:
        # one zero-fill for the histogram and the per-slot w*y*y sums
        buf = torch.zeros(nh + n_slots, dtype=torch.float64, device=dev)
        hist = buf[:nh].view(bd.F, n_slots, bd.Bs, C)
        wyy = buf[nh:]
    else:
        hist = torch.zeros((bd.F, n_slots, bd.Bs, C), dtype=torch.float64, device=dev)
        wyy = None
    ret = (lambda: (hist, wyy)) if want_wyy else (lambda: hist)
    native = dev.type == "cuda" if use_native is None else use_native
    if native:
        lib = _lib()
        kern = env("H2O3_HIST_KERNEL", "quad")
        total = int(sum(counts))
        if total == 0:
            return ret()
        quad = bd.code_bytes == 1 and bd.Fp % 4 == 0 and bd.Bs <= 256 and kern == "quad" and mode in (0, 1, 2)
        pack = quad and mode == 0 and unit_w and env("H2O3_HIST_PACK", "1") == "1"
        # H2O3_HIST_BIG=1 (A/B): one 1024-thread workgroup per CU with up to 160 KB of LDS histogram
        big = env("H2O3_HIST_BIG", "0") == "1"
        qbudget = 156 * 1024 if big else _LDS_BUDGET
        bm = None
        if quad:
            bm = bm_groups(bd.F, bd.Fp, bd.Bs, pack or mode == 2)
            n_fg, fgw = bm if bm is not None else quad_groups(bd.F, bd.Fp, bd.Bs, pack, qbudget)
        pkw = False
        if not quad:
            # wide (2-byte) codes, 0/1 weights: one packed u64 LDS atomic per
            # (row, feature) -- half the LDS per feature, so ~2x the features
            # per workgroup and half the re-reads of the rows per level
            pkw = mode == 0 and unit_w and bd.code_bytes == 2 and env("H2O3_HIST_PACK", "1") == "1"
            FG = feature_group(bd.F, bd.Bs, 2 if pkw else mode, budget=_PK_BUDGET if pkw else _LDS_BUDGET)
            n_fg = (bd.F + FG - 1) // FG
        chunk = hist_chunk(total, n_fg, target_blocks)
        if pkw and chunk >= (1 << 23):
            pkw = False
            FG = feature_group(bd.F, bd.Bs, mode)
            n_fg = (bd.F + FG - 1) // FG
        if pack and chunk >= (1 << 23):
            pack = False
            bm = bm_groups(bd.F, bd.Fp, bd.Bs, mode == 2)
            n_fg, fgw = bm if bm is not None else quad_groups(bd.F, bd.Fp, bd.Bs, False, qbudget)
        items = make_work(starts, counts, range(n_slots), chunk)
        if len(items) == 0:
            return ret()
        work = _h2d(items, dev)

        def _need(fg):
            if need_mask is None:
                return None
            m = need_mask[:, :bd.F].to(device=dev, dtype=torch.bool)
            ng = (bd.F + fg - 1) // fg
            if ng * fg > bd.F:
                m = torch.cat([m, torch.zeros((m.shape[0], ng * fg - bd.F), dtype=torch.bool, device=dev)], 1)
            return m.view(m.shape[0], ng, fg).any(2).to(torch.uint8).contiguous()
        threads = 512 if chunk >= 8192 else 256
        if vmax is None:
            vmax = channel_max(va, vb, mode)
        s0, s1 = (fixed_point_scale(m, chunk) for m in vmax)
        if quad:
            bq = -1
            if pack:
                s1, bq = _pack_scale(vmax[1] if vb is None else max(vmax[1], 0.0), chunk)
            need = _need(fgw)
            if bm is not None:
                part = bm_part(len(items), n_fg, bd.Bs, fgw, pack or mode == 2, dev)
                rc = lib.h2o_hist_bm(_ptr(bd.codes), bd.Fp, _ptr(ridx), _ptr(va), _ptr(vb), _ptr(work), len(items),
                                     bd.F, 0, bd.Bs, s0, s1, _ptr(hist), n_slots, mode, _ptr(wyy), 1 if posv else 0,
                                     bq, fgw, _ptr(need), None, _ptr(part), _stream())
                if rc != 0:
                    raise RuntimeError(f"h2o_hist_bm failed: error {rc} (F={bd.F}, Fp={bd.Fp}, G={fgw})")
                return ret()
            rc = lib.h2o_hist_quad3(_ptr(bd.codes), bd.Fp, _ptr(ridx), _ptr(va), _ptr(vb), _ptr(work), len(items),
                                    bd.F, 0, bd.Bs, s0, s1, _ptr(hist), n_slots, mode, 1024 if big else 512, _ptr(wyy),
                                    1 if posv else 0, bq, fgw, _ptr(need), _stream())
            if rc != 0:
                raise RuntimeError(f"h2o_hist_quad3 failed: error {rc} (F={bd.F}, Fp={bd.Fp}, fgw={fgw})")
            return ret()
        need = _need(FG)
        if pkw:
            s1p, bqp = _pack_scale(vmax[1] if vb is None else max(vmax[1], 0.0), chunk)
            rc = lib.h2o_hist_build_pk(_ptr(bd.codes), bd.code_bytes, bd.Fp, _ptr(ridx), _ptr(va), _ptr(vb),
                                       _ptr(work), len(items), bd.F, FG, bd.Bs, s1p, bqp, _ptr(hist), n_slots,
                                       threads, _ptr(wyy), 1 if posv else 0, _ptr(need), _stream())
            if rc != 0:
                raise RuntimeError(f"h2o_hist_build_pk failed: hip error {rc}")
            return ret()
        rc = lib.h2o_hist_build(_ptr(bd.codes), bd.code_bytes, bd.Fp, _ptr(ridx), _ptr(va), _ptr(vb), _ptr(work),
                                len(items), bd.F, FG, bd.Bs, s0, s1, _ptr(hist), n_slots, mode, threads, _ptr(wyy),
                                1 if posv else 0, _ptr(need), _stream())
        if rc != 0:
            raise RuntimeError(f"h2o_hist_build failed: hip error {rc}")
        return ret()
    if posv:
        # expand position-ordered payloads to row order for the reference path
        va_r = torch.empty_like(va)
        va_r[ridx.long()] = va
        vb_r = None
        if vb is not None:
            vb_r = torch.empty_like(vb)
            vb_r[ridx.long()] = vb
        va, vb = va_r, vb_r
    _hist_build_torch(bd, ridx, va, vb, mode, starts, counts, hist)
    if wyy is not None:
        for slot, (st, ct) in enumerate(zip(starts, counts)):
            r = ridx[st: st + ct].long()
            w = vb[r].to(torch.float64) if vb is not None else torch.ones(r.numel(), dtype=torch.float64, device=dev)
            y = va[r].to(torch.float64)
            wyy[slot] = (w * y * y).sum()
    return ret()


def _hist_build_torch(bd, ridx, va, vb, mode, starts, counts, hist):
    F, Bs = bd.F, bd.Bs
    C = channels(mode)
    codes = bd.codes
    for slot, (st, ct) in enumerate(zip(starts, counts)):
        if ct <= 0:
            continue
        r = ridx[st: st + ct].long()
        a = va[r].to(torch.float32)
        if mode == 0:
            w = vb[r].to(torch.float32) if vb is not None else torch.ones_like(a)
            vals = torch.stack([w, w * a], 1)
        elif mode == 1:
            vals = torch.stack([a, vb[r].to(torch.float32)], 1)
        else:
            w = vb[r].to(torch.float32) if vb is not None else torch.ones_like(a)
            vals = w.reshape(-1, 1)
        cd = codes[r][:, :F].to(torch.int64)  # [n, F]
        idx = (torch.arange(F, device=cd.device).reshape(1, F) * Bs + cd).reshape(-1)
        flat = torch.zeros((F * Bs, C), dtype=torch.float64, device=cd.device)
        v = vals.unsqueeze(1).expand(-1, F, C).reshape(-1, C).to(torch.float64)
        flat.index_add_(0, idx, v)
        hist[:, slot] = flat.reshape(F, Bs, C)
    return hist


_PAIR_CHUNK = 16384
# pairs of one node per workgroup in pair_hist_dev (1 = one pair per workgroup)
_PAIR_KP = int(os.environ.get("H2O3_PAIR_KP", 4))


def pair_hist(bd, ridx, va, vb, mode, node_st, node_ct, pair_node, pair_feat, vmax=None, posv=False,
              want_wyy=False, use_native=None, chunk=_PAIR_CHUNK):
    """Histograms of (node, feature) PAIRS straight from the rows (the
    mtries-sampled columns of a wide frontier, DRF deep levels): pair i covers
    the rows of node pair_node[i] (segment [node_st, node_st + node_ct) of
    ridx) on feature pair_feat[i] (global index).  node_st / node_ct /
    pair_node / pair_feat are host int arrays; pairs of one node must be
    consecutive.  Returns (Hp [P, Bs, 2] float64, wyy [n_nodes] float64 or
    None): wyy = per-node sum of w*y*y (mode 0), taken from each node's first
    pair.  mode 0: (w, w*y) with vb = weights (or NaN-masked va when vb is
    None); mode 1: (g, h).  HIP kernel `pair_hist_kernel` (tree_hist.hip) on
    the GPU, an index_add reference otherwise."""
    assert mode in (0, 1)
    dev = ridx.device
    st = np.asarray(node_st, dtype=np.int64)
    ct = np.asarray(node_ct, dtype=np.int64)
    pn = np.asarray(pair_node, dtype=np.int64)
    pf = np.asarray(pair_feat, dtype=np.int64)
    P, n = pn.size, st.size
    Bs = bd.Bs
    first = np.ones(P, dtype=bool)
    first[1:] = pn[1:] != pn[:-1]
    wyy_n = torch.zeros(n, dtype=torch.float64, device=dev) if (want_wyy and mode == 0) else None
    native = (dev.type == "cuda" and bd.codes_col is not None) if use_native is None else use_native
    if P == 0:
        return torch.zeros((0, Bs, 2), dtype=torch.float64, device=dev), wyy_n
    if native:
        lib = _lib()
        if not getattr(lib, "_typed_pair", False):
            lib.h2o_pair_hist.argtypes = [_c_void, _c_int, _c_ll, _c_void, _c_void, _c_void, _c_void, _c_int,
                                          _c_void, _c_int, _c_int, _c_int, ctypes.c_float, ctypes.c_float, _c_void,
                                          _c_void, _c_void]
            lib._typed_pair = True
        pct = ct[pn]
        nch = np.maximum((pct + chunk - 1) // chunk, 0)
        live = pct > 0
        rep = np.repeat(np.arange(P), nch)
        k = np.arange(int(nch.sum())) - np.repeat(np.cumsum(nch) - nch, nch)
        start = st[pn][rep] + k * chunk
        cnt = np.minimum(chunk, pct[rep] - k * chunk)
        flags = (nch[rep] == 1).astype(np.int64) | first[rep].astype(np.int64) * 2
        items = np.stack([rep, start, cnt, flags], 1).astype(np.int32)
        Hp = torch.empty((P, Bs, 2), dtype=torch.float64, device=dev)
        multi = np.nonzero((nch > 1) | ~live)[0]
        if multi.size:
            Hp.index_fill_(0, _h2d(multi.astype(np.int64), dev), 0.0)
        pwyy = torch.zeros(P, dtype=torch.float64, device=dev) if wyy_n is not None else None
        if len(items):
            buf = _h2d(np.concatenate([items.reshape(-1), pf.astype(np.int32)]), dev)
            work, pfd = buf[:4 * len(items)], buf[4 * len(items):]
            if vmax is None:
                vmax = channel_max(va, vb, mode)
            s0, s1 = (fixed_point_scale(m, min(chunk, int(pct.max()))) for m in vmax)
            rc = lib.h2o_pair_hist(_ptr(bd.codes_col), bd.code_bytes, bd.codes_col.stride(0), _ptr(ridx), _ptr(va),
                                   _ptr(vb), _ptr(work), len(items), _ptr(pfd), Bs, mode, 1 if posv else 0, s0, s1,
                                   _ptr(Hp), _ptr(pwyy), _stream())
            if rc != 0:
                raise RuntimeError(f"h2o_pair_hist failed: {rc}")
        if wyy_n is not None:
            fi = np.nonzero(first)[0]
            wyy_n[_h2d(pn[fi], dev)] = pwyy[_h2d(fi.astype(np.int64), dev)]
        return Hp, wyy_n
    # reference path: expand every pair's rows, one index_add
    if posv:
        va_r = torch.empty_like(va)
        va_r[ridx.long()] = va
        vb_r = None
        if vb is not None:
            vb_r = torch.empty_like(vb)
            vb_r[ridx.long()] = vb
        va, vb = va_r, vb_r
    pct = torch.as_tensor(ct[pn], device=dev)
    tot = int(pct.sum())
    Hp = torch.zeros((P, Bs, 2), dtype=torch.float64, device=dev)
    if tot == 0:
        return Hp, wyy_n
    prep = torch.repeat_interleave(torch.arange(P, device=dev), pct)
    off = torch.arange(tot, device=dev) - torch.repeat_interleave(torch.cumsum(pct, 0) - pct, pct)
    pos = torch.as_tensor(st[pn], device=dev)[prep] + off
    rows = ridx[pos].long()
    feat = torch.as_tensor(pf, device=dev)[prep]
    code = bd.codes_col[feat, rows].to(torch.int64) if bd.codes_col is not None else \
        bd.codes[rows, feat].to(torch.int64)
    code = code & 0xFFFF if bd.code_bytes == 2 else code
    a = va[rows].to(torch.float64)
    if mode == 0:
        w = vb[rows].to(torch.float64) if vb is not None else (~torch.isnan(a)).to(torch.float64)
        a = torch.nan_to_num(a) if vb is None else a
        vals = torch.stack([w, w * a], 1)
    else:
        vals = torch.stack([a, vb[rows].to(torch.float64)], 1)
    Hp.view(-1, 2).index_add_(0, prep * Bs + code, vals)
    if wyy_n is not None:
        fp = torch.as_tensor(first, device=dev)[prep]
        nodes = torch.as_tensor(pn, device=dev)[prep]
        wyy_n.index_add_(0, nodes[fp], (vals[:, 1] * a)[fp])
    return Hp, wyy_n


def pair_hist_dev(bd, ridx, va, vb, mode, node_st, node_ct, sel, vmax, posv=False, chunk=_PAIR_CHUNK, fbins=None):
    """pair_hist for a frontier whose pairs are given ON THE DEVICE: sel
    [n, k] global feature ids per node (node-major pairs p = i * k + j), so
    no pair list crosses to the host.  node_st / node_ct: host arrays.  The
    work list is the host's per-node chunk table expanded by k on the device.
    Returns (Hp [n*k, Bs, 2] f64, wyy [n] f64 or None, pfeat [n*k] int32)."""
    dev = ridx.device
    lib = _lib()
    if not getattr(lib, "_typed_pair", False):
        lib.h2o_pair_hist.argtypes = [_c_void, _c_int, _c_ll, _c_void, _c_void, _c_void, _c_void, _c_int,
                                      _c_void, _c_int, _c_int, _c_int, ctypes.c_float, ctypes.c_float, _c_void,
                                      _c_void, _c_void]
        lib._typed_pair = True
    st = np.asarray(node_st, dtype=np.int64)
    ct = np.asarray(node_ct, dtype=np.int64)
    n, k = sel.shape
    P = n * k
    Bs = bd.Bs
    nch = (ct + chunk - 1) // chunk
    rep = np.repeat(np.arange(n), nch)
    c = np.arange(int(nch.sum())) - np.repeat(np.cumsum(nch) - nch, nch)
    tab = np.stack([rep, st[rep] + c * chunk, np.minimum(chunk, ct[rep] - c * chunk), (nch[rep] == 1)], 1)
    multi = np.nonzero((nch > 1) | (ct == 0))[0]
    tab_d = _h2d(np.concatenate([tab.astype(np.int32).reshape(-1), multi.astype(np.int32)]), dev)
    m = len(tab)
    kp = _PAIR_KP if k > 1 else 1
    if kp > 1:
        # groups of up to kp consecutive pairs of one node per workgroup
        ng = -(-k // kp)
        items = tab_d[:4 * m].view(m, 1, 4).expand(m, ng, 4).clone()
        g = torch.arange(ng, dtype=torch.int32, device=dev).view(1, ng)
        items[:, :, 0] = items[:, :, 0] * k + g * kp
        items[:, :, 3] += (g == 0).to(torch.int32) * 2 + torch.clamp(k - g * kp, max=kp) * 256
        n_items = m * ng
    else:
        items = tab_d[:4 * m].view(m, 1, 4).expand(m, k, 4).clone()
        j = torch.arange(k, dtype=torch.int32, device=dev).view(1, k)
        items[:, :, 0] = items[:, :, 0] * k + j
        items[:, :, 3] += (j == 0).to(torch.int32) * 2
        n_items = m * k
    pfeat = sel.to(torch.int32).reshape(-1).contiguous()
    Hp = torch.empty((P, Bs, 2), dtype=torch.float64, device=dev)
    if multi.size:
        Hp.view(n, -1).index_fill_(0, tab_d[4 * m:].long(), 0.0)
    want_wyy = mode == 0
    pwyy = torch.zeros(P, dtype=torch.float64, device=dev) if want_wyy else None
    if m:
        s0, s1 = (fixed_point_scale(v, min(chunk, int(ct.max()))) for v in vmax)
        fn = lib.h2o_pair_hist4 if kp > 1 else lib.h2o_pair_hist
        if kp > 1 and not getattr(lib, "_typed_pair4", False):
            lib.h2o_pair_hist4.argtypes = lib.h2o_pair_hist.argtypes
            lib.h2o_pair_hist4b.argtypes = lib.h2o_pair_hist.argtypes + [_c_void]
            lib._typed_pair4 = True
        args = [_ptr(bd.codes_col), bd.code_bytes, bd.codes_col.stride(0), _ptr(ridx), _ptr(va), _ptr(vb),
                _ptr(items), n_items, _ptr(pfeat), Bs, mode, 1 if posv else 0, s0, s1, _ptr(Hp), _ptr(pwyy),
                _stream()]
        if kp > 1 and fbins is not None:
            # bins past each feature's own codes stay unwritten (see h2o_pair_hist4b)
            rc = lib.h2o_pair_hist4b(*args, _ptr(fbins))
        else:
            rc = fn(*args)
        if rc != 0:
            raise RuntimeError(f"h2o_pair_hist failed: {rc}")
    return Hp, (pwyy.view(n, k)[:, 0].contiguous() if want_wyy else None), pfeat


def gbm_grad(y, f, w, family, out=None, d=None):
    """GBM residual in one HIP pass (gbm_grad_kernel): y - f (gaussian) or
    y - sigmoid(f) (bernoulli), NaN where w == 0 (w may be None).  f32.
    d: pending per-row leaf values of the previous tree (leaf_scatter), added
    into f (in place) by the same pass."""
    mode = {"gaussian": 0, "bernoulli": 1}[family]
    n = y.numel()
    z = out if out is not None else torch.empty(n, dtype=torch.float32, device=y.device)
    if d is not None and (y.device.type != "cuda" or not f.is_contiguous() or f.dtype != torch.float32):
        f.add_(d.view_as(f))
        d = None
    if y.device.type != "cuda":
        p = f if mode == 0 else torch.sigmoid(f)
        v = (y - p).to(torch.float32)
        if w is not None:
            v = torch.where(w > 0, v, torch.full_like(v, float("nan")))
        z.copy_(v)
        return z
    lib = _lib()
    if not getattr(lib, "_typed_grad", False):
        lib.h2o_gbm_grad.argtypes = [_c_void, _c_void, _c_void, _c_int, _c_ll, _c_void, _c_void, _c_void]
        lib._typed_grad = True
    yc, fc = y.contiguous().to(torch.float32), f.contiguous().to(torch.float32)
    wc = w.contiguous().to(torch.float32) if w is not None else None
    rc = lib.h2o_gbm_grad(_ptr(yc), _ptr(fc), _ptr(wc), mode, n, _ptr(z), _ptr(d), _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_gbm_grad failed: {rc}")
    return z


def partition(bd, ridx, ridx_out, feats, masks, starts, counts, use_native=None, chunk=16384, payload=None):
    """Stable-partition each segment i by masks[i][code(row, feats[i])] (1 =
    left).  Writes ridx_out and returns per-segment left counts (host list).
    payload = (pa, pb, pa_out, pb_out): position-ordered float arrays moved
    together with the row ids."""
    dev = ridx.device
    n = len(starts)
    if n == 0:
        return []
    native = dev.type == "cuda" if use_native is None else use_native
    if native:
        lib = _lib()
        items = make_work(starts, counts, range(n), chunk)
        if len(items) == 0:
            return [0] * n
        work = _h2d(items, dev)
        nw = len(items)
        feat_t = _h2d(np.asarray(feats, dtype=np.int32), dev)
        masks = masks.to(torch.uint8).contiguous()
        cnt = torch.empty(nw, dtype=torch.int32, device=dev)
        if bd.codes_col is not None:
            codes, rs, fs = bd.codes_col, 1, bd.nrows_local
        else:
            codes, rs, fs = bd.codes, bd.Fp, 1
        ballot = env("H2O3_PART", "ballot") == "ballot" and (payload is None or payload[1] is None)
        if ballot:
            words = (items[:, 2].astype(np.int64) + 63) // 64
            fb_h = (np.cumsum(words) - words).astype(np.int32)
            fbase = _h2d(fb_h, dev)
            flags = torch.empty(int(words.sum()) + 1, dtype=torch.int64, device=dev)
            rc = lib.h2o_part_flags(_ptr(codes), bd.code_bytes, rs, fs, _ptr(ridx), _ptr(work), _ptr(fbase), nw,
                                    _ptr(feat_t), _ptr(masks), bd.Bs, _ptr(flags), _ptr(cnt), _stream())
        else:
            rc = lib.h2o_part_count(_ptr(codes), bd.code_bytes, rs, fs, _ptr(ridx), _ptr(work), nw, _ptr(feat_t),
                                    _ptr(masks), bd.Bs, _ptr(cnt), _stream())
        if rc != 0:
            raise RuntimeError(f"h2o_part_count failed: {rc}")
        # per-node exclusive scans of the chunk counts (chunks of a node are
        # consecutive in `items`), vectorized on the host
        cnt_h = cnt.cpu().numpy().astype(np.int64)
        slot = items[:, 0].astype(np.int64)
        nleft = np.bincount(slot, weights=cnt_h, minlength=n).astype(np.int64)
        csum = np.cumsum(cnt_h) - cnt_h                       # global exclusive
        first = np.ones(len(items), dtype=bool)
        first[1:] = slot[1:] != slot[:-1]
        first_idx = np.maximum.accumulate(np.where(first, np.arange(len(items)), 0))
        lpre = csum - csum[first_idx]
        st_arr = np.asarray(starts, dtype=np.int64)[slot]
        rpre = (items[:, 1].astype(np.int64) - st_arr) - lpre
        loff = (st_arr + lpre).astype(np.int32)
        roff = (st_arr + nleft[slot] + rpre).astype(np.int32)
        loff_d = _h2d(loff, dev)
        roff_d = _h2d(roff, dev)
        pa, pb, pa_o, pb_o = payload if payload is not None else (None, None, None, None)
        if ballot:
            rc = lib.h2o_part_compact(_ptr(ridx), _ptr(work), _ptr(fbase), nw, _ptr(flags), _ptr(loff_d),
                                      _ptr(roff_d), _ptr(ridx_out), _ptr(pa), _ptr(pa_o), _stream())
            if rc != 0:
                raise RuntimeError(f"h2o_part_compact failed: {rc}")
            return nleft.tolist()
        rc = lib.h2o_part_scatter(_ptr(codes), bd.code_bytes, rs, fs, _ptr(ridx), _ptr(work), nw, _ptr(feat_t),
                                  _ptr(masks), bd.Bs, _ptr(loff_d), _ptr(roff_d), _ptr(ridx_out), _ptr(pa), _ptr(pb),
                                  _ptr(pa_o), _ptr(pb_o), _stream())
        if rc != 0:
            raise RuntimeError(f"h2o_part_scatter failed: {rc}")
        return nleft.tolist()
    out = []
    for i, (st, ct) in enumerate(zip(starts, counts)):
        seg = ridx[st: st + ct]
        if bd.codes_col is not None:
            c = bd.codes_col[feats[i]][seg.long()].to(torch.int64)
        else:
            c = bd.codes[seg.long(), feats[i]].to(torch.int64)
        left = masks[i].to(torch.bool)[c]
        l = seg[left]
        r = seg[~left]
        ridx_out[st: st + l.numel()] = l
        ridx_out[st + l.numel(): st + ct] = r
        if payload is not None:
            pa, pb, pa_o, pb_o = payload
            for src, dst in ((pa, pa_o), (pb, pb_o)):
                v = src[st: st + ct]
                dst[st: st + l.numel()] = v[left]
                dst[st + l.numel(): st + ct] = v[~left]
        out.append(int(l.numel()))
    return out


def _part_chunk(total):
    """Rows per partition work item: 16K at 100M rows (6K+ workgroups); at
    smaller row counts down to 4K so the flag / compaction passes still see
    ~2K workgroups (12.5M rows: 763 -> 2035)."""
    ev = env("H2O3_PART_CHUNK")
    if ev:
        return int(ev)
    return int(max(4096, min(16384, -(-int(total) // 2048 // 64) * 64)))


def iota_i32(out) -> bool:
    """out[:] = 0..n-1 (int32, device) by the 16-byte-store kernel; False when
    it does not apply (the caller then uses torch.arange)."""
    lib = _lib()
    if lib is None or out.dtype != torch.int32 or not out.is_cuda or out.data_ptr() % 16:
        return False
    if not getattr(lib, "_typed_iota", False):
        lib.h2o_iota_i32.argtypes = [_c_void, ctypes.c_longlong, _c_void]
        lib._typed_iota = True
    return lib.h2o_iota_i32(_ptr(out), out.numel(), _stream()) == 0


def partition_async(bd, ridx, ridx_out, feat_d, masks, starts, counts, chunk=None, payload=None, pk=None,
                    pk_col=0):
    """Sync-free ballot partition of EVERY segment i by masks[i][code(row,
    feat_d[i])] (feat_d, masks on device; a segment whose mask is all ones stays
    in place).  The per-chunk left counts are scanned into compaction offsets by
    one device kernel, so the host never waits between the flag and compaction
    passes; returns the per-segment left counts as a DEVICE int64 tensor (and,
    with pk, also writes them as doubles into column pk_col of the [n, stride]
    split record, so they come back with the level's single host transfer).
    payload = (pa, None, pa_out, None)."""
    dev = ridx.device
    n = len(starts)
    lib = _lib()
    if not getattr(lib, "_typed_async", False):
        lib.h2o_part_offsets.argtypes = [_c_void, _c_void, _c_int, _c_int, _c_void, _c_void, _c_void, _c_void,
                                         _c_int, _c_int, _c_void]
        lib._typed_async = True
    if chunk is None:
        chunk = _part_chunk(sum(counts))
    nleft = torch.empty(n, dtype=torch.int64, device=dev)   # zeroed by the offsets kernel
    st = np.asarray(starts, dtype=np.int64).reshape(-1)
    ct = np.asarray(counts, dtype=np.int64).reshape(-1)
    nch = (ct + chunk - 1) // chunk
    nw = int(nch.sum())
    if nw == 0:
        nleft.zero_()
        if pk is not None:
            pk[:, pk_col] = 0.0
        return nleft
    wd = (ct + 63) // 64
    total_words = int(wd.sum())
    buf = torch.empty(13 * nw, dtype=torch.int32, device=dev)
    meta = buf[: 8 * nw].view(torch.int64)
    work = buf[8 * nw: 12 * nw]
    fbase = buf[12 * nw:]
    if chunk % 64 == 0 and env("H2O3_PART_ITEMS", "dev") == "dev":
        # per-chunk records written on the device from the O(frontier) segment table
        if not getattr(lib, "_typed_items", False):
            lib.h2o_part_items.argtypes = [_c_void, _c_int, _c_int, _c_int, _c_void, _c_void, _c_void, _c_void]
            lib._typed_items = True
        seg = _h2d(np.concatenate([st, ct, np.cumsum(nch) - nch, np.cumsum(wd) - wd]), dev)
        rc = lib.h2o_part_items(_ptr(seg), n, chunk, nw, _ptr(work), _ptr(meta), _ptr(fbase), _stream())
        if rc != 0:
            raise RuntimeError(f"h2o_part_items failed: {rc}")
    else:
        items = make_work(starts, counts, range(n), chunk)
        words = (items[:, 2].astype(np.int64) + 63) // 64
        fb_h = (np.cumsum(words) - words).astype(np.int64)
        slot = items[:, 0].astype(np.int64)
        first = np.ones(nw, dtype=bool)
        first[1:] = slot[1:] != slot[:-1]
        first_idx = np.maximum.accumulate(np.where(first, np.arange(nw), 0))
        st_arr = st[slot]
        pos = items[:, 1].astype(np.int64) - st_arr
        # ONE host->device upload: per-chunk meta (int64 x4), the work items and the
        # flag-word bases (int32 views of the same buffer)
        buf.copy_(_h2d(np.concatenate([np.stack([slot, first_idx, st_arr, pos], 0).reshape(-1).view(np.int32),
                                       items.reshape(-1), fb_h.astype(np.int32)]), dev))
    feat_t = feat_d if feat_d.dtype == torch.int32 else feat_d.to(torch.int32)
    masks = masks if masks.dtype == torch.uint8 else masks.to(torch.uint8)
    cnt = torch.empty(nw, dtype=torch.int32, device=dev)
    if bd.codes_col is not None:
        codes, rs, fs = bd.codes_col, 1, bd.nrows_local
    else:
        codes, rs, fs = bd.codes, bd.Fp, 1
    flags = torch.empty(total_words + 1, dtype=torch.int64, device=dev)
    rc = lib.h2o_part_flags(_ptr(codes), bd.code_bytes, rs, fs, _ptr(ridx), _ptr(work), _ptr(fbase), nw,
                            _ptr(feat_t), _ptr(masks), bd.Bs, _ptr(flags), _ptr(cnt), _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_part_flags failed: {rc}")
    loff = torch.empty(nw, dtype=torch.int32, device=dev)
    roff = torch.empty(nw, dtype=torch.int32, device=dev)
    stride = pk.stride(0) if pk is not None else 0
    rc = lib.h2o_part_offsets(_ptr(cnt), _ptr(meta), nw, n, _ptr(loff), _ptr(roff), _ptr(nleft), _ptr(pk),
                              stride, pk_col, _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_part_offsets failed: {rc}")
    pa, _, pa_o, _ = payload if payload is not None else (None, None, None, None)
    rc = lib.h2o_part_compact(_ptr(ridx), _ptr(work), _ptr(fbase), nw, _ptr(flags), _ptr(loff), _ptr(roff),
                              _ptr(ridx_out), _ptr(pa), _ptr(pa_o), _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_part_compact failed: {rc}")
    return nleft


def hist_build_dev(bd, ridx, va, vb, mode, rec, rec_cols, starts, counts, vmax, posv=False, unit_w=False,
                   target_blocks=None):
    """Next-level histograms of the lighter child of every splitting node,
    with the work list built ON THE DEVICE from the level's split record
    (child_work_kernel): launched right after the partition, before the host
    reads the split decisions, so the host's level bookkeeping overlaps GPU
    work.  rec: [n, stride] f64 device record; rec_cols = (ok, nleft, wl, wr)
    column indices.  Returns (Hb [F, n, Bs, C] with pair j in slot j, wyy [n]
    or None, slots [3n] int32 (build | der | par), counts [2] int32 (#pairs,
    #items)) -- capacities n = len(starts) -- or None when the quad kernel does
    not apply (the caller then builds after the host sync as before)."""
    dev = ridx.device
    if dev.type != "cuda" or bd.code_bytes != 1 or bd.Fp % 4 != 0 or bd.Bs > 256 or mode not in (0, 1, 2) or \
            env("H2O3_HIST_KERNEL", "quad") != "quad":
        return None
    lib = _lib()
    if not getattr(lib, "_typed_dev", False):
        lib.h2o_child_work.argtypes = [_c_void, _c_void, _c_void] + [_c_int] * 8 + [_c_void, _c_void, _c_void,
                                                                                  _c_void]
        lib.h2o_hist_quad4.argtypes = [_c_void, _c_int, _c_void, _c_void, _c_void, _c_void, _c_int, _c_int, _c_int,
                                       _c_int, ctypes.c_float, ctypes.c_float, _c_void, _c_int, _c_int, _c_int,
                                       _c_void, _c_int, _c_ll, _c_int, _c_void, _c_void, _c_void]
        lib.h2o_hist_sibling_dev.argtypes = [_c_void, _c_void, _c_void, _c_int, _c_int, _c_int, _c_int, _c_int,
                                             _c_int, _c_int, _c_void, _c_void, _c_void, _c_void, _c_void, _c_void]
        lib._typed_dev = True
    n = len(starts)
    C = channels(mode)
    pack = mode == 0 and unit_w and env("H2O3_HIST_PACK", "1") == "1"
    bm = bm_groups(bd.F, bd.Fp, bd.Bs, pack or mode == 2)
    n_fg, fgw = bm if bm is not None else quad_groups(bd.F, bd.Fp, bd.Bs, pack)
    total = int(sum(counts))
    chunk = hist_chunk((total + 1) // 2, n_fg, target_blocks)   # the lighter children: <= half the rows
    if pack and chunk >= (1 << 23):
        pack = False
        bm = bm_groups(bd.F, bd.Fp, bd.Bs, mode == 2)
        n_fg, fgw = bm if bm is not None else quad_groups(bd.F, bd.Fp, bd.Bs, False)
    cap = n + total // chunk + 1
    stc = np.concatenate([np.asarray(starts, dtype=np.int64), np.asarray(counts, dtype=np.int64)])
    stc_d = _h2d(stc, dev)
    ibuf = torch.empty(4 * cap + 3 * n + 2, dtype=torch.int32, device=dev)
    work, slots, cnts = ibuf[:4 * cap], ibuf[4 * cap:4 * cap + 3 * n], ibuf[4 * cap + 3 * n:]
    ok_c, nl_c, wl_c, wr_c = rec_cols
    rc = lib.h2o_child_work(_ptr(stc_d), _ptr(stc_d[n:]), _ptr(rec), rec.stride(0), ok_c, nl_c, wl_c, wr_c, n, chunk,
                            cap, _ptr(work), _ptr(slots), _ptr(cnts), _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_child_work failed: {rc}")
    nh = bd.F * n * bd.Bs * C
    want_wyy = mode == 0
    buf = torch.zeros(nh + (n if want_wyy else 0), dtype=torch.float64, device=dev)
    Hb = buf[:nh].view(bd.F, n, bd.Bs, C)
    wyy = buf[nh:] if want_wyy else None
    if vmax is None:
        vmax = channel_max(va, vb, mode)
    s0, s1 = (fixed_point_scale(m, chunk) for m in vmax)
    bq = -1
    if pack:
        s1, bq = _pack_scale(vmax[1] if vb is None else max(vmax[1], 0.0), chunk)
    if bm is not None:
        part = bm_part(cap, n_fg, bd.Bs, fgw, pack or mode == 2, dev)
        rc = lib.h2o_hist_bm(_ptr(bd.codes), bd.Fp, _ptr(ridx), _ptr(va), _ptr(vb), _ptr(work), cap, bd.F, 0, bd.Bs,
                             s0, s1, _ptr(Hb), n, mode, _ptr(wyy), 1 if posv else 0, bq, fgw, None, _ptr(cnts),
                             _ptr(part), _stream())
        if rc != 0:
            raise RuntimeError(f"h2o_hist_bm failed: {rc}")
        return Hb, wyy, slots, cnts
    rc = lib.h2o_hist_quad4(_ptr(bd.codes), bd.Fp, _ptr(ridx), _ptr(va), _ptr(vb), _ptr(work), cap, bd.F, 0, bd.Bs,
                            s0, s1, _ptr(Hb), n, mode, 512, _ptr(wyy), 1 if posv else 0, bq, fgw, None, _ptr(cnts),
                            _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_hist_quad4 failed: {rc}")
    return Hb, wyy, slots, cnts


def hist_sibling_dev(Hb, H_prev, slots, cnts, clamp_mask, wyy_b=None, wyy_prev=None):
    """hist_sibling with the device-built pair list of hist_build_dev: output
    capacity 2 * n pairs (n = Hb.shape[1]); the caller slices the first
    2 * #pairs slots once the host knows #pairs."""
    lib = _lib()
    F, nb, Bs, C = Hb.shape
    H = torch.empty((F, 2 * nb, Bs, C), dtype=Hb.dtype, device=Hb.device)
    wyy = torch.empty(2 * nb, dtype=torch.float64, device=Hb.device) if wyy_b is not None else None
    Hp = H_prev.contiguous()
    rc = lib.h2o_hist_sibling_dev(_ptr(Hb), _ptr(Hp), _ptr(slots), nb, Hp.shape[1], 2 * nb, F, Bs * C, C, clamp_mask,
                                  _ptr(H), _ptr(wyy_b), _ptr(wyy_prev), _ptr(wyy), _ptr(cnts), _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_hist_sibling_dev failed: {rc}")
    return H, wyy


def hist_sibling(Hb, H_prev, build_slots, der_slots, par_slots, n_front, clamp_mask, wyy_b=None, wyy_prev=None):
    """Next-level histograms in one kernel: built children copied, siblings =
    parent - built (clamped at 0 on the channels of clamp_mask).  Returns
    (H [F, n_front, Bs, C], wyy [n_front] or None)."""
    lib = _lib()
    if not getattr(lib, "_typed_sib", False):
        lib.h2o_hist_sibling.argtypes = [_c_void, _c_void, _c_void, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                                         _c_int, _c_void, _c_void, _c_void, _c_void, _c_void]
        lib._typed_sib = True
    F, nb, Bs, C = Hb.shape
    H = torch.empty((F, n_front, Bs, C), dtype=Hb.dtype, device=Hb.device)
    slots = _h2d(np.asarray([build_slots, der_slots, par_slots], dtype=np.int32).reshape(-1), Hb.device)
    wyy = torch.empty(n_front, dtype=torch.float64, device=Hb.device) if wyy_b is not None else None
    Hb = Hb.contiguous()
    Hp = H_prev.contiguous()
    rc = lib.h2o_hist_sibling(_ptr(Hb), _ptr(Hp), _ptr(slots), nb, Hp.shape[1], n_front, F, Bs * C, C, clamp_mask,
                              _ptr(H), _ptr(wyy_b), _ptr(wyy_prev), _ptr(wyy), _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_hist_sibling failed: {rc}")
    return H, wyy


def fill_nid(ridx, leaf_ids, starts, counts, nrows, use_native=None):
    """Per-row leaf index from leaf segments."""
    dev = ridx.device
    if dev.type == "cuda" and use_native is None:
        nid = _fill_nid_tiled(ridx, leaf_ids, starts, counts, nrows)
        if nid is not None:
            return nid
    nid = torch.full((nrows,), -1, dtype=torch.int32, device=dev)
    native = dev.type == "cuda" if use_native is None else use_native
    if native:
        lib = _lib()
        items = make_work(starts, counts, leaf_ids, 65536)
        if len(items):
            work = _h2d(items, dev)
            rc = lib.h2o_fill_nid(_ptr(ridx), _ptr(work), len(items), _ptr(nid), _stream())
            if rc != 0:
                raise RuntimeError(f"h2o_fill_nid failed: {rc}")
        return nid
    for lid, st, ct in zip(leaf_ids, starts, counts):
        nid[ridx[st: st + ct].long()] = lid
    return nid


def _fill_nid_tiled(ridx, leaf_ids, starts, counts, nrows):
    """Leaf segments that tile [0, nrows) of the row permutation (every row
    ends in exactly one leaf): position -> segment by one device searchsorted
    over the sorted segment starts, then one scatter through ridx.  Deep DRF
    trees have ~10^5 leaves: this replaces a per-leaf work list (host list
    conversion + one workgroup per tiny segment).  None if the segments do not
    tile the rows."""
    st = np.asarray(starts, dtype=np.int64).reshape(-1)
    ct = np.asarray(counts, dtype=np.int64).reshape(-1)
    lid = np.asarray(leaf_ids, dtype=np.int64).reshape(-1)
    m = ct > 0
    st, ct, lid = st[m], ct[m], lid[m]
    if st.size == 0 or st.size != ct.size:
        return None
    o = np.argsort(st, kind="stable")
    st, ct, lid = st[o], ct[o], lid[o]
    if st[0] != 0 or st[-1] + ct[-1] != nrows or (st.size > 1 and not np.array_equal(st[1:], st[:-1] + ct[:-1])):
        return None
    dev = ridx.device
    bounds = _h2d(st, dev)
    lid_d = _h2d(lid.astype(np.int32), dev)
    pos = torch.arange(nrows, device=dev, dtype=torch.int64)
    seg = torch.searchsorted(bounds, pos, right=True) - 1
    nid = torch.empty(nrows, dtype=torch.int32, device=dev)
    nid[ridx[:nrows].long()] = lid_d[seg]
    return nid


def leaf_pass(ridx, z, w, leaf_ids, starts, counts, n_leaves, nrows, mode, chunk=65536, want_nid=True):
    """Per-leaf gamma sums from the raw residual z (one gather per row; w None
    = unit weights), optionally fused with the nid fill.  Returns (nid, [L, 2] f64)."""
    dev = ridx.device
    lib = _lib()
    if not getattr(lib, "_typed_leaf", False):
        lib.h2o_leaf_pass.argtypes = [_c_void, _c_void, _c_void, _c_void, _c_int, _c_int, _c_void, _c_void, _c_void]
        lib._typed_leaf = True
    out = torch.zeros((n_leaves, 2), dtype=torch.float64, device=dev)
    nid = torch.zeros(nrows, dtype=torch.int32, device=dev) if want_nid else None
    items = make_work(starts, counts, leaf_ids, chunk)
    if len(items) == 0:
        return nid, out
    work = _h2d(items, dev)
    z = z.to(torch.float32).contiguous()
    w = None if w is None else w.to(torch.float32).contiguous()
    rc = lib.h2o_leaf_pass(_ptr(ridx), _ptr(z), _ptr(w), _ptr(work), len(items), int(mode), _ptr(nid), _ptr(out),
                           _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_leaf_pass failed: {rc}")
    return nid, out


def leaf_pos_sums(zpos, leaf_ids, starts, counts, n_leaves, mode, chunk=65536):
    """Per-leaf gamma sums from the position-ordered NaN-masked residual
    payload (contiguous reads).  Returns [L, 2] f64 on device."""
    lib = _lib()
    if not getattr(lib, "_typed_lpos", False):
        lib.h2o_leaf_pos.argtypes = [_c_void, _c_void, _c_int, _c_int, _c_void, _c_void]
        lib.h2o_leaf_update.argtypes = [_c_void, _c_void, _c_int, _c_void, _c_void, _c_void]
        lib._typed_lpos = True
    out = torch.zeros((n_leaves, 2), dtype=torch.float64, device=zpos.device)
    items = make_work(starts, counts, leaf_ids, chunk)
    if len(items):
        work = _h2d(items, zpos.device)
        rc = lib.h2o_leaf_pos(_ptr(zpos), _ptr(work), len(items), int(mode), _ptr(out), _stream())
        if rc != 0:
            raise RuntimeError(f"h2o_leaf_pos failed: {rc}")
    return out


def col_sample(n, elig_d, k, seed):
    """[n, k] int64 per-node feature samples without replacement from the
    eligible global feature ids elig_d (device int64, ascending), each row
    ascending (HIP selection sampling, col_sample_kernel)."""
    dev = elig_d.device
    out = torch.empty((n, k), dtype=torch.int64, device=dev)
    lib = _lib()
    if not getattr(lib, "_typed_csamp", False):
        lib.h2o_col_sample.argtypes = [_c_int, _c_int, _c_void, _c_int, ctypes.c_ulonglong, _c_void, _c_void]
        lib._typed_csamp = True
    rc = lib.h2o_col_sample(int(n), int(elig_d.numel()), _ptr(elig_d), int(k), int(seed) & ((1 << 64) - 1),
                            _ptr(out), _stream())
    if rc != 0:
        raise RuntimeError(f"h2o_col_sample failed: {rc}")
    return out


def leaf_scatter(ridx, d, vals, leaf_ids, starts, counts, chunk=65536):
    """d[ridx[p]] = vals[leaf] over the leaf segments (write-only scatter;
    every row of the tiling is written)."""
    if d.device.type != "cuda":
        for lid, st, ct in zip(leaf_ids, starts, counts):
            d[ridx[st: st + ct].long()] = vals[lid]
        return d
    lib = _lib()
    if not getattr(lib, "_typed_lscat", False):
        lib.h2o_leaf_scatter.argtypes = [_c_void, _c_void, _c_int, _c_void, _c_void, _c_void]
        lib._typed_lscat = True
    items = make_work(starts, counts, leaf_ids, chunk)
    if len(items):
        work = _h2d(items, d.device)
        rc = lib.h2o_leaf_scatter(_ptr(ridx), _ptr(work), len(items), _ptr(vals), _ptr(d), _stream())
        if rc != 0:
            raise RuntimeError(f"h2o_leaf_scatter failed: {rc}")
    return d


def leaf_update(ridx, f, vals, leaf_ids, starts, counts, chunk=65536):
    """f[ridx[p]] += vals[leaf(p)] over the leaf segments (f: contiguous f32)."""
    lib = _lib()
    if not getattr(lib, "_typed_lpos", False):
        lib.h2o_leaf_pos.argtypes = [_c_void, _c_void, _c_int, _c_int, _c_void, _c_void]
        lib.h2o_leaf_update.argtypes = [_c_void, _c_void, _c_int, _c_void, _c_void, _c_void]
        lib._typed_lpos = True
    items = make_work(starts, counts, leaf_ids, chunk)
    if len(items):
        work = _h2d(items, f.device)
        rc = lib.h2o_leaf_update(_ptr(ridx), _ptr(work), len(items), _ptr(vals), _ptr(f), _stream())
        if rc != 0:
            raise RuntimeError(f"h2o_leaf_update failed: {rc}")


def seg_sum2(ridx, a, b, leaf_ids, starts, counts, n_leaves, use_native=None, chunk=65536):
    """Per-leaf sums of a[r] (and b[r]) over leaf segments of ridx -> [L, 2] f64."""
    dev = ridx.device
    out = torch.zeros((n_leaves, 2), dtype=torch.float64, device=dev)
    native = dev.type == "cuda" if use_native is None else use_native
    if native:
        lib = _lib()
        if not getattr(lib, "_typed_seg", False):
            lib.h2o_seg_sum2.argtypes = [_c_void, _c_void, _c_void, _c_void, _c_int, _c_void, _c_void]
            lib._typed_seg = True
        items = make_work(starts, counts, leaf_ids, chunk)
        if len(items) == 0:
            return out
        work = _h2d(items, dev)
        a = a.to(torch.float32).contiguous()
        b = None if b is None else b.to(torch.float32).contiguous()
        rc = lib.h2o_seg_sum2(_ptr(ridx), _ptr(a), _ptr(b), _ptr(work), len(items), _ptr(out), _stream())
        if rc != 0:
            raise RuntimeError(f"h2o_seg_sum2 failed: {rc}")
        return out
    for lid, st, ct in zip(leaf_ids, starts, counts):
        r = ridx[st: st + ct].long()
        out[lid, 0] = a[r].to(torch.float64).sum()
        if b is not None:
            out[lid, 1] = b[r].to(torch.float64).sum()
    return out
