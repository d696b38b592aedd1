// GPU tree engine kernels: per-node feature histograms (LDS-staged), stable
// row partition, per-row leaf assignment and per-leaf segment sums.
//
// Re-design of the reference's ScoreBuildHistogram2 MRTask
// (h2o-algos/src/main/java/hex/tree/ScoreBuildHistogram2.java) and the
// DHistogram accumulation (hex/tree/DHistogram.java:updateHisto): instead of
// one Java histogram object per (node, column) filled chunk-by-chunk, rows are
// kept grouped by tree node (ridx permutation + per-node segments), the
// binned feature matrix is row-major uint8/uint16, and one workgroup
// accumulates a [feature-group x bins x channels] histogram of one node's row
// range in LDS before flushing the non-zero bins to HBM with f64 atomics.
//
// Lane mapping (the CDNA4 part): a wave64 instruction covers FGL features x
// (64/FGL) rows — lane = (row_sub, feature).  All lanes of one row read
// consecutive code bytes of that row (coalesced), the row's gradient pair is
// a broadcast load, and lanes update *different* features' histograms, so
// same-address LDS atomic collisions inside a wave only happen between the
// (64/FGL) rows of one instruction.  (The naive lane=row mapping made all 64
// lanes hit one feature's 256 bins at once and was ~25x slower.)
//
// Channels (MODE):
//   0 : H2O squared-error criterion  (w, w*y)     C = 2   (node sum w*y*y is a
//       separate segment reduction: only the node total enters the split test)
//   1 : second-order (XGBoost)       (g, h)       C = 2
//   2 : weighted count               (w)          C = 1
//
// Histogram layout in HBM: hist[F][n_slots][Bs][C] f64 (feature-major so a
// multi-GPU reduce-scatter can shard by feature).
#include "common.h"
#include <stdlib.h>
#include <algorithm>

template <int MODE> struct Chan { static constexpr int C = MODE == 2 ? 1 : 2; };

// work[i] = (slot, pos_start, pos_count, unused);  grid = (n_work, n_feature_groups)
// PACK (MODE 0, 0/1 weights; the wide-code UniformAdaptive histograms): one
// 64-bit LDS atomic per (row, feature) as in hist_quad_kernel (count in bits
// 63..40, biased fixed-point response below), so a 1025-bin feature takes
// 8.2 KB of LDS instead of 16.4 KB and a workgroup covers twice the features
// -- every feature group re-reads the rows' indices, responses and code
// sectors, which is what the 1024-cell level histograms pay for.
template <typename CodeT, int MODE, bool HAS_VB, bool POSV, bool PACK = false>
__global__ __launch_bounds__(512) void hist_build_kernel(
    const CodeT* __restrict__ codes, int Fp, const int* __restrict__ ridx,
    const float* __restrict__ va, const float* __restrict__ vb,
    const int4* __restrict__ work, int F, int Bs, int FGL, float s0, float s1,
    double* __restrict__ hist, int n_slots, double* __restrict__ wyy_out, const uint8_t* __restrict__ need,
    long long bq = 0) {
  constexpr int C = Chan<MODE>::C;
  constexpr int CL = PACK ? 1 : C;                // u64 LDS words per bin
  const int RPW = 64 / FGL;                     // rows per wave instruction
  extern __shared__ __attribute__((aligned(16))) unsigned long long ldsq[];
  const int4 wk = work[blockIdx.x];
  // need[slot * n_fg + group] == 0: no feature of this group is eligible at
  // this node (DRF mtries / column sampling) -> the histogram stays zero
  if (need != nullptr && need[(size_t)wk.x * gridDim.y + blockIdx.y] == 0) return;
  const int fg0 = blockIdx.y * FGL;
  const int nf = min(FGL, F - fg0);
  const int stride_f = Bs * CL;
  const int total = FGL * stride_f;
  for (int i = threadIdx.x; i < total; i += blockDim.x) ldsq[i] = 0ull;
  __syncthreads();
  const unsigned long long pk_off = (1ull << 40) + (unsigned long long)bq;

  const int lane = threadIdx.x & 63;
  const int fl = lane % FGL;                    // feature within group
  const int rs = lane / FGL;                    // row sub-index
  const bool lane_ok = rs < RPW;                // 64 % FGL lanes idle
  const bool fok = fl < nf && lane_ok;
  const int nwaves = blockDim.x >> 6;
  const int wv = threadIdx.x >> 6;
  unsigned long long* hbase = ldsq + fl * stride_f;
  // node sum of w*y*y (MODE 0): accumulated once per row by the fl==0 lanes of
  // feature group 0, so the SE split test needs no extra pass over the rows
  const bool do_wyy = (MODE == 0) && wyy_out != nullptr && blockIdx.y == 0 && fl == 0 && lane_ok;
  double wyy = 0.0;
  const int pend = wk.y + wk.z;
  const int step = nwaves * RPW;
  // U rows per lane per iteration, every load unconditional (clamped index)
  // so hipcc keeps all gathers in flight instead of branching around each
  // load with a vmcnt(0) (cdna_hip_programming.md §5 "Three .s-level traps" c).
  constexpr int U = 8;
  const int fcl = min(fl, max(nf - 1, 0));
  const CodeT* cbase = codes + fg0 + fcl;
  for (int p0 = wk.y + wv * RPW + (lane_ok ? rs : 0); p0 < pend; p0 += U * step) {
    int rr[U];
    float c0[U], c1[U], yv[U];
    int code[U];
#pragma unroll
    for (int u = 0; u < U; ++u) rr[u] = ridx[min(p0 + u * step, pend - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = rr[u];
      // POSV: the gradient pair is stored in row-permutation (position) order
      // and moved by the partition kernel, so it is read contiguously here
      const int vi = POSV ? min(p0 + u * step, pend - 1) : r;
      if (MODE == 0) {
        const float y = va[vi];
        const float w = HAS_VB ? vb[vi] : 1.f;
        c0[u] = w; c1[u] = w * y;
        yv[u] = y;
      } else if (MODE == 1) {
        c0[u] = va[vi]; c1[u] = vb[vi];
      } else {
        c0[u] = HAS_VB ? vb[vi] : 1.f; c1[u] = 0.f;
      }
      code[u] = (int)cbase[(size_t)r * Fp];
    }
    // Fixed-point accumulation: v * 2^k is exact in f32 (power-of-two scale)
    // and exact as int64, so the LDS sums are exact and order-independent.
    // 64-bit integer LDS atomics run ~5.5x faster than ds_add_f32 on gfx950
    // (scripts/hist_microbench.hip: 1.78 vs 9.83 ms, 10M rows x 100 features).
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool inr = p0 + u * step < pend;
      if (MODE == 0 && do_wyy && inr) wyy += (double)c1[u] * (double)yv[u];
      if (PACK) {
        // 0/1 weights: a row of weight 0 adds nothing
        if (fok && inr && c0[u] != 0.f)
          __hip_atomic_fetch_add(hbase + code[u], pk_off + (unsigned long long)__float2ll_rn(c1[u] * s1),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        continue;
      }
      const bool ok = fok && inr && (c0[u] != 0.f || c1[u] != 0.f);
      if (ok) {
        unsigned long long* h = hbase + code[u] * C;
        __hip_atomic_fetch_add(h, (unsigned long long)__float2ll_rn(c0[u] * s0), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        if (C > 1)
          __hip_atomic_fetch_add(h + 1, (unsigned long long)__float2ll_rn(c1[u] * s1), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  __syncthreads();
  if (MODE == 0 && wyy_out != nullptr && blockIdx.y == 0) {
    wyy = wave_sum(wyy);
    if (lane == 0) gbl_add(wyy_out + wk.x, wyy);
  }
  const double inv0 = 1.0 / (double)s0, inv1 = 1.0 / (double)s1;
  if (PACK) {
    const int tot = nf * Bs;
    for (int i = threadIdx.x; i < tot; i += blockDim.x) {
      const unsigned long long v = ldsq[i];
      if (v != 0) {
        const int j = i / Bs, b = i - (i / Bs) * Bs;
        const long long cnt = (long long)(v >> 40);
        const long long low = (long long)(v & ((1ull << 40) - 1));
        double* o = hist + ((size_t)(fg0 + j) * n_slots + wk.x) * (Bs * 2) + 2 * b;
        gbl_add(o, (double)cnt);
        gbl_add(o + 1, (double)(low - cnt * bq) * inv1);
      }
    }
    return;
  }
  const int tot_real = nf * stride_f;
  for (int i = threadIdx.x; i < tot_real; i += blockDim.x) {
    const long long q = (long long)ldsq[i];
    if (q != 0) {
      const int j = i / stride_f;
      const int rem = i - j * stride_f;
      const double v = (double)q * ((C == 1 || (rem & 1) == 0) ? inv0 : inv1);
      gbl_add(hist + ((size_t)(fg0 + j) * n_slots + wk.x) * stride_f + rem, v);
    }
  }
}

// ---------------------------------------------------------------------------
// Grouped-lane histogram kernel for uint8 codes (rows 8-byte aligned).
// A workgroup owns one group of fgw features (runtime, a multiple of 4*LW,
// at most 64*LW); lane = (row_sub, slot q): each lane loads LW dwords = 4*LW
// consecutive codes of its row and performs 4*LW x C LDS atomics, so a wave
// instruction covers floor(64 / (fgw / 4LW)) rows.  Per-feature LDS regions
// are padded by C entries.  Blocks are ordered (chunk, group) with the group
// fastest and remapped XCD-contiguously, so the group blocks of one row chunk
// run on the same XCD and share its L2 lines for the row gathers.
//
// What bounds it (MI355X, scripts/hist_fsweep_mb.py + scripts/pmc_hist.sh):
// the cost is per group PASS over the rows, not per feature -- F = 100 at
// 4 x 32 lanes took as long as F = 128, and a separate tail launch for
// features 96..99 cost as much as a full pass because it re-reads every
// 128-B code row from HBM.  So the host picks the FEWEST groups that fit the
// LDS budget (F = 100 -> 3 groups of 36 features: 9 lanes per row, 7 rows per
// wave instruction, 63 of 64 lanes busy) in ONE launch.
//
// PACK (MODE 0, weights all 0/1): ONE 64-bit LDS atomic per (row, feature):
// bits 63..40 = row count, bits 39..0 = sum of the biased fixed-point
// response q + Bq (q = rint(y * s1), Bq = rint(vmax * s1) so every term is
// >= 0 and no carry crosses into the count).  Decoded in the flush as
// count and (low - count * Bq) / s1.  Halves the LDS atomics of the
// unweighted GBM / sampled DRF histograms; the response is quantised at
// 1/s1 = chunk * 2 * vmax / 2^40 (f32-level resolution, exact summation).
//
// PIPE: the code/response gathers of iteration i+1 and the row indices of
// iteration i+2 are issued before the atomics of iteration i (PMC on the
// unpipelined loop: SQ_WAIT_ANY = 69% of wave cycles, waves parked on the
// dependent ridx -> codes gathers; pipelined: root 6.8 -> 5.5 ms, depth-3
// level 4.2 -> 2.9 ms at 100M x 100).  Loads use clamped indices, so no
// branch guards them.
// ---------------------------------------------------------------------------
template <int LW> struct CodeW { using T = unsigned int; };
template <> struct CodeW<2> { using T = uint2; };
__device__ __forceinline__ unsigned int code_at(unsigned int w, int hi, int sh) { return (w >> sh) & 0xffu; }
__device__ __forceinline__ unsigned int code_at(uint2 w, int hi, int sh) { return ((hi ? w.y : w.x) >> sh) & 0xffu; }

template <int MODE, bool HAS_VB, bool POSV, bool PACK, bool PIPE = true, int LW = 1>
__global__ __launch_bounds__(1024) void hist_quad_kernel(
    const uint8_t* __restrict__ codes, int Fp, const int* __restrict__ ridx,
    const float* __restrict__ va, const float* __restrict__ vb,
    const int4* __restrict__ work, int n_work, int n_fg, int fgw, int F, int foff, int Bs, float s0, float s1,
    double* __restrict__ hist, int n_slots, double* __restrict__ wyy_out, long long bq,
    const uint8_t* __restrict__ need, const int* __restrict__ n_work_dev) {
  using CT = typename CodeW<LW>::T;
  constexpr int C = Chan<MODE>::C;
  constexpr int CL = PACK ? 1 : C;       // u64 entries per bin in LDS
  constexpr int NK = 4 * LW;             // features per lane
  constexpr int U = 4;                   // rows per lane per iteration
  extern __shared__ __attribute__((aligned(16))) unsigned long long ldsq[];
  // n_work_dev: the work list was built on the device (child_work_kernel) and
  // the grid is an upper bound -- blocks past the real count leave at once.
  // The XCD remap runs over the REAL block count (remapping over the padded
  // grid put every live block on the first XCDs: +20% level time)
  const int nwg = n_work_dev != nullptr ? n_work_dev[1] * n_fg : n_work * n_fg;
  if ((int)blockIdx.x >= nwg) return;
  const int lb = xcd_remap(blockIdx.x, nwg);
  const int fgi = lb % n_fg;
  const int4 wk = work[lb / n_fg];
  if (need != nullptr && need[(size_t)wk.x * n_fg + fgi] == 0) return;   // no eligible feature in this group
  const int fg0 = foff + fgi * fgw;
  const int nf = min(fgw, F - fg0);
  const int LPR = fgw / NK;              // lanes per row
  const int RPW = 64 / LPR;              // rows per wave instruction (64 % LPR lanes idle)
  const int stride_f = Bs * CL + CL;
  const int total = fgw * stride_f;
  for (int i = threadIdx.x; i < total; i += blockDim.x) ldsq[i] = 0ull;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int q = lane % LPR;        // feature slot of the lane
  const int rs = lane / LPR;       // row within the wave instruction
  const bool lane_ok = rs < RPW;
  const int wv = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const bool do_wyy = (MODE == 0) && wyy_out != nullptr && fgi == 0 && q == 0 && lane_ok;
  double wyy = 0.0;
  const int pend = wk.y + wk.z;
  const int step = nwaves * RPW;
  const uint8_t* cbase = codes + fg0 + NK * q;
  unsigned long long* hb[NK];
  bool fk[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    hb[k] = ldsq + (NK * q + k) * stride_f;
    fk[k] = lane_ok && NK * q + k < nf;
  }
  const int p_first = wk.y + wv * RPW + (lane_ok ? rs : 0);
  int rA[U], rB[U];
  CT cwA[U];
  float xaA[U], xbA[U];
  auto load_r = [&](int p, int (&r)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = ridx[min(p + u * step, pend - 1)];
  };
  auto load_v = [&](int p, const int (&r)[U], CT (&cw)[U], float (&xa)[U], float (&xb)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int vi = POSV ? min(p + u * step, pend - 1) : r[u];
      xa[u] = (MODE == 2) ? 0.f : va[vi];
      xb[u] = (HAS_VB || MODE == 1) ? vb[vi] : 1.f;
      cw[u] = *reinterpret_cast<const CT*>(cbase + (size_t)r[u] * Fp);
    }
  };
  if (PIPE) {
    load_r(p_first, rA);
    load_v(p_first, rA, cwA, xaA, xbA);
    load_r(p_first + U * step, rB);
  }
  for (int p0 = p_first; p0 < pend; p0 += U * step) {
    CT cw[U];
    float c0[U], c1[U], yv[U], xa[U], xb[U];
    if (PIPE) {
#pragma unroll
      for (int u = 0; u < U; ++u) { cw[u] = cwA[u]; xa[u] = xaA[u]; xb[u] = xbA[u]; }
      load_v(p0 + U * step, rB, cwA, xaA, xbA);
      load_r(p0 + 2 * U * step, rB);
    } else {
      int rr[U];
      load_r(p0, rr);
      load_v(p0, rr, cw, xa, xb);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (MODE == 0) {
        // without vb a NaN response marks a zero-weight row (out-of-bag /
        // sampled-out): one gather per row instead of two
        const float y = xa[u];
        const float w = HAS_VB ? xb[u] : (y == y ? 1.f : 0.f);
        c0[u] = w; c1[u] = w != 0.f ? w * y : 0.f; yv[u] = w != 0.f ? y : 0.f;
      } else if (MODE == 1) {
        c0[u] = xa[u]; c1[u] = xb[u]; yv[u] = 0.f;
      } else {
        c0[u] = xb[u]; c1[u] = 0.f; yv[u] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool inr = p0 + u * step < pend;
      if (MODE == 0 && do_wyy && inr) wyy += (double)c1[u] * (double)yv[u];
      if (!inr || (c0[u] == 0.f && c1[u] == 0.f)) continue;
      if (PACK) {
        const unsigned long long a = (1ull << 40) + (unsigned long long)(__float2ll_rn(yv[u] * s1) + bq);
#pragma unroll
        for (int k = 0; k < NK; ++k) {
          if (!fk[k]) continue;
          __hip_atomic_fetch_add(hb[k] + code_at(cw[u], k >> 2, 8 * (k & 3)), a, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        continue;
      }
      const unsigned long long a0 = (unsigned long long)__float2ll_rn(c0[u] * s0);
      const unsigned long long a1 = (unsigned long long)__float2ll_rn(c1[u] * s1);
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        if (!fk[k]) continue;
        unsigned long long* h = hb[k] + code_at(cw[u], k >> 2, 8 * (k & 3)) * CL;
        __hip_atomic_fetch_add(h, a0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (C > 1) __hip_atomic_fetch_add(h + 1, a1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  __syncthreads();
  if (MODE == 0 && wyy_out != nullptr && fgi == 0) {
    wyy = wave_sum(wyy);
    if (lane == 0) gbl_add(wyy_out + wk.x, wyy);
  }
  const double inv0 = 1.0 / (double)s0, inv1 = 1.0 / (double)s1;
  const int per_f = Bs * C;
  if (PACK) {
    const int tot = nf * Bs;
    for (int i = threadIdx.x; i < tot; i += blockDim.x) {
      const int j = i / Bs;
      const int b = i - j * Bs;
      const unsigned long long v = ldsq[j * stride_f + b];
      if (v != 0) {
        const long long cnt = (long long)(v >> 40);
        const long long low = (long long)(v & ((1ull << 40) - 1));
        double* o = hist + ((size_t)(fg0 + j) * n_slots + wk.x) * per_f + 2 * b;
        gbl_add(o, (double)cnt);
        gbl_add(o + 1, (double)(low - cnt * bq) * inv1);
      }
    }
    return;
  }
  const int tot_real = nf * per_f;
  for (int i = threadIdx.x; i < tot_real; i += blockDim.x) {
    const int j = i / per_f;
    const int rem = i - j * per_f;
    const long long v = (long long)ldsq[j * stride_f + rem];
    if (v != 0) {
      const double d = (double)v * ((C == 1 || (rem & 1) == 0) ? inv0 : inv1);
      gbl_add(hist + ((size_t)(fg0 + j) * n_slots + wk.x) * per_f + rem, d);
    }
  }
}

struct QuadArgs {
  dim3 grid; int threads; size_t lds; hipStream_t s;
  const uint8_t* cc; int Fp; const int* ridx; const float* va; const float* vb; const int4* wk;
  int n_work, n_fg, fgw, F, foff, Bs; float s0, s1; double* hist; int n_slots; double* wyy; long long bq;
  const uint8_t* need; const int* n_work_dev; unsigned long long* part = nullptr;
};

template <int M, bool V, bool PV, bool PK, bool PIPE = true, int LW = 1>
static void lq(const QuadArgs& a) {
  hipLaunchKernelGGL((hist_quad_kernel<M, V, PV, PK, PIPE, LW>), a.grid, dim3(a.threads), a.lds, a.s, a.cc, a.Fp,
                     a.ridx, a.va, a.vb, a.wk, a.n_work, a.n_fg, a.fgw, a.F, a.foff, a.Bs, a.s0, a.s1, a.hist,
                     a.n_slots, a.wyy, a.bq, a.need, a.n_work_dev);
}

static int env_int(const char* k, int d) {
  const char* v = getenv(k);
  return v ? atoi(v) : d;
}

// A/B switches: H2O3_HIST_PIPE=0 (unpipelined loop), H2O3_HIST_LW=2 (8 codes
// per lane: one dwordx2 gather; measured 0-6% faster on scattered deep levels,
// 5-10% slower at the contiguous root, off by default)
template <int M, bool V, bool PV, bool PK>
static void lq_var(int lw, const QuadArgs& a) {
  static const int pipe = env_int("H2O3_HIST_PIPE", 1);
  if (!pipe) lq<M, V, PV, PK, false>(a);
  else if (lw == 2) lq<M, V, PV, PK, true, 2>(a);
  else lq<M, V, PV, PK>(a);
}

template <int M, bool V>
static void lq_pv(int posv, int pack, int lw, const QuadArgs& a) {
  if (pack) { if (posv) lq_var<M, V, true, true>(lw, a); else lq_var<M, V, false, true>(lw, a); }
  else { if (posv) lq_var<M, V, true, false>(lw, a); else lq_var<M, V, false, false>(lw, a); }
}

// Histograms of features [foff, F) in n_fg = ceil((F - foff) / fgw) groups of
// fgw features (a multiple of 4, at most 64; tree_ops.quad_groups picks it).
// pack_bq >= 0 selects the packed single-atomic path (MODE 0, 0/1 weights).
extern "C" int h2o_hist_quad4(const void* codes, int Fp, const int* ridx, const float* va, const float* vb,
                              const int* work, int n_work, int F, int foff, int Bs, float s0, float s1,
                              double* hist, int n_slots, int mode, int threads, double* wyy, int posv,
                              long long pack_bq, int fgw, const uint8_t* need, const int* n_work_dev,
                              hipStream_t s);
extern "C" int h2o_hist_quad3(const void* codes, int Fp, const int* ridx, const float* va, const float* vb,
                              const int* work, int n_work, int F, int foff, int Bs, float s0, float s1,
                              double* hist, int n_slots, int mode, int threads, double* wyy, int posv,
                              long long pack_bq, int fgw, const uint8_t* need, hipStream_t s) {
  return h2o_hist_quad4(codes, Fp, ridx, va, vb, work, n_work, F, foff, Bs, s0, s1, hist, n_slots, mode, threads,
                        wyy, posv, pack_bq, fgw, need, nullptr, s);
}

// n_work_dev != nullptr: n_work is the CAPACITY of the device-built work list
// (grid upper bound); the real count is n_work_dev[1].
extern "C" int h2o_hist_quad4(const void* codes, int Fp, const int* ridx, const float* va, const float* vb,
                              const int* work, int n_work, int F, int foff, int Bs, float s0, float s1,
                              double* hist, int n_slots, int mode, int threads, double* wyy, int posv,
                              long long pack_bq, int fgw, const uint8_t* need, const int* n_work_dev,
                              hipStream_t s) {
  if (n_work <= 0 || foff >= F) return 0;
  if (Fp % 4 != 0 || foff % 4 != 0 || Bs > 256 || mode < 0 || mode > 2) return -1;
  if (fgw < 4 || fgw > 64 || fgw % 4 != 0) return -2;
  const bool pack = pack_bq >= 0 && mode == 0;
  const int n_fg = (F - foff + fgw - 1) / fgw;
  if (foff + n_fg * fgw > Fp) return -3;       // every code dword read lies inside the row
  static const int lw_env = env_int("H2O3_HIST_LW", 1);
  const int lw = (lw_env == 2 && fgw % 8 == 0 && foff % 8 == 0 && Fp % 8 == 0) ? 2 : 1;
  const int C = mode == 2 ? 1 : 2;
  const int CL = pack ? 1 : C;
  QuadArgs a;
  a.grid = dim3(n_work * n_fg); a.threads = threads;
  a.lds = (size_t)fgw * (Bs * CL + CL) * sizeof(unsigned long long); a.s = s;
  if (a.lds > 160 * 1024) return -4;
  a.cc = (const uint8_t*)codes; a.Fp = Fp; a.ridx = ridx; a.va = va; a.vb = vb; a.wk = (const int4*)work;
  a.n_work = n_work; a.n_fg = n_fg; a.fgw = fgw; a.F = F; a.foff = foff; a.Bs = Bs; a.s0 = s0; a.s1 = s1;
  a.hist = hist; a.n_slots = n_slots; a.wyy = wyy; a.bq = pack_bq; a.need = need; a.n_work_dev = n_work_dev;
  switch (mode) {
    case 0: if (vb) lq_pv<0, true>(posv, pack, lw, a); else lq_pv<0, false>(posv, pack, lw, a); break;
    case 1: lq_pv<1, true>(posv, 0, lw, a); break;
    default: if (vb) lq_pv<2, true>(posv, 0, lw, a); else lq_pv<2, false>(posv, 0, lw, a); break;
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Bank-conflict-free bin-major histogram kernel (uint8 codes, the default).
//
// PMC on hist_quad_kernel (scripts/pmc_gbm.sh, 100M x 100 GBM): 65% of the
// LDS-array cycles were bank-conflict cycles (7.5 extra cycles per
// ds_add_u64) and ~11 VALU instructions ran per LDS atomic (the f32 -> int64
// conversion alone is ~14 instructions, the per-row w*y*y sum in f64 for
// every lane, per-feature exec masks).  With the [feature][bin] layout the
// bank of an atomic is (feature*257 + code) mod 16: random for random codes.
//
// Layout here: [bin][slot] (x channel) u64 -- a bin row of G feature slots
// (PITCH = G * CL u64 = 128..512 B, a multiple of 128 B, so the bank of an
// entry depends on its slot only).  Lane (rs, q) of a wave instruction (LPR =
// G/4 lanes per row, RPW = 64/LPR rows) holds the dword of codes 4q..4q+3 of
// its row; in atomic k it adds byte kk = (k + rs) & 3 into slot kk*LPR + q.
// The 16 lanes of an LDS lane group then hit 16 distinct slots mod 16 (and
// 32 lanes distinct slots mod 32 for G >= 32) whatever the codes are: one
// LDS cycle per group.  The rotation costs nothing (per-lane shift).
//
// Fixed point without the int64 conversion sequence: fma in f64 against a
// 2^52-scale magic constant leaves rint(v * s) (+ bias) in the mantissa bits
// (3 VALU ops: cvt, fma, and/sub).  PACK (MODE 0, 0/1 weights): ONE atomic of
// (count << 40) + biased response, as in hist_quad_kernel.
//
// Flush: a wave reads 4 bins x 16 slots (consecutive LDS words) and adds
// 4 consecutive bins of 16 features to HBM: 64-B contiguous f64 atomics.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long fx_signed(float v, float s) {
  // 2^52 + 2^51: |v*s| < 2^51 lands in the mantissa, two's complement after the subtract
  const double d = __fma_rn((double)v, (double)s, 6755399441055744.0);
  return (unsigned long long)(__double_as_longlong(d) - 0x4338000000000000LL);
}

template <int G, int CL, int MODE, bool HAS_VB, bool POSV, bool PACK, int LW = 2>
__global__ __launch_bounds__(1024) void hist_bm_kernel(
    const uint8_t* __restrict__ codes, int Fp, const int* __restrict__ ridx,
    const float* __restrict__ va, const float* __restrict__ vb,
    const int4* __restrict__ work, int n_work, int n_fg, int F, int foff, int Bs, float s0, float s1,
    double* __restrict__ hist, int n_slots, double* __restrict__ wyy_out, long long bq,
    const uint8_t* __restrict__ need, const int* __restrict__ n_work_dev, unsigned long long* __restrict__ part,
    int dbg) {
  constexpr int C = Chan<MODE>::C;
  constexpr int NK = 4 * LW;              // codes per lane (LW dwords)
  constexpr int LPR = G / NK;             // lanes per row
  constexpr int RPW = 64 / LPR;           // rows per wave instruction
  constexpr int PITCH = G * CL;           // u64 entries per bin row
  constexpr int U = 4;                    // rows per lane per iteration
  constexpr int PD = 2;                   // iterations in the load ring
  using CT = typename CodeW<LW>::T;
  static_assert(CL == 1 || C == 2, "two LDS channels need a two-channel mode");
  static_assert(LPR >= 1, "group narrower than one lane's codes");
  extern __shared__ __attribute__((aligned(16))) unsigned long long ldsq[];
  const int nwg = n_work_dev != nullptr ? n_work_dev[1] * n_fg : n_work * n_fg;
  if ((int)blockIdx.x >= nwg) return;
  const int lb = xcd_remap(blockIdx.x, nwg);
  const int fgi = lb % n_fg;
  int4 wk = work[lb / n_fg];
  // workgroup-uniform: keep the segment in SGPRs (the buffer descriptors below need it there)
  wk.x = __builtin_amdgcn_readfirstlane(wk.x);
  wk.y = __builtin_amdgcn_readfirstlane(wk.y);
  wk.z = __builtin_amdgcn_readfirstlane(wk.z);
  if (need != nullptr && need[(size_t)wk.x * n_fg + fgi] == 0) return;   // no eligible feature in this group
  const int fg0 = foff + fgi * G;
  const int nf = min(G, F - fg0);
  {
    const int n2 = Bs * PITCH / 2;
    ulonglong2* z = reinterpret_cast<ulonglong2*>(ldsq);
    for (int i = threadIdx.x; i < n2; i += blockDim.x) z[i] = make_ulonglong2(0ull, 0ull);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int q = lane % LPR;
  const int rs = lane / LPR;
  const int wv = threadIdx.x >> 6;
  const int nwaves = __builtin_amdgcn_readfirstlane((int)(blockDim.x >> 6));
  // atomic k of a row takes code kk = (k & ~3) | ((k + rs) & 3) of the lane's
  // NK codes (the dword is fixed by k, the byte rotates with the row) into
  // slot kk*LPR + q: the rows of an LDS lane group hit disjoint slots
  unsigned sh[NK], sb[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int kk = (k & ~3) | ((k + rs) & 3);
    sh[k] = 8u * kk;
    sb[k] = (unsigned)((kk * LPR + q) * 8);
  }
  const bool blk_wyy = MODE == 0 && wyy_out != nullptr && fgi == 0;   // workgroup-uniform
  double wyyd = 0.0;
  const int pend = wk.y + wk.z;
  const int step = nwaves * RPW;
  const uint8_t* cbase = codes + fg0 + NK * q;
  const int p_first = wk.y + wv * RPW + rs;
  const unsigned long long pk_off = (1ull << 40) + (unsigned long long)bq;   // count 1 + response bias
  // position-indexed arrays through buffer descriptors sized to [0, pend):
  // loads past the segment return 0 (no clamp), the row offset is one VGPR
  // and the unrolled stride u*step goes into the scalar offset
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)ridx, (short)0, pend * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)va, (short)0, POSV ? pend * 4 : 0,
                                                                      0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)vb, (short)0,
                                                                      (POSV && vb) ? pend * 4 : 0, 0x00020000);
  // Register ring of PD iterations, no copies: stage d of a round processes
  // iteration i from ring slot d, then refills slot d with the gathers of
  // iteration i + PD (row ids loaded a round earlier) and the row ids of
  // iteration i + 2 PD.
  int R[PD][U];
  CT CW[PD][U];
  float XA[PD][U], XB[PD][U];
  auto load_r = [&](int p, int (&r)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = __builtin_amdgcn_raw_buffer_load_b32(rr, p * 4, u * step * 4, 0);
  };
  auto load_v = [&](int p, const int (&r)[U], CT (&cw)[U], float (&xa)[U], float (&xb)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (POSV) {
        xa[u] = (MODE == 2) ? 0.f : __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(ra, p * 4, u * step * 4, 0));
        xb[u] = (HAS_VB || MODE == 1) ? __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, p * 4, u * step * 4, 0))
                                      : 1.f;
      } else {
        xa[u] = (MODE == 2) ? 0.f : va[r[u]];
        xb[u] = (HAS_VB || MODE == 1) ? vb[r[u]] : 1.f;
      }
      cw[u] = *reinterpret_cast<const CT*>(cbase + (size_t)(unsigned)r[u] * (unsigned)Fp);
    }
  };
  const int IT = U * step;                 // positions per iteration (all waves)
#pragma unroll
  for (int d = 0; d < PD; ++d) load_r(p_first + d * IT, R[d]);
#pragma unroll
  for (int d = 0; d < PD; ++d) {
    load_v(p_first + d * IT, R[d], CW[d], XA[d], XB[d]);
    load_r(p_first + (PD + d) * IT, R[d]);
  }
  for (int p0r = p_first; p0r < pend; p0r += PD * IT) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const int p0 = p0r + d * IT;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool inr = p0 + u * step < pend;
        float c0, c1, yv = 0.f;
        if (MODE == 0) {
          // without vb a NaN response marks a zero-weight row (one gather per row)
          const float y = XA[d][u];
          const float w = HAS_VB ? XB[d][u] : (y == y ? 1.f : 0.f);
          c0 = w;
          c1 = w != 0.f ? w * y : 0.f;
          yv = w != 0.f ? y : 0.f;
          // per-row f64 products, like every other histogram kernel (the node
          // total enters the split gains: same rounding -> same trees)
          if (blk_wyy && inr) wyyd += (double)c1 * (double)yv;
        } else if (MODE == 1) {
          c0 = XA[d][u]; c1 = XB[d][u];
        } else {
          c0 = XB[d][u]; c1 = 0.f;
        }
        if (!inr || (c0 == 0.f && c1 == 0.f) || (dbg & 2)) continue;
        unsigned long long a0, a1 = 0ull;
        if (PACK) {
          // weights are 0/1: count 1, response y; the even magic constant of
          // fx_signed rounds ties like __float2ll_rn, the bias is added after
          a0 = fx_signed(yv, s1) + pk_off;
        } else {
          a0 = fx_signed(c0, s0);
          if (CL == 2) a1 = fx_signed(c1, s1);
        }
#pragma unroll
        for (int k = 0; k < NK; ++k) {
          unsigned word;
          if constexpr (LW == 2) word = (k & 4) ? CW[d][u].y : CW[d][u].x;
          else word = CW[d][u];
          const unsigned code = __builtin_amdgcn_ubfe(word, sh[k] & 31u, 8);
          unsigned long long* h = reinterpret_cast<unsigned long long*>(
              reinterpret_cast<char*>(ldsq) + code * (unsigned)(PITCH * 8) + sb[k]);
          __hip_atomic_fetch_add(h, a0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (CL == 2) __hip_atomic_fetch_add(h + G, a1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      load_v(p0 + PD * IT, R[d], CW[d], XA[d], XB[d]);
      load_r(p0 + 2 * PD * IT, R[d]);
    }
  }
  __syncthreads();
  if (blk_wyy) {
    double v = q == 0 ? wyyd : 0.0;      // the LPR lanes of a row saw the same rows
    v = wave_sum(v);
    if (lane == 0) gbl_add(wyy_out + wk.x, v);
  }
  if (part != nullptr) {
    // partial image out with plain coalesced stores; hist_bm_reduce_kernel
    // sums the partials of each node (a float-atomic flush of every entry ran
    // at ~1.3 TB/s of added bytes: 35% of a deep level at 12.5M rows)
    if (dbg & 1) return;
    const int n2 = Bs * PITCH / 2;
    const ulonglong2* src = reinterpret_cast<const ulonglong2*>(ldsq);
    ulonglong2* dst = reinterpret_cast<ulonglong2*>(part + ((size_t)(lb / n_fg) * n_fg + fgi) * (size_t)(Bs * PITCH));
    for (int i2 = threadIdx.x; i2 < n2; i2 += blockDim.x) dst[i2] = src[i2];
    return;
  }
  const double inv0 = 1.0 / (double)s0, inv1 = 1.0 / (double)s1;
  const int si = lane & 15, bi = lane >> 4;
  constexpr int NSG = G / 16;
  const int nbq = (dbg & 1) ? 0 : (Bs + 3) >> 2;
  for (int e = wv; e < nbq * NSG; e += nwaves) {
    const int b = (e / NSG) * 4 + bi;
    const int slot = (e % NSG) * 16 + si;
    const int fl = NK * (slot % LPR) + slot / LPR;
    if (b >= Bs || fl >= nf) continue;
    double* o = hist + ((size_t)(fg0 + fl) * n_slots + wk.x) * (size_t)(Bs * C) + (size_t)b * C;
    const unsigned long long v = ldsq[b * PITCH + slot];
    if (PACK) {
      if (v != 0ull) {
        const long long cnt = (long long)(v >> 40);
        const long long low = (long long)(v & ((1ull << 40) - 1));
        if (dbg & 4) {   // timing probe only: integer (L2) atomics at the same addresses
          unsigned long long* ou = reinterpret_cast<unsigned long long*>(o);
          __hip_atomic_fetch_add(ou, (unsigned long long)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(ou + 1, (unsigned long long)(low - cnt * bq), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        } else {
          gbl_add(o, (double)cnt);
          gbl_add(o + 1, (double)(low - cnt * bq) * inv1);
        }
      }
    } else {
      if (v != 0ull) gbl_add(o, (double)(long long)v * inv0);
      if (CL == 2) {
        const unsigned long long v1 = ldsq[b * PITCH + G + slot];
        if (v1 != 0ull) gbl_add(o + 1, (double)(long long)v1 * inv1);
      }
    }
  }
}

// microbenchmark phase switches (scripts/hist_bm_mb.py): 1 = no flush, 2 = no
// LDS atomics, 4 = flush with integer atomics.  Results are wrong with any
// bit set; 0 in production.
static int g_bm_dbg = 0;
extern "C" void h2o_hist_bm_set_debug(int flags) { g_bm_dbg = flags; }

template <int G, int CL, int M, bool V, bool PV, bool PK, int LW>
static int lbm_u(const QuadArgs& a) {
  auto kern = hist_bm_kernel<G, CL, M, V, PV, PK, LW>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(kern, a.grid, dim3(a.threads), a.lds, a.s, a.cc, a.Fp, a.ridx, a.va, a.vb, a.wk, a.n_work,
                     a.n_fg, a.F, a.foff, a.Bs, a.s0, a.s1, a.hist, a.n_slots, a.wyy, a.bq, a.need, a.n_work_dev,
                     a.part, g_bm_dbg);
  return (int)hipGetLastError();
}

// H2O3_HIST_BM_LW: codes per lane (1 -> 4, 2 -> 8; A/B of the per-row work amortisation)
template <int G, int CL, int M, bool V, bool PV, bool PK>
static int lbm(const QuadArgs& a) {
  static const int lw = env_int("H2O3_HIST_BM_LW", 2);
  // G = 16: 8 rows share a 16-lane group, too many for 4 byte rotations -> 4 codes per lane
  return (lw == 1 || G == 16) ? lbm_u<G, CL, M, V, PV, PK, 1>(a) : lbm_u<G, CL, M, V, PV, PK, 2>(a);
}

template <int G, int CL, int M, bool PK>
static int lbm_v(bool vb, bool posv, const QuadArgs& a) {
  if (M == 1) return posv ? lbm<G, CL, M, true, true, PK>(a) : lbm<G, CL, M, true, false, PK>(a);
  if (vb) return posv ? lbm<G, CL, M, true, true, PK>(a) : lbm<G, CL, M, true, false, PK>(a);
  return posv ? lbm<G, CL, M, false, true, PK>(a) : lbm<G, CL, M, false, false, PK>(a);
}

template <int G>
static int lbm_g(int mode, bool pack, bool vb, bool posv, const QuadArgs& a) {
  if (pack) return lbm_v<G, 1, 0, true>(vb, posv, a);
  if (mode == 2) return lbm_v<G, 1, 2, false>(vb, posv, a);
  if constexpr (G <= 32) {
    if (mode == 0) return lbm_v<G, 2, 0, false>(vb, posv, a);
    return lbm_v<G, 2, 1, false>(vb, posv, a);
  }
  return (int)hipErrorInvalidValue;
}

// Sum of the per-workgroup partial images of hist_bm_kernel by node: block
// (tile, group, item chunk) reads a 16-bin x 16-slot tile of up to BM_RED
// consecutive items' partials (16 x 128-B rows per load, coalesced), sums in
// int64 (exact, like the LDS accumulation) while the items belong to one
// node and adds each node's sums to the f64 histogram (16 features x 16
// consecutive bins per wave-instruction: 256-B contiguous runs).
#define BM_RED 32
__global__ __launch_bounds__(256) void hist_bm_reduce_kernel(
    const unsigned long long* __restrict__ part, const int4* __restrict__ work, int n_work,
    const int* __restrict__ n_work_dev, int n_fg, int F, int foff, int G, int CL, int lpr, int nk, int Bs, int C,
    int pack, long long bq, float s0, float s1, const uint8_t* __restrict__ need, double* __restrict__ hist,
    int n_slots) {
  const int nw = n_work_dev != nullptr ? n_work_dev[1] : n_work;
  const int i0 = blockIdx.z * BM_RED;
  if (i0 >= nw) return;
  const int i1 = min(nw, i0 + BM_RED);
  const int g = blockIdx.y;
  const int PITCH = G * CL;
  const int nbt = (Bs + 15) / 16;   // Bs % 16 may be 4, 8 or 12 (few-bin frames)
  const int b = (blockIdx.x % nbt) * 16 + (threadIdx.x >> 4);
  if (b >= Bs) return;               // no barriers below: idle lanes of a partial tile leave
  const int sl = (blockIdx.x / nbt) * 16 + (threadIdx.x & 15);
  const int ch = sl / G, slot = sl - ch * G;
  const int fg0 = foff + g * G;
  const int fl = nk * (slot % lpr) + slot / lpr;
  const bool live = fl < min(G, F - fg0);
  const double inv0 = 1.0 / (double)s0, inv1 = 1.0 / (double)s1;
  const size_t E = (size_t)Bs * PITCH;
  const size_t eoff = (size_t)b * PITCH + sl;
  long long a0 = 0, a1 = 0;   // PACK: count, response; else: channel value
  int cur = -1;
  auto flush = [&]() {
    if (cur < 0 || !live || (a0 == 0 && a1 == 0)) return;
    double* o = hist + ((size_t)(fg0 + fl) * n_slots + cur) * (size_t)(Bs * C) + (size_t)b * C;
    if (pack) {
      gbl_add(o, (double)a0);
      gbl_add(o + 1, (double)a1 * inv1);
    } else {
      gbl_add(o + ch, (double)a0 * (ch == 0 ? inv0 : inv1));
    }
  };
  for (int i = i0; i < i1; ++i) {
    const int s = work[i].x;
    if (need != nullptr && need[(size_t)s * n_fg + g] == 0) continue;   // the workgroup skipped it
    if (s != cur) {
      flush();
      cur = s; a0 = 0; a1 = 0;
    }
    const unsigned long long v = part[((size_t)i * n_fg + g) * E + eoff];
    if (pack) {
      const long long cnt = (long long)(v >> 40);
      a0 += cnt;
      a1 += (long long)(v & ((1ull << 40) - 1)) - cnt * bq;
    } else {
      a0 += (long long)v;
    }
  }
  flush();
}

// Bin-major conflict-free histograms of features [foff, F) in n_fg = ceil((F -
// foff) / G) groups of G in {16, 32, 64} features (G <= 32 for the two-channel
// modes); every group's code dwords lie inside the row (foff + n_fg*G <= Fp).
// pack_bq >= 0 selects the packed single-atomic path (MODE 0, 0/1 weights).
// n_work_dev != nullptr: device-built work list (n_work = capacity).
// part != nullptr: [n_work][n_fg][Bs][G*CL] u64 scratch for the two-pass
// flush (partial images + hist_bm_reduce_kernel); nullptr: f64 atomic flush.
extern "C" int h2o_hist_bm(const void* codes, int Fp, const int* ridx, const float* va, const float* vb,
                           const int* work, int n_work, int F, int foff, int Bs, float s0, float s1,
                           double* hist, int n_slots, int mode, double* wyy, int posv, long long pack_bq, int G,
                           const uint8_t* need, const int* n_work_dev, unsigned long long* part, hipStream_t s) {
  if (n_work <= 0 || foff >= F) return 0;
  if (Fp % 4 != 0 || foff % 4 != 0 || Bs > 256 || Bs % 4 != 0 || mode < 0 || mode > 2) return -1;
  const bool pack = pack_bq >= 0 && mode == 0;
  const int CL = (pack || mode == 2) ? 1 : 2;
  if (!(G == 16 || G == 32 || G == 64) || (CL == 2 && G == 64)) return -2;
  const int n_fg = (F - foff + G - 1) / G;
  if (foff + n_fg * G > Fp) return -3;       // every code dword read lies inside the row
  QuadArgs a;
  a.grid = dim3(n_work * n_fg); a.threads = 1024;
  a.lds = (size_t)Bs * G * CL * sizeof(unsigned long long); a.s = s;
  if (a.lds > 160 * 1024) return -4;
  a.cc = (const uint8_t*)codes; a.Fp = Fp; a.ridx = ridx; a.va = va; a.vb = vb; a.wk = (const int4*)work;
  a.n_work = n_work; a.n_fg = n_fg; a.fgw = G; a.F = F; a.foff = foff; a.Bs = Bs; a.s0 = s0; a.s1 = s1;
  a.hist = hist; a.n_slots = n_slots; a.wyy = wyy; a.bq = pack_bq; a.need = need; a.n_work_dev = n_work_dev;
  a.part = part;
  const int rc = G == 64 ? lbm_g<64>(mode, pack, vb != nullptr, posv != 0, a)
               : G == 32 ? lbm_g<32>(mode, pack, vb != nullptr, posv != 0, a)
                         : lbm_g<16>(mode, pack, vb != nullptr, posv != 0, a);
  if (rc != 0 || part == nullptr || (g_bm_dbg & 1)) return rc;
  static const int lw_env = env_int("H2O3_HIST_BM_LW", 2);
  const int lw = (lw_env == 1 || G == 16) ? 1 : 2;   // as lbm() picks it
  const int nk = 4 * lw, lpr = G / nk;
  const int C = mode == 2 ? 1 : 2;
  dim3 rg(((Bs + 15) / 16) * (G * CL / 16), n_fg, (n_work + BM_RED - 1) / BM_RED);
  hipLaunchKernelGGL(hist_bm_reduce_kernel, rg, dim3(256), 0, s, part, (const int4*)work, n_work, n_work_dev, n_fg,
                     F, foff, G, CL, lpr, nk, Bs, C, pack ? 1 : 0, pack_bq, s0, s1, need, hist, n_slots);
  return (int)hipGetLastError();
}

template <typename CodeT>
static int launch_hist(const void* codes, int Fp, const int* ridx, const float* va, const float* vb,
                       const int4* work, int n_work, int F, int FG, int Bs, float s0, float s1, double* hist,
                       int n_slots, int mode, int threads, double* wyy, int posv, const uint8_t* need,
                       hipStream_t s, long long pack_bq = -1) {
  const int n_fg = (F + FG - 1) / FG;
  dim3 grid(n_work, n_fg);
  const int C = mode == 2 ? 1 : 2;
  const CodeT* cc = (const CodeT*)codes;
  if (pack_bq >= 0 && mode == 0) {
    const size_t lds = (size_t)FG * Bs * sizeof(unsigned long long);
    if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
#define H2O_PK(V, PV)                                                                                        \
  {                                                                                                          \
    auto kern = hist_build_kernel<CodeT, 0, V, PV, true>;                                                    \
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=      \
        hipSuccess)                                                                                          \
      return (int)hipErrorInvalidValue;                                                                      \
    hipLaunchKernelGGL(kern, grid, dim3(threads), lds, s, cc, Fp, ridx, va, vb, work, F, Bs, FG, s0, s1,     \
                       hist, n_slots, wyy, need, pack_bq);                                                   \
  }
    if (vb) {
      if (posv) H2O_PK(true, true) else H2O_PK(true, false)
    } else {
      if (posv) H2O_PK(false, true) else H2O_PK(false, false)
    }
#undef H2O_PK
    return (int)hipGetLastError();
  }
  size_t lds = (size_t)FG * Bs * C * sizeof(unsigned long long);
  switch (mode) {
#define H2O_LH(M, V) if (posv) H2O_LH2(M, V, true); else H2O_LH2(M, V, false)
#define H2O_LH2(M, V, PV) hipLaunchKernelGGL((hist_build_kernel<CodeT, M, V, PV>), grid, dim3(threads), lds, s, cc, Fp, ridx, va, vb, work, F, Bs, FG, s0, s1, hist, n_slots, wyy, need)
    case 0: if (vb) H2O_LH(0, true); else H2O_LH(0, false); break;
    case 1: H2O_LH(1, true); break;
    default: if (vb) H2O_LH(2, true); else H2O_LH(2, false); break;
#undef H2O_LH
#undef H2O_LH2
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Stable partition of each splitting node's row segment into [left | right].
// A split is a per-node "go-left" mask over all Bs bin codes (NA code
// included), so numeric thresholds, NA direction and categorical bitsets
// (hex/tree/DTree.java Split + IcedBitSet) are one lookup.
//
// work[i] = (slot, pos_start, pos_count, chunk_id); chunks of one node are in
// position order.  Pass 1 counts lefts per chunk; the host scans the counts
// per node; pass 2 scatters each chunk stably.
// code of (row r, feature f) = codes[r*rs + f*fs]  (row- or column-major)
template <typename CodeT>
__device__ __forceinline__ void load_items(const CodeT* __restrict__ codes, long long rs, long long fs, int f,
                                           const int* __restrict__ ridx, int p0, int end, int (&r)[16],
                                           int (&c)[16]) {
  // 16 consecutive positions per thread; all loads unconditional (clamped)
  if (p0 + 16 <= end && (p0 & 3) == 0) {
    const int4* v = reinterpret_cast<const int4*>(ridx + p0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int4 x = v[q];
      r[4 * q] = x.x; r[4 * q + 1] = x.y; r[4 * q + 2] = x.z; r[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = ridx[min(p0 + k, end - 1)];
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) c[k] = (int)codes[(size_t)r[k] * rs + (size_t)f * fs];
}

template <typename CodeT>
__global__ __launch_bounds__(256) void part_count_kernel(
    const CodeT* __restrict__ codes, long long rs, long long fs, const int* __restrict__ ridx,
    const int4* __restrict__ work, const int* __restrict__ feat, const uint8_t* __restrict__ masks,
    int Bs, int* __restrict__ cnt) {
  __shared__ uint8_t m[4096];
  __shared__ int red[4];
  const int4 wk = work[blockIdx.x];
  const int f = feat[wk.x];
  for (int i = threadIdx.x; i < Bs; i += blockDim.x) m[i] = masks[(size_t)wk.x * Bs + i];
  __syncthreads();
  const int end = wk.y + wk.z;
  int local = 0;
  for (int base = wk.y; base < end; base += 256 * 16) {
    const int p0 = base + threadIdx.x * 16;
    if (p0 >= end) continue;
    int r[16], c[16];
    load_items<CodeT>(codes, rs, fs, f, ridx, p0, end, r, c);
#pragma unroll
    for (int k = 0; k < 16; ++k) local += (p0 + k < end && m[c[k]]) ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) local += __shfl_xor(local, o, 64);
  if (lane_id() == 0) red[wave_id()] = local;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// loff[i], roff[i]: destination start of chunk i's left / right rows.
template <typename CodeT>
__global__ __launch_bounds__(256) void part_scatter_kernel(
    const CodeT* __restrict__ codes, long long rs, long long fs, const int* __restrict__ ridx,
    const int4* __restrict__ work, const int* __restrict__ feat, const uint8_t* __restrict__ masks,
    int Bs, const int* __restrict__ loff, const int* __restrict__ roff, int* __restrict__ out,
    const float* __restrict__ pa, const float* __restrict__ pb, float* __restrict__ pa_out,
    float* __restrict__ pb_out) {
  __shared__ uint8_t m[4096];
  __shared__ int wsum[4];
  const int4 wk = work[blockIdx.x];
  const int f = feat[wk.x];
  for (int i = threadIdx.x; i < Bs; i += blockDim.x) m[i] = masks[(size_t)wk.x * Bs + i];
  __syncthreads();
  int lbase = loff[blockIdx.x], rbase = roff[blockIdx.x];
  const int end = wk.y + wk.z;
  const int lane = lane_id(), wv = wave_id();
  for (int base = wk.y; base < end; base += 256 * 16) {
    const int p0 = base + threadIdx.x * 16;
    int r[16], c[16];
    unsigned bits = 0;
    int nl = 0, nv = 0;
    if (p0 < end) {
      load_items<CodeT>(codes, rs, fs, f, ridx, p0, end, r, c);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const bool v = p0 + k < end;
        const bool L = v && m[c[k]];
        bits |= (L ? 1u : 0u) << k;
        nl += L ? 1 : 0;
        nv += v ? 1 : 0;
      }
    }
    // block exclusive scan of nl (positions are in thread order)
    int incl = nl;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int u = __shfl_up(incl, d, 64);
      if (lane >= d) incl += u;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int wpre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int s = wsum[w];
      wpre += (w < wv) ? s : 0;
      tot += s;
    }
    const int lpre = wpre + incl - nl;                 // lefts before this thread in the tile
    const int tile_first = base;
    const int pos_before = max(0, min(p0, end) - tile_first);  // valid positions before this thread
    int li = lbase + lpre;
    int ri = rbase + (pos_before - lpre);
    if (p0 < end) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (p0 + k < end) {
          // row payload (position-ordered gradient pair) moves with the row id
          const int dst = ((bits >> k) & 1u) ? li++ : ri++;
          out[dst] = r[k];
          if (pa) { pa_out[dst] = pa[p0 + k]; pb_out[dst] = pb[p0 + k]; }
        }
      }
    }
    const int tile_n = min(256 * 16, end - base);
    lbase += tot;
    rbase += tile_n - tot;
    __syncthreads();
  }
}
// ---------------------------------------------------------------------------
// Ballot partition (v2).  Pass 1 (flags): positions are walked in 256-wide
// coalesced strides; each wave ballots its 64 go-left bits, stores them as
// one u64 (flags[fbase + (p - start) / 64]) and the block counts lefts.
// Pass 2 (compact): re-reads ridx coalesced + the flag words (no second
// random code gather), ranks every position with popc over the ballot and
// the running per-wave / per-block prefix, so each wave's lefts (rights)
// land in ONE contiguous run -> coalesced stores, stable order.
// ---------------------------------------------------------------------------
template <typename CodeT>
__global__ __launch_bounds__(256) void part_flags_kernel(
    const CodeT* __restrict__ codes, long long rs, long long fs, const int* __restrict__ ridx,
    const int4* __restrict__ work, const int* __restrict__ fbase, const int* __restrict__ feat,
    const uint8_t* __restrict__ masks, int Bs, unsigned long long* __restrict__ flags, int* __restrict__ cnt,
    const int* __restrict__ nw_dev) {
  __shared__ uint8_t m[4096];
  __shared__ int red[4];
  if (nw_dev != nullptr && (int)blockIdx.x >= nw_dev[1]) return;   // device-built work list: grid = capacity
  const int4 wk = work[blockIdx.x];
  const int f = feat[wk.x];
  for (int i = threadIdx.x; i < Bs; i += blockDim.x) m[i] = masks[(size_t)wk.x * Bs + i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int end = wk.y + wk.z;
  const int fb = fbase[blockIdx.x];
  int local = 0;
  constexpr int U = 8;   // 8 strides of 256 positions in flight per thread
  for (int base = wk.y; base < end; base += 256 * U) {
    int r[U], c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = ridx[min(base + u * 256 + (int)threadIdx.x, end - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = (int)codes[(size_t)r[u] * rs + (size_t)f * fs];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = base + u * 256 + (int)threadIdx.x;
      const bool L = p < end && m[c[u]];
      const unsigned long long bal = __ballot(L);
      const int w0 = base + u * 256 + wv * 64;        // first position of this wave's 64
      if (lane == 0 && w0 < end) flags[fb + (w0 - wk.y) / 64] = bal;
      local += L ? 1 : 0;
    }
  }
  local = (int)wave_sum((float)local);
  if (lane == 0) red[wv] = local;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Compaction: each thread moves U positions per iteration (U strides of 256
// positions): the row ids, payloads and flag words of all U strides are
// loaded up front, ONE barrier publishes the U x 4 per-wave left / right
// counts, and every stride's destinations follow from the running prefix (the
// one-stride loop waited on two barriers per 256 positions: 0.11 ms per level
// at 12.5M rows, 4x the bytes it moves).
template <int U>
__global__ __launch_bounds__(256) void part_compact_kernel(
    const int* __restrict__ ridx, const int4* __restrict__ work, const int* __restrict__ fbase,
    const unsigned long long* __restrict__ flags, const int* __restrict__ loff, const int* __restrict__ roff,
    int* __restrict__ out, const float* __restrict__ pa, float* __restrict__ pa_out, const int* __restrict__ nw_dev) {
  __shared__ int wl[U][4], wr_[U][4];
  if (nw_dev != nullptr && (int)blockIdx.x >= nw_dev[1]) return;
  const int4 wk = work[blockIdx.x];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int end = wk.y + wk.z;
  const int fb = fbase[blockIdx.x];
  int lbase = loff[blockIdx.x], rbase = roff[blockIdx.x];
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int base = wk.y; base < end; base += 256 * U) {
    int r[U];
    float a[U];
    unsigned long long bal[U], valid[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = base + u * 256 + (int)threadIdx.x;
      const int pc = min(p, end - 1);
      r[u] = ridx[pc];
      a[u] = pa ? pa[pc] : 0.f;
      const int w0 = base + u * 256 + wv * 64;
      bal[u] = (w0 < end) ? flags[fb + (w0 - wk.y) / 64] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      valid[u] = __ballot(base + u * 256 + (int)threadIdx.x < end);
      const int nl_w = __popcll(bal[u] & valid[u]);
      if (lane == 0) { wl[u][wv] = nl_w; wr_[u][wv] = __popcll(valid[u]) - nl_w; }
    }
    __syncthreads();
    int lrun = 0, rrun = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int lpre = lrun, rpre = rrun;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        lpre += (w < wv) ? wl[u][w] : 0;
        rpre += (w < wv) ? wr_[u][w] : 0;
        lrun += wl[u][w];
        rrun += wr_[u][w];
      }
      if ((valid[u] >> lane) & 1ull) {
        const bool L = (bal[u] >> lane) & 1ull;
        const int dst = L ? (lbase + lpre + __popcll(bal[u] & valid[u] & below))
                          : (rbase + rpre + __popcll(~bal[u] & valid[u] & below));
        out[dst] = r[u];
        if (pa) pa_out[dst] = a[u];
      }
    }
    lbase += lrun;
    rbase += rrun;
    __syncthreads();
  }
}


// Histogram subtraction for the next level: built children are copied, their
// siblings are parent - built.  slots = [build_slot[nb], der_slot[nb],
// par_slot[nb]] (int32).  Channels whose bit is set in clamp_mask are clamped at
// 0 (weights, counts); the others (w*y, gradients) may be negative.  One block
// per (feature, pair), threads over the Bs*C values; wyy (per-node sum w*y*y)
// follows the same rule (block (0, pair) writes it).
__global__ __launch_bounds__(256) void hist_sibling_kernel(const double* __restrict__ Hb,
                                                           const double* __restrict__ Hp,
                                                           const int* __restrict__ slots, int nb, int np, int nf,
                                                           int BsC, int C, int clamp_mask,
                                                           double* __restrict__ H, const double* __restrict__ wyy_b,
                                                           const double* __restrict__ wyy_p,
                                                           double* __restrict__ wyy_out,
                                                           const int* __restrict__ nb_dev) {
  const int j = blockIdx.x;          // pair
  if (nb_dev != nullptr && j >= nb_dev[0]) return;   // device-built pair list: grid is an upper bound
  const int f = blockIdx.y;          // feature
  const int bs = slots[j], ds = slots[nb + j], ps = slots[2 * nb + j];
  const double* hb = Hb + ((size_t)f * nb + j) * BsC;
  const double* hp = Hp + ((size_t)f * np + ps) * BsC;
  double* ob = H + ((size_t)f * nf + bs) * BsC;
  double* od = H + ((size_t)f * nf + ds) * BsC;
  for (int i = threadIdx.x; i < BsC; i += blockDim.x) {
    const double b = hb[i];
    double d = hp[i] - b;
    if ((clamp_mask >> (i % C)) & 1) d = fmax(d, 0.0);
    ob[i] = b;
    od[i] = d;
  }
  if (wyy_b != nullptr && f == 0 && threadIdx.x == 0) {
    wyy_out[bs] = wyy_b[j];
    wyy_out[ds] = wyy_p[ps] - wyy_b[j];
  }
}

// Compaction offsets of the sync-free partition, one workgroup: per chunk i of
// node s = meta[0][i] (chunks of a node are consecutive), lpre = left rows of
// the node's earlier chunks; loff = start + lpre, roff = start + nleft[s] +
// (pos - lpre).  Writes nleft (double) into pk[s * stride + col].
__global__ __launch_bounds__(1024) void part_offsets_kernel(const int* __restrict__ cnt,
                                                            const long long* __restrict__ meta, int nw, int n,
                                                            int* __restrict__ loff, int* __restrict__ roff,
                                                            long long* __restrict__ nleft, double* __restrict__ pk,
                                                            int stride, int col) {
  __shared__ long long carry;
  const long long* slot = meta;
  const long long* first = meta + nw;
  const long long* st = meta + 2 * (long long)nw;
  const long long* pos = meta + 3 * (long long)nw;
  for (int s = threadIdx.x; s < n; s += blockDim.x) nleft[s] = 0;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  // pass 2: global exclusive scan of cnt, 1024 chunks per tile: inclusive
  // scan inside each wave by shuffles, wave totals scanned by wave 0 -- two
  // barriers per tile (the Hillis-Steele LDS scan took 20; 113 us -> ~10 us
  // per level at 6k chunks)
  __shared__ long long wtot[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  for (int base = 0; base < nw; base += blockDim.x) {
    const int i = base + threadIdx.x;
    const long long v = i < nw ? (long long)cnt[i] : 0;
    long long x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long t = __shfl_up(x, o, 64);
      if (lane >= o) x += t;
    }
    if (lane == 63) wtot[wv] = x;
    __syncthreads();
    if (wv == 0) {
      long long w = lane < nwv ? wtot[lane] : 0;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const long long t = __shfl_up(w, o, 64);
        if (lane >= o) w += t;
      }
      if (lane < nwv) wtot[lane] = w;   // inclusive prefix of wave totals
    }
    __syncthreads();
    const long long before = (wv > 0 ? wtot[wv - 1] : 0) + carry;
    if (i < nw) loff[i] = (int)(before + x - v);   // global exclusive prefix, rebased per node below
    __syncthreads();
    if (threadIdx.x == 0) carry += wtot[nwv - 1];
    __syncthreads();
  }
  __syncthreads();
  // node totals from the scan (chunks of a node are consecutive): the node's
  // last chunk holds prefix_end - prefix_start -- no same-address atomics
  for (int i = threadIdx.x; i < nw; i += blockDim.x)
    if (i == nw - 1 || first[i + 1] != first[i])
      nleft[slot[i]] = (long long)loff[i] + cnt[i] - (long long)loff[first[i]];
  for (int i = threadIdx.x; i < nw; i += blockDim.x) roff[i] = loff[first[i]];   // node's first-chunk prefix
  __syncthreads();
  for (int i = threadIdx.x; i < nw; i += blockDim.x) {
    const long long lpre = (long long)loff[i] - (long long)roff[i];
    const long long s = slot[i];
    loff[i] = (int)(st[i] + lpre);
    roff[i] = (int)(st[i] + nleft[s] + pos[i] - lpre);
  }
  __syncthreads();
  if (pk != nullptr)
    for (int s = threadIdx.x; s < n; s += blockDim.x) pk[(size_t)s * stride + col] = (double)nleft[s];
}


// Leaf gamma sums from the POSITION-ordered NaN-masked residual payload the
// partition already moved with the rows (contiguous reads, no row gather);
// NaN = zero-weight row.  mode 0: (sum z, count), mode 1 (bernoulli): (sum z,
// sum |z|(1-|z|)).  work[i] = (leaf, start, count, -).
__global__ __launch_bounds__(256) void leaf_pos_kernel(const float* __restrict__ zp, const int4* __restrict__ work,
                                                       int mode, double* __restrict__ out,
                                                       const int* __restrict__ nw_dev) {
  if (nw_dev != nullptr && (int)blockIdx.x >= nw_dev[1]) return;
  const int4 wk = work[blockIdx.x];
  double sa = 0.0, sb = 0.0;
  const int end = wk.y + wk.z;
  for (int p = wk.y + threadIdx.x; p < end; p += 256) {
    const float z = zp[p];
    if (z == z) {
      sa += (double)z;
      if (mode == 1) {
        const double az = fabs((double)z);
        sb += az * (1.0 - az);
      } else {
        sb += 1.0;
      }
    }
  }
  sa = wave_sum(sa);
  sb = wave_sum(sb);
  __shared__ double red[2][4];
  if (lane_id() == 0) { red[0][wave_id()] = sa; red[1][wave_id()] = sb; }
  __syncthreads();
  if (threadIdx.x == 0) {
    gbl_add(out + 2 * wk.x, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    gbl_add(out + 2 * wk.x + 1, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

// f[ridx[p]] += val[leaf] over the leaf segments: the prediction update without
// materialising per-row leaf ids.
__global__ __launch_bounds__(256) void leaf_update_kernel(const int* __restrict__ ridx, const int4* __restrict__ work,
                                                          const float* __restrict__ val, float* __restrict__ f) {
  const int4 wk = work[blockIdx.x];
  const float v = val[wk.x];
  for (int p = wk.y + threadIdx.x; p < wk.y + wk.z; p += 256) f[ridx[p]] += v;
}

// d[ridx[p]] = val[leaf] over the leaf segments: a write-only scatter of the
// per-row leaf value (no read of f), folded into f by the next tree's
// residual pass (gbm_grad_kernel with d) or an explicit contiguous add.
__global__ __launch_bounds__(256) void leaf_scatter_kernel(const int* __restrict__ ridx, const int4* __restrict__ work,
                                                           const float* __restrict__ val, float* __restrict__ d,
                                                           const int* __restrict__ nw_dev) {
  if (nw_dev != nullptr && (int)blockIdx.x >= nw_dev[1]) return;
  const int4 wk = work[blockIdx.x];
  const float v = val[wk.x];
  const int end = wk.y + wk.z;
  // 4 row ids loaded before the 4 random stores: more scatter writes in
  // flight per thread than the load -> store -> load chain
  int p = wk.y + threadIdx.x;
  for (; p + 3 * 256 < end; p += 4 * 256) {
    const int r0 = ridx[p], r1 = ridx[p + 256], r2 = ridx[p + 512], r3 = ridx[p + 768];
    d[r0] = v; d[r1] = v; d[r2] = v; d[r3] = v;
  }
  for (; p < end; p += 256) d[ridx[p]] = v;
}

// Per-node column sampling without replacement (DRF mtries, GBM
// col_sample_rate): one thread per node runs selection sampling (Knuth's
// algorithm S) over the m eligible features -- feature j is taken with
// probability (k - taken) / (m - j) -- so the k ids come out already in
// ascending order, with no random-key sort / top-k (which cost ~8 launches
// and a host sync per tree level).  Uniforms from a splitmix64 hash of
// (seed, node, j): deterministic for a seed.
__device__ __forceinline__ unsigned long long smix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void col_sample_kernel(int n, int m, const long long* __restrict__ elig, int k,
                                                         unsigned long long seed, long long* __restrict__ out) {
  const int node = blockIdx.x * blockDim.x + threadIdx.x;
  if (node >= n) return;
  const unsigned long long base = smix64(seed ^ ((unsigned long long)node * 0xD1B54A32D192ED03ull));
  long long* o = out + (size_t)node * k;
  int taken = 0;
  for (int j = 0; j < m && taken < k; ++j) {
    const double u = (double)(smix64(base + (unsigned long long)j) >> 11) * (1.0 / 9007199254740992.0);
    if (u * (double)(m - j) < (double)(k - taken)) o[taken++] = elig[j];
  }
}

// nid[ridx[p]] = leaf for p in segment.  work[i] = (leaf_id, start, count, -)
__global__ __launch_bounds__(256) void fill_nid_kernel(const int* __restrict__ ridx, const int4* __restrict__ work,
                                                       int* __restrict__ nid) {
  const int4 wk = work[blockIdx.x];
  for (int p = wk.y + threadIdx.x; p < wk.y + wk.z; p += blockDim.x) nid[ridx[p]] = wk.x;
}

// ridx = 0, 1, ..., n-1 with 16-byte stores (the root of every tree; a torch
// arange runs the indexed elementwise kernel at ~2.4 TB/s of writes)
__global__ __launch_bounds__(256) void iota_i32_kernel(int* __restrict__ out, long long n) {
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int b = (int)(4 * i);
    reinterpret_cast<int4*>(out)[i] = make_int4(b, b + 1, b + 2, b + 3);
  }
  for (long long i = 4 * n4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (int)i;
}

extern "C" {

int h2o_iota_i32(int* out, long long n, hipStream_t s) {
  if (n <= 0) return 0;
  if (((uintptr_t)out & 15) != 0) return -1;
  const long long blocks = std::min<long long>((n / 4 + 255) / 256 + 1, 4096);
  hipLaunchKernelGGL(iota_i32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, out, n);
  return (int)hipGetLastError();
}

int h2o_hist_build(const void* codes, int code_bytes, int Fp, const int* ridx, const float* va,
                   const float* vb, const int* work, int n_work, int F, int FG, int Bs, float s0, float s1,
                   double* hist, int n_slots, int mode, int threads, double* wyy, int posv, const uint8_t* need,
                   hipStream_t s) {
  if (n_work <= 0) return 0;
  if (code_bytes == 1)
    return launch_hist<uint8_t>(codes, Fp, ridx, va, vb, (const int4*)work, n_work, F, FG, Bs, s0, s1, hist, n_slots, mode, threads, wyy, posv, need, s);
  return launch_hist<uint16_t>(codes, Fp, ridx, va, vb, (const int4*)work, n_work, F, FG, Bs, s0, s1, hist, n_slots, mode, threads, wyy, posv, need, s);
}

// Packed single-atomic histogram (MODE 0, 0/1 weights), any code width.
int h2o_hist_build_pk(const void* codes, int code_bytes, int Fp, const int* ridx, const float* va,
                      const float* vb, const int* work, int n_work, int F, int FG, int Bs, float s1, long long bq,
                      double* hist, int n_slots, int threads, double* wyy, int posv, const uint8_t* need,
                      hipStream_t s) {
  if (n_work <= 0) return 0;
  if (bq < 0) return (int)hipErrorInvalidValue;
  if (code_bytes == 1)
    return launch_hist<uint8_t>(codes, Fp, ridx, va, vb, (const int4*)work, n_work, F, FG, Bs, 1.f, s1, hist, n_slots,
                                0, threads, wyy, posv, need, s, bq);
  return launch_hist<uint16_t>(codes, Fp, ridx, va, vb, (const int4*)work, n_work, F, FG, Bs, 1.f, s1, hist, n_slots,
                               0, threads, wyy, posv, need, s, bq);
}

int h2o_part_flags(const void* codes, int code_bytes, long long rs, long long fs, const int* ridx,
                   const int* work, const int* fbase, int n_work, const int* feat, const uint8_t* masks, int Bs,
                   unsigned long long* flags, int* cnt, hipStream_t s) {
  if (n_work <= 0) return 0;
  if (code_bytes == 1)
    hipLaunchKernelGGL(part_flags_kernel<uint8_t>, dim3(n_work), dim3(256), 0, s, (const uint8_t*)codes, rs, fs,
                       ridx, (const int4*)work, fbase, feat, masks, Bs, flags, cnt, nullptr);
  else
    hipLaunchKernelGGL(part_flags_kernel<uint16_t>, dim3(n_work), dim3(256), 0, s, (const uint16_t*)codes, rs, fs,
                       ridx, (const int4*)work, fbase, feat, masks, Bs, flags, cnt, nullptr);
  return (int)hipGetLastError();
}

int h2o_hist_sibling(const double* Hb, const double* Hp, const int* slots, int nb, int np, int nf, int F, int BsC,
                     int C, int clamp_mask, double* H, const double* wyy_b, const double* wyy_p, double* wyy_out,
                     hipStream_t s) {
  if (nb <= 0 || F <= 0) return 0;
  hipLaunchKernelGGL(hist_sibling_kernel, dim3(nb, F), dim3(256), 0, s, Hb, Hp, slots, nb, np, nf, BsC, C, clamp_mask,
                     H, wyy_b, wyy_p, wyy_out, nullptr);
  return (int)hipGetLastError();
}

// Same with the pair count read on the device (counts[0]); nb = capacity.
int h2o_hist_sibling_dev(const double* Hb, const double* Hp, const int* slots, int nb, int np, int nf, int F,
                         int BsC, int C, int clamp_mask, double* H, const double* wyy_b, const double* wyy_p,
                         double* wyy_out, const int* counts, hipStream_t s) {
  if (nb <= 0 || F <= 0) return 0;
  hipLaunchKernelGGL(hist_sibling_kernel, dim3(nb, F), dim3(256), 0, s, Hb, Hp, slots, nb, np, nf, BsC, C, clamp_mask,
                     H, wyy_b, wyy_p, wyy_out, counts);
  return (int)hipGetLastError();
}

// Next-level histogram work built on the device right after a level's
// partition, so the level's histograms start before the host has read the
// split decisions (the host bookkeeping then overlaps GPU work).  One
// workgroup.  For frontier node i (segment st[i], ct[i]) that splits
// (rec[i*stride + ok_col] > 0) with nleft = rec[..nl_col]: pair j = rank of i
// among splitting nodes; the built child is the lighter one (weights
// rec[wl_col] <= rec[wr_col] -> left, the host's rule); its segment is
// chunked into work items (j, start, count, k).  slots = [build | der | par]
// (stride n): build = 2j + !left, der = 2j + left, par = i.
// counts[0] = #pairs, counts[1] = #work items (capped at cap).
__global__ __launch_bounds__(1024) void child_work_kernel(const long long* __restrict__ st,
                                                          const long long* __restrict__ ct,
                                                          const double* __restrict__ rec, int stride, int ok_col,
                                                          int nl_col, int wl_col, int wr_col, int n, int chunk,
                                                          int cap, int4* __restrict__ work, int* __restrict__ slots,
                                                          int* __restrict__ counts) {
  __shared__ long long wtot[2][16];
  __shared__ long long carry[2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  if (threadIdx.x == 0) carry[0] = carry[1] = 0;
  __syncthreads();
  for (int base = 0; base < n; base += blockDim.x) {
    const int i = base + threadIdx.x;
    long long sp = 0, nch = 0, start = 0, cnt = 0;
    bool bl = true;
    if (i < n && rec[(size_t)i * stride + ok_col] > 0) {
      const long long nl = (long long)rec[(size_t)i * stride + nl_col];
      bl = rec[(size_t)i * stride + wl_col] <= rec[(size_t)i * stride + wr_col];
      cnt = bl ? nl : ct[i] - nl;
      start = bl ? st[i] : st[i] + nl;
      sp = 1;
      nch = (cnt + chunk - 1) / chunk;
    }
    long long a = sp, b = nch;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long ta = __shfl_up(a, o, 64), tb = __shfl_up(b, o, 64);
      if (lane >= o) { a += ta; b += tb; }
    }
    if (lane == 63) { wtot[0][wv] = a; wtot[1][wv] = b; }
    __syncthreads();
    if (wv == 0) {
      long long x = lane < nwv ? wtot[0][lane] : 0, y = lane < nwv ? wtot[1][lane] : 0;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const long long tx = __shfl_up(x, o, 64), ty = __shfl_up(y, o, 64);
        if (lane >= o) { x += tx; y += ty; }
      }
      if (lane < nwv) { wtot[0][lane] = x; wtot[1][lane] = y; }
    }
    __syncthreads();
    const long long j = carry[0] + (wv > 0 ? wtot[0][wv - 1] : 0) + a - sp;
    const long long it0 = carry[1] + (wv > 0 ? wtot[1][wv - 1] : 0) + b - nch;
    if (sp) {
      slots[j] = (int)(2 * j + (bl ? 0 : 1));
      slots[n + j] = (int)(2 * j + (bl ? 1 : 0));
      slots[2 * n + j] = i;
      for (long long k = 0; k < nch && it0 + k < cap; ++k) {
        const long long p = start + k * chunk;
        work[it0 + k] = make_int4((int)j, (int)p, (int)min((long long)chunk, cnt - k * chunk), (int)k);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) { carry[0] += wtot[0][nwv - 1]; carry[1] += wtot[1][nwv - 1]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    counts[0] = (int)carry[0];
    counts[1] = (int)min(carry[1], (long long)cap);
  }
}

int h2o_child_work(const long long* st, const long long* ct, const double* rec, int stride, int ok_col, int nl_col,
                   int wl_col, int wr_col, int n, int chunk, int cap, int* work, int* slots, int* counts,
                   hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(child_work_kernel, dim3(1), dim3(1024), 0, s, st, ct, rec, stride, ok_col, nl_col, wl_col, wr_col,
                     n, chunk, cap, (int4*)work, slots, counts);
  return (int)hipGetLastError();
}

int h2o_part_offsets(const int* cnt, const long long* meta, int nw, int n, int* loff, int* roff, long long* nleft,
                     double* pk, int stride, int col, hipStream_t s) {
  if (nw <= 0) return 0;
  hipLaunchKernelGGL(part_offsets_kernel, dim3(1), dim3(1024), 0, s, cnt, meta, nw, n, loff, roff, nleft, pk, stride,
                     col);
  return (int)hipGetLastError();
}

int h2o_part_compact(const int* ridx, const int* work, const int* fbase, int n_work,
                     const unsigned long long* flags, const int* loff, const int* roff, int* out, const float* pa,
                     float* pa_out, hipStream_t s) {
  if (n_work <= 0) return 0;
  static const int cu = [] { const char* e = getenv("H2O3_PART_U"); return e ? atoi(e) : 4; }();
  if (cu == 1)
    hipLaunchKernelGGL(part_compact_kernel<1>, dim3(n_work), dim3(256), 0, s, ridx, (const int4*)work, fbase, flags,
                       loff, roff, out, pa, pa_out, nullptr);
  else
    hipLaunchKernelGGL(part_compact_kernel<4>, dim3(n_work), dim3(256), 0, s, ridx, (const int4*)work, fbase, flags,
                       loff, roff, out, pa, pa_out, nullptr);
  return (int)hipGetLastError();
}

int h2o_part_count(const void* codes, int code_bytes, long long rs, long long fs, const int* ridx,
                   const int* work, int n_work, const int* feat, const uint8_t* masks, int Bs, int* cnt,
                   hipStream_t s) {
  if (n_work <= 0) return 0;
  if (code_bytes == 1)
    hipLaunchKernelGGL(part_count_kernel<uint8_t>, dim3(n_work), dim3(256), 0, s, (const uint8_t*)codes, rs, fs, ridx, (const int4*)work, feat, masks, Bs, cnt);
  else
    hipLaunchKernelGGL(part_count_kernel<uint16_t>, dim3(n_work), dim3(256), 0, s, (const uint16_t*)codes, rs, fs, ridx, (const int4*)work, feat, masks, Bs, cnt);
  return (int)hipGetLastError();
}

int h2o_part_scatter(const void* codes, int code_bytes, long long rs, long long fs, const int* ridx,
                     const int* work, int n_work, const int* feat, const uint8_t* masks, int Bs,
                     const int* loff, const int* roff, int* out, const float* pa, const float* pb,
                     float* pa_out, float* pb_out, hipStream_t s) {
  if (n_work <= 0) return 0;
  if (code_bytes == 1)
    hipLaunchKernelGGL(part_scatter_kernel<uint8_t>, dim3(n_work), dim3(256), 0, s, (const uint8_t*)codes, rs, fs, ridx, (const int4*)work, feat, masks, Bs, loff, roff, out, pa, pb, pa_out, pb_out);
  else
    hipLaunchKernelGGL(part_scatter_kernel<uint16_t>, dim3(n_work), dim3(256), 0, s, (const uint16_t*)codes, rs, fs, ridx, (const int4*)work, feat, masks, Bs, loff, roff, out, pa, pb, pa_out, pb_out);
  return (int)hipGetLastError();
}

int h2o_fill_nid(const int* ridx, const int* work, int n_work, int* nid, hipStream_t s) {
  if (n_work <= 0) return 0;
  hipLaunchKernelGGL(fill_nid_kernel, dim3(n_work), dim3(256), 0, s, ridx, (const int4*)work, nid);
  return (int)hipGetLastError();
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Per-leaf sums of two row vectors over the leaf segments of the row
// permutation (the GBM GammaPass numerator/denominator, DRF leaf means):
// no per-row atomics onto a handful of leaf addresses — each block reduces a
// chunk of one segment in registers/LDS and issues one f64 atomic per channel.
// work[i] = (leaf, start, count, -)
__global__ __launch_bounds__(256) void seg_sum2_kernel(const int* __restrict__ ridx, const float* __restrict__ a,
                                                       const float* __restrict__ b, const int4* __restrict__ work,
                                                       double* __restrict__ out) {
  const int4 wk = work[blockIdx.x];
  double sa = 0.0, sb = 0.0;
  for (int p = wk.y + threadIdx.x; p < wk.y + wk.z; p += blockDim.x) {
    const int r = ridx[p];
    sa += (double)a[r];
    if (b) sb += (double)b[r];
  }
  sa = wave_sum(sa);
  sb = wave_sum(sb);
  __shared__ double red[2][4];
  if (lane_id() == 0) { red[0][wave_id()] = sa; red[1][wave_id()] = sb; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ta = 0.0, tb = 0.0;
    for (int w = 0; w < (int)(blockDim.x / 64); ++w) { ta += red[0][w]; tb += red[1][w]; }
    gbl_add(out + 2 * wk.x, ta);
    if (b) gbl_add(out + 2 * wk.x + 1, tb);
  }
}

// Fused leaf pass (GBM gaussian / bernoulli): nid[ridx[p]] = leaf and the
// leaf's gamma sums in ONE walk over the leaf segments.
//   mode 0 (gaussian):  (sum w z, sum w)
//   mode 1 (bernoulli): (sum w z, sum w |z| (1 - |z|))   (z = y - p, so p(1-p) = |z|(1-|z|))
// work[i] = (leaf_id, start, count, -)
__global__ __launch_bounds__(256) void leaf_pass_kernel(const int* __restrict__ ridx, const float* __restrict__ z,
                                                        const float* __restrict__ w, const int4* __restrict__ work,
                                                        int mode, int* __restrict__ nid, double* __restrict__ out) {
  const int4 wk = work[blockIdx.x];
  double sa = 0.0, sb = 0.0;
  const int end = wk.y + wk.z;
  constexpr int U = 4;
  for (int p0 = wk.y + threadIdx.x; p0 < end; p0 += U * 256) {
    int r[U];
    float zz[U], ww[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = ridx[min(p0 + u * 256, end - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      zz[u] = z[r[u]];
      ww[u] = w ? w[r[u]] : 1.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (p0 + u * 256 < end) {
        if (nid) nid[r[u]] = wk.x;
        const double wz = (double)ww[u] * (double)zz[u];
        sa += wz;
        if (mode == 1) {
          const double az = fabs((double)zz[u]);
          sb += (double)ww[u] * az * (1.0 - az);
        } else {
          sb += (double)ww[u];
        }
      }
    }
  }
  sa = wave_sum(sa);
  sb = wave_sum(sb);
  __shared__ double red[2][4];
  if (lane_id() == 0) { red[0][wave_id()] = sa; red[1][wave_id()] = sb; }
  __syncthreads();
  if (threadIdx.x == 0) {
    gbl_add(out + 2 * wk.x, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    gbl_add(out + 2 * wk.x + 1, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

extern "C" int h2o_leaf_pass(const int* ridx, const float* z, const float* w, const int* work, int n_work, int mode,
                             int* nid, double* out, hipStream_t s) {
  if (n_work <= 0) return 0;
  hipLaunchKernelGGL(leaf_pass_kernel, dim3(n_work), dim3(256), 0, s, ridx, z, w, (const int4*)work, mode, nid, out);
  return (int)hipGetLastError();
}

extern "C" int h2o_seg_sum2(const int* ridx, const float* a, const float* b, const int* work, int n_work, double* out,
                            hipStream_t s) {
  if (n_work <= 0) return 0;
  hipLaunchKernelGGL(seg_sum2_kernel, dim3(n_work), dim3(256), 0, s, ridx, a, b, (const int4*)work, out);
  return (int)hipGetLastError();
}

extern "C" int h2o_leaf_pos(const float* zp, const int* work, int n_work, int mode, double* out, hipStream_t s) {
  if (n_work <= 0) return 0;
  hipLaunchKernelGGL(leaf_pos_kernel, dim3(n_work), dim3(256), 0, s, zp, (const int4*)work, mode, out, nullptr);
  return (int)hipGetLastError();
}

extern "C" int h2o_col_sample(int n, int m, const long long* elig, int k, unsigned long long seed, long long* out,
                              hipStream_t s) {
  if (n <= 0 || k <= 0) return 0;
  if (k > m) return 1;
  hipLaunchKernelGGL(col_sample_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, m, elig, k, seed, out);
  return (int)hipGetLastError();
}

extern "C" int h2o_leaf_scatter(const int* ridx, const int* work, int n_work, const float* val, float* d,
                                hipStream_t s) {
  if (n_work <= 0) return 0;
  hipLaunchKernelGGL(leaf_scatter_kernel, dim3(n_work), dim3(256), 0, s, ridx, (const int4*)work, val, d, nullptr);
  return (int)hipGetLastError();
}

extern "C" int h2o_leaf_update(const int* ridx, const int* work, int n_work, const float* val, float* f,
                               hipStream_t s) {
  if (n_work <= 0) return 0;
  hipLaunchKernelGGL(leaf_update_kernel, dim3(n_work), dim3(256), 0, s, ridx, (const int4*)work, val, f);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Row-direct (node, feature) PAIR histograms for column-sampled frontiers
// (DRF mtries, col_sample_rate at deep levels).  Reference: DRF samples
// mtries columns per node and ScoreBuildHistogram only fills those columns'
// DHistograms (hex/tree/drf/DRF.java, hex/tree/DTree.java:UndecidedNode
// scoreCols).  A level histogram [F][n][Bs][C] is mostly empty there (22 of
// 500 features per node) and, at 10^4 nodes x 1024 bins, larger than the
// memory budget -- so the old path rebuilt it in node batches from every row's
// full code row.  Here ONE workgroup builds ONE pair's histogram in LDS from
// the node's rows: the split feature's code comes from the column-major copy
// (codes_col[f][row], a 1- or 2-byte gather), the responses from the
// position-ordered payload or by row.  int64 fixed-point LDS atomics (exact,
// order-independent sums, like the level kernels).  Output is a compact
// [P][Bs][C] f64 buffer: a plain store when the node's rows fit one work item
// (no zero-fill of the buffer), f64 global atomics when a large node is spread
// over several items (those pairs' rows are pre-zeroed by the caller).
// work[i] = (pair, start, count, flags): bit0 = the pair's only work item
// (store), bit1 = also sum w*y*y into pwyy[pair] (one pair per node, MODE 0).
// MODE 0: channels (w, w*y), NaN response = zero-weight row when !HAS_VB;
// MODE 1: (g, h) = (va, vb).
// ---------------------------------------------------------------------------
template <typename CodeT, int MODE, bool HAS_VB, bool POSV>
__global__ __launch_bounds__(256) void pair_hist_kernel(const CodeT* __restrict__ codes_col, long long ncol,
                                                        const int* __restrict__ ridx, const float* __restrict__ va,
                                                        const float* __restrict__ vb,
                                                        const int4* __restrict__ work,
                                                        const int* __restrict__ pfeat, int Bs, float s0, float s1,
                                                        double* __restrict__ Hp, double* __restrict__ pwyy) {
  constexpr int C = 2;
  extern __shared__ __attribute__((aligned(16))) unsigned long long lh[];
  __shared__ double red[4];
  const int4 wk = work[blockIdx.x];
  const int pair = wk.x;
  const CodeT* cc = codes_col + (size_t)pfeat[pair] * (size_t)ncol;
  const int nb = Bs * C;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) lh[i] = 0ull;
  __syncthreads();
  const bool do_wyy = MODE == 0 && (wk.w & 2) != 0 && pwyy != nullptr;
  double wyy = 0.0;
  const int end = wk.y + wk.z;
  constexpr int U = 4;
  for (int p0 = wk.y + (int)threadIdx.x; p0 < end; p0 += U * 256) {
    int r[U];
    unsigned int c[U];
    float xa[U], xb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = ridx[min(p0 + u * 256, end - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int vi = POSV ? min(p0 + u * 256, end - 1) : r[u];
      xa[u] = va[vi];
      xb[u] = HAS_VB ? vb[vi] : 1.f;
    }
    // zero-weight rows (out-of-bag / NaN response) skip their code gather:
    // DRF trees carry the whole frame through the partition
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = MODE != 0 || (HAS_VB ? xb[u] != 0.f : xa[u] == xa[u]);
      c[u] = live ? (unsigned int)cc[r[u]] : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (p0 + u * 256 >= end) continue;
      float c0, c1;
      if (MODE == 0) {
        const float y = xa[u];
        const float w = HAS_VB ? xb[u] : (y == y ? 1.f : 0.f);
        if (w == 0.f) continue;
        c0 = w;
        c1 = w * y;
        if (do_wyy) wyy += (double)c1 * (double)y;
      } else {
        c0 = xa[u];
        c1 = xb[u];
      }
      unsigned long long* h = lh + c[u] * C;
      __hip_atomic_fetch_add(h, (unsigned long long)__float2ll_rn(c0 * s0), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(h + 1, (unsigned long long)__float2ll_rn(c1 * s1), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
  const double i0 = 1.0 / (double)s0, i1 = 1.0 / (double)s1;
  double* o = Hp + (size_t)pair * nb;
  const bool single = (wk.w & 1) != 0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    const long long v = (long long)lh[i];
    const double d = (double)v * ((i & 1) ? i1 : i0);
    if (single) o[i] = d;
    else if (v != 0) gbl_add(o + i, d);
  }
  if (do_wyy) {
    wyy = wave_sum(wyy);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = wyy;
    __syncthreads();
    if (threadIdx.x == 0) {
      const double t = red[0] + red[1] + red[2] + red[3];
      if (single) pwyy[pair] = t;
      else gbl_add(pwyy + pair, t);
    }
  }
}

// Several pairs of the SAME node per workgroup (KP <= 4 consecutive pairs,
// LDS = KP x Bs x 2 x 8 B): the node's row ids and responses are read once per
// group instead of once per pair; every pair still gathers its own code.
// work[i].w: bit0 = single item (store), bit1 = wyy (group holds the node's
// first pair), bits 8..15 = pairs in the group.
template <typename CodeT, int MODE, bool HAS_VB, bool POSV, int KP>
__global__ __launch_bounds__(256) void pair_hist_multi_kernel(const CodeT* __restrict__ codes_col, long long ncol,
                                                              const int* __restrict__ ridx,
                                                              const float* __restrict__ va,
                                                              const float* __restrict__ vb,
                                                              const int4* __restrict__ work,
                                                              const int* __restrict__ pfeat, int Bs, float s0,
                                                              float s1, double* __restrict__ Hp,
                                                              double* __restrict__ pwyy,
                                                              const int* __restrict__ fbins) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lh[];
  __shared__ double red[4];
  const int4 wk = work[blockIdx.x];
  const int pair0 = wk.x;
  const int np = (wk.w >> 8) & 0xff;
  const CodeT* cc[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) cc[j] = codes_col + (size_t)pfeat[pair0 + min(j, np - 1)] * (size_t)ncol;
  const int nb = Bs * 2;
  for (int i = threadIdx.x; i < KP * nb; i += blockDim.x) lh[i] = 0ull;
  __syncthreads();
  const bool do_wyy = MODE == 0 && (wk.w & 2) != 0 && pwyy != nullptr;
  double wyy = 0.0;
  const int end = wk.y + wk.z;
  constexpr int U = 2;
  for (int p0 = wk.y + (int)threadIdx.x; p0 < end; p0 += U * 256) {
    int r[U];
    unsigned int c[U][KP];
    float xa[U], xb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = ridx[min(p0 + u * 256, end - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int vi = POSV ? min(p0 + u * 256, end - 1) : r[u];
      xa[u] = va[vi];
      xb[u] = HAS_VB ? vb[vi] : 1.f;
    }
    // zero-weight rows (out-of-bag / NaN response) skip their KP code gathers
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = MODE != 0 || (HAS_VB ? xb[u] != 0.f : xa[u] == xa[u]);
#pragma unroll
      for (int j = 0; j < KP; ++j) c[u][j] = live ? (unsigned int)cc[j][r[u]] : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (p0 + u * 256 >= end) continue;
      float c0, c1;
      if (MODE == 0) {
        const float y = xa[u];
        const float w = HAS_VB ? xb[u] : (y == y ? 1.f : 0.f);
        if (w == 0.f) continue;
        c0 = w;
        c1 = w * y;
        if (do_wyy) wyy += (double)c1 * (double)y;
      } else {
        c0 = xa[u];
        c1 = xb[u];
      }
      const unsigned long long a0 = (unsigned long long)__float2ll_rn(c0 * s0);
      const unsigned long long a1 = (unsigned long long)__float2ll_rn(c1 * s1);
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        if (j < np) {
          unsigned long long* h = lh + j * nb + c[u][j] * 2;
          __hip_atomic_fetch_add(h, a0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(h + 1, a1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
  }
  __syncthreads();
  const double i0 = 1.0 / (double)s0, i1 = 1.0 / (double)s1;
  double* o = Hp + (size_t)pair0 * nb;
  const bool single = (wk.w & 1) != 0;
  // fbins: a pair's feature has fbins[f] codes below the NA bin (Bs - 1); the
  // always-empty bins between them are not written (the scoring and select
  // kernels read only [0, fbins) and the NA bin of narrow pairs) -- at deep
  // levels the 1025-bin outputs of the 256-bin numeric pairs were most of the
  // kernel's HBM writes
  int fb[KP];
#pragma unroll
  for (int j = 0; j < KP; ++j) fb[j] = (fbins != nullptr && j < np) ? min(fbins[pfeat[pair0 + j]], Bs - 1) : Bs - 1;
  for (int i = threadIdx.x; i < np * nb; i += blockDim.x) {
    const int j = i / nb, b = (i - j * nb) >> 1;
    int fbj = fb[0];
#pragma unroll
    for (int q = 1; q < KP; ++q) fbj = j == q ? fb[q] : fbj;
    if (b >= fbj && b < Bs - 1) continue;
    const long long v = (long long)lh[i];
    const double d = (double)v * ((i & 1) ? i1 : i0);
    if (single) o[i] = d;
    else if (v != 0) gbl_add(o + i, d);
  }
  if (do_wyy) {
    wyy = wave_sum(wyy);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = wyy;
    __syncthreads();
    if (threadIdx.x == 0) {
      const double t = red[0] + red[1] + red[2] + red[3];
      if (single) pwyy[pair0] = t;
      else gbl_add(pwyy + pair0, t);
    }
  }
}

template <typename CodeT, int MODE>
static void pair_hist_multi_launch(bool has_vb, bool posv, int n_work, size_t lds, hipStream_t s,
                                   const void* codes_col, long long ncol, const int* ridx, const float* va,
                                   const float* vb, const int4* work, const int* pfeat, int Bs, float s0, float s1,
                                   double* Hp, double* pwyy, const int* fbins) {
  const CodeT* cc = (const CodeT*)codes_col;
#define PHM(V, PV)                                                                                          \
  hipLaunchKernelGGL((pair_hist_multi_kernel<CodeT, MODE, V, PV, 4>), dim3(n_work), dim3(256), lds, s, cc, \
                     ncol, ridx, va, vb, work, pfeat, Bs, s0, s1, Hp, pwyy, fbins)
  if (has_vb) { if (posv) PHM(true, true); else PHM(true, false); }
  else { if (posv) PHM(false, true); else PHM(false, false); }
#undef PHM
}

// Grouped version of h2o_pair_hist: work[i].w bits 8..15 = pairs in the group
// (<= 4, consecutive pairs of one node starting at work[i].x).
static int pair_hist4_impl(const void* codes_col, int code_bytes, long long ncol, const int* ridx,
                           const float* va, const float* vb, const int* work, int n_work, const int* pfeat,
                           int Bs, int mode, int posv, float s0, float s1, double* Hp, double* pwyy,
                           hipStream_t s, const int* fbins);

extern "C" int h2o_pair_hist4(const void* codes_col, int code_bytes, long long ncol, const int* ridx,
                              const float* va, const float* vb, const int* work, int n_work, const int* pfeat,
                              int Bs, int mode, int posv, float s0, float s1, double* Hp, double* pwyy,
                              hipStream_t s) {
  return pair_hist4_impl(codes_col, code_bytes, ncol, ridx, va, vb, work, n_work, pfeat, Bs, mode, posv, s0, s1,
                         Hp, pwyy, s, nullptr);
}

// h2o_pair_hist4 that leaves each pair's bins [fbins[f], Bs - 1) unwritten.
extern "C" int h2o_pair_hist4b(const void* codes_col, int code_bytes, long long ncol, const int* ridx,
                               const float* va, const float* vb, const int* work, int n_work, const int* pfeat,
                               int Bs, int mode, int posv, float s0, float s1, double* Hp, double* pwyy,
                               hipStream_t s, const int* fbins) {
  return pair_hist4_impl(codes_col, code_bytes, ncol, ridx, va, vb, work, n_work, pfeat, Bs, mode, posv, s0, s1,
                         Hp, pwyy, s, fbins);
}

static int pair_hist4_impl(const void* codes_col, int code_bytes, long long ncol, const int* ridx,
                           const float* va, const float* vb, const int* work, int n_work, const int* pfeat,
                           int Bs, int mode, int posv, float s0, float s1, double* Hp, double* pwyy,
                           hipStream_t s, const int* fbins) {
  if (n_work <= 0) return 0;
  if (Bs < 2 || Bs > 4096 || (mode != 0 && mode != 1) || (mode == 1 && vb == nullptr)) return -1;
  const size_t lds = (size_t)4 * Bs * 2 * sizeof(unsigned long long);
  if (lds > 160 * 1024) return -2;
  const int4* w = (const int4*)work;
  const bool hv = vb != nullptr;
  if (code_bytes == 1) {
    if (mode == 0) pair_hist_multi_launch<uint8_t, 0>(hv, posv, n_work, lds, s, codes_col, ncol, ridx, va, vb, w, pfeat, Bs, s0, s1, Hp, pwyy, fbins);
    else pair_hist_multi_launch<uint8_t, 1>(hv, posv, n_work, lds, s, codes_col, ncol, ridx, va, vb, w, pfeat, Bs, s0, s1, Hp, pwyy, fbins);
  } else {
    if (mode == 0) pair_hist_multi_launch<uint16_t, 0>(hv, posv, n_work, lds, s, codes_col, ncol, ridx, va, vb, w, pfeat, Bs, s0, s1, Hp, pwyy, fbins);
    else pair_hist_multi_launch<uint16_t, 1>(hv, posv, n_work, lds, s, codes_col, ncol, ridx, va, vb, w, pfeat, Bs, s0, s1, Hp, pwyy, fbins);
  }
  return (int)hipGetLastError();
}

template <typename CodeT, int MODE>
static void pair_hist_launch(bool has_vb, bool posv, int n_work, size_t lds, hipStream_t s, const void* codes_col,
                             long long ncol, const int* ridx, const float* va, const float* vb, const int4* work,
                             const int* pfeat, int Bs, float s0, float s1, double* Hp, double* pwyy) {
  const CodeT* cc = (const CodeT*)codes_col;
#define PHL(V, PV)                                                                                                \
  hipLaunchKernelGGL((pair_hist_kernel<CodeT, MODE, V, PV>), dim3(n_work), dim3(256), lds, s, cc, ncol, ridx, va, \
                     vb, work, pfeat, Bs, s0, s1, Hp, pwyy)
  if (has_vb) { if (posv) PHL(true, true); else PHL(true, false); }
  else { if (posv) PHL(false, true); else PHL(false, false); }
#undef PHL
}

// codes_col: [F][ncol] column-major codes (code_bytes 1 or 2); work: n_work x
// int4 (pair, start, count, flags); pfeat[pair] = global feature; Hp:
// [P][Bs][2] f64; pwyy: [P] f64 (MODE 0, may be null).
extern "C" int h2o_pair_hist(const void* codes_col, int code_bytes, long long ncol, const int* ridx, const float* va,
                             const float* vb, const int* work, int n_work, const int* pfeat, int Bs, int mode,
                             int posv, float s0, float s1, double* Hp, double* pwyy, hipStream_t s) {
  if (n_work <= 0) return 0;
  if (Bs < 2 || Bs > 4096 || (mode != 0 && mode != 1) || (mode == 1 && vb == nullptr)) return -1;
  const size_t lds = (size_t)Bs * 2 * sizeof(unsigned long long);
  const int4* w = (const int4*)work;
  const bool hv = vb != nullptr;
  if (code_bytes == 1) {
    if (mode == 0) pair_hist_launch<uint8_t, 0>(hv, posv, n_work, lds, s, codes_col, ncol, ridx, va, vb, w, pfeat, Bs, s0, s1, Hp, pwyy);
    else pair_hist_launch<uint8_t, 1>(hv, posv, n_work, lds, s, codes_col, ncol, ridx, va, vb, w, pfeat, Bs, s0, s1, Hp, pwyy);
  } else {
    if (mode == 0) pair_hist_launch<uint16_t, 0>(hv, posv, n_work, lds, s, codes_col, ncol, ridx, va, vb, w, pfeat, Bs, s0, s1, Hp, pwyy);
    else pair_hist_launch<uint16_t, 1>(hv, posv, n_work, lds, s, codes_col, ncol, ridx, va, vb, w, pfeat, Bs, s0, s1, Hp, pwyy);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// GBM residual for the position-ordered payload in ONE pass (the torch chain
// sigmoid / sub / where / clone read and wrote the 100M-row vectors five
// times): z = y - f (mode 0, gaussian) or y - 1 / (1 + exp(-f)) (mode 1,
// bernoulli), NaN where the row weight is 0 (out-of-sample rows; the
// histogram and leaf kernels treat NaN as weight 0).  Reference:
// hex/tree/gbm/GBM.java ComputePredAndRes / Distribution.negHalfGradient.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gbm_grad_kernel(const float* __restrict__ y, float* __restrict__ f,
                                                       const float* __restrict__ w, int mode, long long n,
                                                       float* __restrict__ z, const float* __restrict__ d) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    float fi = f[i];
    if (d != nullptr) {          // previous tree's per-row leaf values (leaf_scatter_kernel)
      fi += d[i];
      f[i] = fi;
    }
    const float p = mode == 1 ? 1.f / (1.f + expf(-fi)) : fi;
    float v = y[i] - p;
    if (w != nullptr && !(w[i] > 0.f)) v = __builtin_nanf("");
    z[i] = v;
  }
}

extern "C" int h2o_gbm_grad(const float* y, float* f, const float* w, int mode, long long n, float* z,
                            const float* d, hipStream_t s) {
  if (n <= 0) return 0;
  const long long blocks = std::min<long long>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(gbm_grad_kernel, dim3((unsigned)blocks), dim3(256), 0, s, y, f, w, mode, n, z, d);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Partition work items built on the device: the host uploads only the
// per-segment (start, count, first-chunk index, first-flag-word index) table
// (O(frontier) numbers) and every chunk's record -- work int4 (segment,
// start, count, k), the offsets kernel's meta (segment, first chunk of the
// segment, segment start, position in segment) and the flag-word base -- is
// written here (the host numpy version cost ~0.2 ms per level at 2K chunks).
// seg: [4][n] int64.  chunk % 64 == 0.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void part_items_kernel(const long long* __restrict__ seg, int n, int chunk, int nw,
                                                         int4* __restrict__ work, long long* __restrict__ meta,
                                                         int* __restrict__ fbase) {
  const long long* st = seg;
  const long long* ct = seg + n;
  const long long* cb = seg + 2 * (long long)n;
  const long long* wb = seg + 3 * (long long)n;
  for (int c = blockIdx.x * 256 + threadIdx.x; c < nw; c += gridDim.x * 256) {
    int lo = 0, hi = n - 1;   // last segment whose first chunk index is <= c
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (cb[mid] <= c) lo = mid;
      else hi = mid - 1;
    }
    const int s = lo;
    const long long k = c - cb[s];
    const long long start = st[s] + k * chunk;
    const long long cnt = min((long long)chunk, ct[s] - k * chunk);
    work[c] = make_int4(s, (int)start, (int)cnt, (int)k);
    meta[c] = s;
    meta[(long long)nw + c] = cb[s];
    meta[2 * (long long)nw + c] = st[s];
    meta[3 * (long long)nw + c] = k * chunk;
    fbase[c] = (int)(wb[s] + k * (chunk / 64));
  }
}

extern "C" int h2o_part_items(const long long* seg, int n, int chunk, int nw, int* work, long long* meta,
                              int* fbase, hipStream_t s) {
  if (nw <= 0) return 0;
  if (chunk % 64 != 0 || n <= 0) return -1;
  const int blocks = std::min((nw + 255) / 256, 1024);
  hipLaunchKernelGGL(part_items_kernel, dim3(blocks), dim3(256), 0, s, seg, n, chunk, nw, (int4*)work, meta, fbase);
  return (int)hipGetLastError();
}

// ===========================================================================
// Device-resident tree level loop (models/tree/devtree.py).
//
// Reference: hex/tree/SharedTree.java:481-516 (scoreAndBuildTrees: one
// buildLayer per level, DTree.DecidedNode per split node), GBM.java:464.
//
// A whole tree runs as a fixed kernel sequence with NO host round trip: the
// frontier of level d is a heap of 2^d slots (slot i's children are slots 2i
// and 2i+1 of level d+1; absent nodes have count 0), and every per-level work
// list (histogram chunks of the lighter children, partition chunks, leaf
// chunks) is built on the device by dt_items_kernel from the level's split
// records, with launch grids sized to fixed capacities and early-exiting
// workgroups.  The sequence is therefore static -- the host captures it once
// as a hipGraph and replays it per tree -- and the tree comes back as ONE
// [2^(D+1)-1][DT_RS] f64 record read once per tree.
// ===========================================================================
#define DT_RS 16
enum {
  DT_GAIN = 0, DT_FEAT = 1, DT_T = 2, DT_OPT = 3, DT_L0 = 4, DT_L1 = 5, DT_R0 = 6, DT_R1 = 7, DT_T0 = 8, DT_T1 = 9,
  DT_OK = 10, DT_NL = 11, DT_NAW = 12, DT_ST = 13, DT_CT = 14, DT_VAL = 15
};
#define DT_MAXN 4096

// Segment of slot i for the three work-list kinds:
//   kind 0 (level): the slot's own rows (partition, root histogram);
//   kind 1 (child): the lighter child of a splitting parent slot (by the
//                   weight channel wch of the record's L / R sums; ties left);
//   kind 2 (leaf) : heap node i when it is a leaf (count > 0 and level == D or
//                   no split); i is a heap index into the whole record.
__device__ __forceinline__ void dt_seg(int kind, const double* __restrict__ rec, int i, int D, int wch,
                                       long long& start, long long& cnt) {
  const double* r = rec + (size_t)i * DT_RS;
  start = 0;
  cnt = 0;
  const long long st = (long long)r[DT_ST], ct = (long long)r[DT_CT];
  if (kind == 0) {
    start = st; cnt = ct;
  } else if (kind == 1) {
    if (r[DT_OK] > 0.0) {
      const long long nl = (long long)r[DT_NL];
      const bool bl = r[DT_L0 + wch] <= r[DT_R0 + wch];
      cnt = bl ? nl : ct - nl;
      start = bl ? st : st + nl;
    }
  } else {
    const int lv = 31 - __clz(i + 1);
    if (ct > 0 && (lv == D || !(r[DT_OK] > 0.0))) { start = st; cnt = ct; }
  }
}

// One workgroup: per-slot chunk counts scanned into item bases (LDS), then all
// threads write the items (slot found by binary search over the bases).
// work[it] = (slot, start, count, k); fbase[it] (optional) = the item's first
// ballot word (partition flags: the slot's words are contiguous, chunk % 64 == 0).
// counts[1] = #items (<= cap).
__global__ __launch_bounds__(1024) void dt_items_kernel(int kind, const double* __restrict__ rec, int n, int D,
                                                        int wch, int chunk, int cap, int4* __restrict__ work,
                                                        int* __restrict__ fbase, int* __restrict__ counts) {
  __shared__ int sb[DT_MAXN + 1];
  __shared__ int wb[DT_MAXN + 1];
  __shared__ long long wtot[2][16];
  __shared__ long long carry[2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  if (threadIdx.x == 0) carry[0] = carry[1] = 0;
  __syncthreads();
  for (int base = 0; base < n; base += blockDim.x) {
    const int i = base + threadIdx.x;
    long long start = 0, cnt = 0;
    if (i < n) dt_seg(kind, rec, i, D, wch, start, cnt);
    const long long nch = cnt > 0 ? (cnt + chunk - 1) / chunk : 0;
    const long long nwd = cnt > 0 ? (cnt + 63) / 64 : 0;
    long long a = nch, b = nwd;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long ta = __shfl_up(a, o, 64), tb = __shfl_up(b, o, 64);
      if (lane >= o) { a += ta; b += tb; }
    }
    if (lane == 63) { wtot[0][wv] = a; wtot[1][wv] = b; }
    __syncthreads();
    if (wv == 0) {
      long long x = lane < nwv ? wtot[0][lane] : 0, y = lane < nwv ? wtot[1][lane] : 0;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const long long tx = __shfl_up(x, o, 64), ty = __shfl_up(y, o, 64);
        if (lane >= o) { x += tx; y += ty; }
      }
      if (lane < nwv) { wtot[0][lane] = x; wtot[1][lane] = y; }
    }
    __syncthreads();
    if (i < n) {
      sb[i] = (int)(carry[0] + (wv > 0 ? wtot[0][wv - 1] : 0) + a - nch);
      wb[i] = (int)(carry[1] + (wv > 0 ? wtot[1][wv - 1] : 0) + b - nwd);
    }
    __syncthreads();
    if (threadIdx.x == 0) { carry[0] += wtot[0][nwv - 1]; carry[1] += wtot[1][nwv - 1]; }
    __syncthreads();
  }
  const int total = (int)min(carry[0], (long long)cap);
  for (int it = threadIdx.x; it < total; it += blockDim.x) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {                       // last slot whose base is <= it (empty slots precede it)
      const int mid = (lo + hi + 1) >> 1;
      if (sb[mid] <= it) lo = mid; else hi = mid - 1;
    }
    long long start, cnt;
    dt_seg(kind, rec, lo, D, wch, start, cnt);
    const int k = it - sb[lo];
    const long long p = start + (long long)k * chunk;
    work[it] = make_int4(lo, (int)p, (int)min((long long)chunk, cnt - (long long)k * chunk), k);
    if (fbase != nullptr) fbase[it] = wb[lo] + k * (chunk / 64);
  }
  if (threadIdx.x == 0) { counts[0] = n; counts[1] = total; }
}

// Compaction offsets of the level partition (one workgroup; items of a slot
// are consecutive, item k of a slot starts k * chunk rows into it): global
// exclusive scan of the per-item left counts, per-slot left totals into the
// record (DT_NL), loff / roff per item, and the NEXT level's segments
// (children 2i, 2i+1 of a splitting slot; count 0 otherwise) into rec_next.
__global__ __launch_bounds__(1024) void dt_offsets_kernel(const int* __restrict__ cnt, const int4* __restrict__ work,
                                                          const int* __restrict__ counts, double* __restrict__ rec,
                                                          int n, double* __restrict__ rec_next,
                                                          int* __restrict__ loff, int* __restrict__ roff) {
  __shared__ long long nl_s[DT_MAXN];
  __shared__ long long wtot[16];
  __shared__ long long carry;
  const int nw = counts[1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  for (int s = threadIdx.x; s < n; s += blockDim.x) nl_s[s] = 0;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < nw; base += blockDim.x) {
    const int i = base + threadIdx.x;
    const long long v = i < nw ? (long long)cnt[i] : 0;
    long long x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long t = __shfl_up(x, o, 64);
      if (lane >= o) x += t;
    }
    if (lane == 63) wtot[wv] = x;
    __syncthreads();
    if (wv == 0) {
      long long w = lane < nwv ? wtot[lane] : 0;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const long long t = __shfl_up(w, o, 64);
        if (lane >= o) w += t;
      }
      if (lane < nwv) wtot[lane] = w;
    }
    __syncthreads();
    if (i < nw) loff[i] = (int)(carry + (wv > 0 ? wtot[wv - 1] : 0) + x - v);
    __syncthreads();
    if (threadIdx.x == 0) carry += wtot[nwv - 1];
    __syncthreads();
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nw; i += blockDim.x) {
    const int4 wk = work[i];
    if (i == nw - 1 || work[i + 1].x != wk.x) nl_s[wk.x] = (long long)loff[i] + cnt[i] - (long long)loff[i - wk.w];
  }
  for (int i = threadIdx.x; i < nw; i += blockDim.x) roff[i] = loff[i - work[i].w];
  __syncthreads();
  for (int i = threadIdx.x; i < nw; i += blockDim.x) {
    const int4 wk = work[i];
    const long long st = (long long)rec[(size_t)wk.x * DT_RS + DT_ST];
    const long long lpre = (long long)loff[i] - (long long)roff[i];
    loff[i] = (int)(st + lpre);
    roff[i] = (int)(st + nl_s[wk.x] + ((long long)wk.y - st) - lpre);
  }
  for (int s = threadIdx.x; s < n; s += blockDim.x) {
    double* r = rec + (size_t)s * DT_RS;
    const long long nl = nl_s[s];
    r[DT_NL] = (double)nl;
    if (rec_next != nullptr) {
      double* c = rec_next + (size_t)(2 * s) * DT_RS;
      const bool ok = r[DT_OK] > 0.0;
      const double st = r[DT_ST], ct = r[DT_CT];
      c[DT_ST] = ok ? st : 0.0;
      c[DT_CT] = ok ? (double)nl : 0.0;
      c[DT_RS + DT_ST] = ok ? st + (double)nl : 0.0;
      c[DT_RS + DT_CT] = ok ? ct - (double)nl : 0.0;
    }
  }
}

// Level histograms by subtraction in heap layout: parent slot i's built
// (lighter) child histogram Hb[f][i] goes to slot 2i + !left, the sibling
// Hp[f][i] - Hb[f][i] to the other; a non-splitting parent writes zeros to
// both (absent nodes).  grid (np, Fl), one block per (parent, feature).
__global__ __launch_bounds__(256) void dt_sibling_kernel(const double* __restrict__ Hb, const double* __restrict__ Hp,
                                                         const double* __restrict__ rec_par, int np, int BsC, int C,
                                                         int clamp_mask, int wch, double* __restrict__ H,
                                                         const double* __restrict__ wyy_b,
                                                         const double* __restrict__ wyy_p,
                                                         double* __restrict__ wyy_out) {
  const int i = blockIdx.x, f = blockIdx.y;
  const double* r = rec_par + (size_t)i * DT_RS;
  const bool ok = r[DT_OK] > 0.0;
  const bool bl = r[DT_L0 + wch] <= r[DT_R0 + wch];
  const int bs = 2 * i + (bl ? 0 : 1), ds = 2 * i + (bl ? 1 : 0);
  const double* hb = Hb + ((size_t)f * np + i) * BsC;
  const double* hp = Hp + ((size_t)f * np + i) * BsC;
  double* ob = H + ((size_t)f * 2 * np + bs) * BsC;
  double* od = H + ((size_t)f * 2 * np + ds) * BsC;
  for (int k = threadIdx.x; k < BsC; k += blockDim.x) {
    double b = 0.0, d = 0.0;
    if (ok) {
      b = hb[k];
      d = hp[k] - b;
      if ((clamp_mask >> (k % C)) & 1) d = fmax(d, 0.0);
    }
    ob[k] = b;
    od[k] = d;
  }
  if (wyy_out != nullptr && f == 0 && threadIdx.x == 0) {
    wyy_out[bs] = ok ? wyy_b[i] : 0.0;
    wyy_out[ds] = ok ? wyy_p[i] - wyy_b[i] : 0.0;
  }
}

// Leaf values from the (all-reduced) leaf sums: v = s0 / s1 (0 if s1 == 0),
// clamped to +-maxabs, times the learning rate (device scalar, so a captured
// graph serves every tree).  Existence is global: a node exists when its
// parent split (the record's ok is merged across ranks), so every rank writes
// every leaf's value even when it holds none of the leaf's rows.
__global__ __launch_bounds__(256) void dt_leaf_vals_kernel(double* __restrict__ rec, const double* __restrict__ sums,
                                                           int nh, int D, const float* __restrict__ lr, double maxabs,
                                                           float* __restrict__ vals) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= nh) return;
  const int lv = 31 - __clz(h + 1);
  const bool exists = h == 0 || rec[(size_t)((h - 1) >> 1) * DT_RS + DT_OK] > 0.0;
  const bool leaf = exists && (lv == D || !(rec[(size_t)h * DT_RS + DT_OK] > 0.0));
  double v = 0.0;
  if (leaf) {
    const double den = sums[2 * h + 1];
    v = den != 0.0 ? sums[2 * h] / den : 0.0;
    v = fmin(fmax(v, -maxabs), maxabs) * (double)lr[0];
  }
  vals[h] = (float)v;
  rec[(size_t)h * DT_RS + DT_VAL] = v;
}

// Root record: segment [0, N), everything else zero (the record is re-zeroed
// per tree by the caller's memset).
__global__ void dt_root_kernel(double* __restrict__ rec, long long N) {
  if (threadIdx.x == 0) { rec[DT_ST] = 0.0; rec[DT_CT] = (double)N; }
}

extern "C" {

int h2o_dt_items(int kind, const double* rec, int n, int D, int wch, int chunk, int cap, int* work, int* fbase,
                 int* counts, hipStream_t s) {
  if (n <= 0 || n > DT_MAXN || chunk <= 0 || (fbase != nullptr && chunk % 64 != 0)) return -1;
  hipLaunchKernelGGL(dt_items_kernel, dim3(1), dim3(1024), 0, s, kind, rec, n, D, wch, chunk, cap, (int4*)work, fbase,
                     counts);
  return (int)hipGetLastError();
}

int h2o_dt_offsets(const int* cnt, const int* work, const int* counts, double* rec, int n, double* rec_next, int* loff,
                   int* roff, hipStream_t s) {
  if (n <= 0 || n > DT_MAXN) return -1;
  hipLaunchKernelGGL(dt_offsets_kernel, dim3(1), dim3(1024), 0, s, cnt, (const int4*)work, counts, rec, n, rec_next,
                     loff, roff);
  return (int)hipGetLastError();
}

int h2o_dt_sibling(const double* Hb, const double* Hp, const double* rec_par, int np, int F, int BsC, int C,
                   int clamp_mask, int wch, double* H, const double* wyy_b, const double* wyy_p, double* wyy_out,
                   hipStream_t s) {
  if (np <= 0 || F <= 0) return 0;
  hipLaunchKernelGGL(dt_sibling_kernel, dim3(np, F), dim3(256), 0, s, Hb, Hp, rec_par, np, BsC, C, clamp_mask, wch, H,
                     wyy_b, wyy_p, wyy_out);
  return (int)hipGetLastError();
}

int h2o_dt_leaf_vals(double* rec, const double* sums, int nh, int D, const float* lr, double maxabs, float* vals,
                     hipStream_t s) {
  hipLaunchKernelGGL(dt_leaf_vals_kernel, dim3((nh + 255) / 256), dim3(256), 0, s, rec, sums, nh, D, lr, maxabs, vals);
  return (int)hipGetLastError();
}

int h2o_dt_root(double* rec, long long N, hipStream_t s) {
  hipLaunchKernelGGL(dt_root_kernel, dim3(1), dim3(64), 0, s, rec, N);
  return (int)hipGetLastError();
}

// The partition / leaf kernels with the item count read on the device
// (counts[1]); n_cap = launch capacity.
int h2o_part_flags_dev(const void* codes, int code_bytes, long long rs, long long fs, const int* ridx, const int* work,
                       const int* fbase, int n_cap, const int* feat, const uint8_t* masks, int Bs,
                       unsigned long long* flags, int* cnt, const int* counts, hipStream_t s) {
  if (n_cap <= 0) return 0;
  if (code_bytes == 1)
    hipLaunchKernelGGL(part_flags_kernel<uint8_t>, dim3(n_cap), dim3(256), 0, s, (const uint8_t*)codes, rs, fs, ridx,
                       (const int4*)work, fbase, feat, masks, Bs, flags, cnt, counts);
  else
    hipLaunchKernelGGL(part_flags_kernel<uint16_t>, dim3(n_cap), dim3(256), 0, s, (const uint16_t*)codes, rs, fs,
                       ridx, (const int4*)work, fbase, feat, masks, Bs, flags, cnt, counts);
  return (int)hipGetLastError();
}

int h2o_part_compact_dev(const int* ridx, const int* work, const int* fbase, int n_cap,
                         const unsigned long long* flags, const int* loff, const int* roff, int* out, const float* pa,
                         float* pa_out, const int* counts, hipStream_t s) {
  if (n_cap <= 0) return 0;
  hipLaunchKernelGGL(part_compact_kernel<4>, dim3(n_cap), dim3(256), 0, s, ridx, (const int4*)work, fbase, flags, loff,
                     roff, out, pa, pa_out, counts);
  return (int)hipGetLastError();
}

int h2o_leaf_pos_dev(const float* zp, const int* work, int n_cap, int mode, double* out, const int* counts,
                     hipStream_t s) {
  if (n_cap <= 0) return 0;
  hipLaunchKernelGGL(leaf_pos_kernel, dim3(n_cap), dim3(256), 0, s, zp, (const int4*)work, mode, out, counts);
  return (int)hipGetLastError();
}

int h2o_leaf_scatter_dev(const int* ridx, const int* work, int n_cap, const float* val, float* d, const int* counts,
                         hipStream_t s) {
  if (n_cap <= 0) return 0;
  hipLaunchKernelGGL(leaf_scatter_kernel, dim3(n_cap), dim3(256), 0, s, ridx, (const int4*)work, val, d, counts);
  return (int)hipGetLastError();
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Device-resident tree, per-node column sampling (GBM col_sample_rate /
// col_sample_rate_change_per_level): the level's [2^d][Fl] split-eligibility
// mask built on the device from the parent records.  Heap slot i of level d
// exists when its parent split; the existing slots are ranked in heap order
// (the level loop's frontier order), and node r draws exactly the sample
// col_sample_kernel draws for frontier node r with the same seed: selection
// sampling of k of the m eligible features (the per-tree column sample) from
// a splitmix64 hash of (seed, r, j).  seed / k / m come from device buffers
// the host refreshes per tree, so the launch stays inside the captured graph.
extern "C" __global__ __launch_bounds__(1024) void dt_colmask_kernel(
    int d, const double* __restrict__ rec_par, const long long* __restrict__ elig, const int* __restrict__ m_dev,
    const int* __restrict__ k_dev, const unsigned long long* __restrict__ seed_dev, int f0, int Fl,
    unsigned char* __restrict__ okm) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int n = 1 << d;
  const int m = m_dev[0], k = k_dev[d];
  const unsigned long long seed = seed_dev[d];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < n; base += blockDim.x) {
    const int i = base + threadIdx.x;
    int ex = 0;
    if (i < n) ex = d == 0 ? 1 : (rec_par[(size_t)(i >> 1) * DT_RS + DT_OK] > 0.0 ? 1 : 0);
    int a = ex;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(a, o, 64);
      if (lane >= o) a += t;
    }
    if (lane == 63) wsum[wv] = a;
    __syncthreads();
    if (wv == 0) {
      int x = lane < nwv ? wsum[lane] : 0;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const int t = __shfl_up(x, o, 64);
        if (lane >= o) x += t;
      }
      if (lane < nwv) wsum[lane] = x;
    }
    __syncthreads();
    const int rank = carry + (wv > 0 ? wsum[wv - 1] : 0) + a - ex;
    if (i < n) {
      unsigned char* row = okm + (size_t)i * Fl;
      for (int f = 0; f < Fl; ++f) row[f] = 0;
      if (ex) {
        const unsigned long long b0 = smix64(seed ^ ((unsigned long long)rank * 0xD1B54A32D192ED03ull));
        int taken = 0;
        for (int j = 0; j < m && taken < k; ++j) {
          const double u = (double)(smix64(b0 + (unsigned long long)j) >> 11) * (1.0 / 9007199254740992.0);
          if (u * (double)(m - j) < (double)(k - taken)) {
            ++taken;
            const long long f = elig[j] - f0;
            if (f >= 0 && f < Fl) row[f] = 1;
          }
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) carry += wsum[nwv - 1];
    __syncthreads();
  }
}

extern "C" int h2o_dt_colmask(int d, const double* rec_par, const long long* elig, const int* m_dev,
                              const int* k_dev, const unsigned long long* seed_dev, int f0, int Fl,
                              unsigned char* okm, hipStream_t s) {
  if (d < 0 || d > 12 || Fl <= 0) return (int)hipErrorInvalidValue;
  if (d > 0 && rec_par == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(dt_colmask_kernel, dim3(1), dim3(1024), 0, s, d, rec_par, elig, m_dev, k_dev, seed_dev, f0,
                     Fl, okm);
  return (int)hipGetLastError();
}
