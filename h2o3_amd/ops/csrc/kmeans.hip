// Fused K-Means Lloyd pass: distances on the f32 matrix cores, per-row
// arg-min, per-cluster sums / weights / within-SS, assignment changes — one
// read of X per iteration.
//
// Reference: hex/kmeans/KMeans.java (Lloyds MRTask: per row the closest
// center by squared distance, then per-cluster column sums, row counts and
// within-cluster SS reduced across the cloud; IterationTask / TotSS), all
// in double on the CPU.
//
// MI355X design: X is a dense row-major f32 [N, P] in HBM.  A persistent
// workgroup of 4 waves walks 64-row tiles (grid-stride, XCD-aware order):
//   1. the tile (64 contiguous rows = one contiguous span of X) is loaded
//      with coalesced dwordx4 loads one tile ahead in registers (with the
//      rows' weights / old assignments: the loop body issues no other global
//      load, so no vmcnt wait ever drains the prefetch) and stored to LDS
//      (row stride P16+4 dwords, P16 = P rounded up to 16, zero tail);
//   2. every wave owns 16 rows and computes their dot products with all
//      centers with v_mfma_f32_16x16x4_f32 (exact f32 products) — lane group
//      g = lane>>4 takes the k-range [g*P16/4, (g+1)*P16/4), so A (rows) and B
//      (centers, resident in LDS for the whole pass) are read as float4;
//   3. d = |c|^2 - 2 x.c, arg-min over the 16 lanes that share a row (xor
//      shuffles, lowest index wins ties like torch.argmin);
//   4. per-cluster sums in LDS: thread (row group, column) owns one column
//      of a private [k, P] copy, reads four rows' sums in one round trip,
//      merges rows of the same cluster in registers and writes each sum
//      back once — no atomics (a returnless ds_add_f32 per (row, column)
//      measured 5x slower than the rest of the pass; one-hot MFMA and
//      per-center register selects were 2-3x slower than this); weights
//      and within-SS (|x|^2 + d_min) per cluster by LDS atomics (2 per row).
// Each workgroup writes one f64 partial (the fixed-point sums converted
// straight to f64; the f32 LDS weights / within-SS are folded into f64
// registers after every 64-row tile, the f32 private-copy sums into the f64
// partial every KM_FOLD tiles, so no f32 sum ever spans more than a few
// thousand rows); h2o_kmeans_reduce adds the partials in f64.  No global
// atomics.  Reference accumulates in double (KMeans.java LloydsIterationTask).
#include "common.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define KM_ROWS 64
#define KM_THREADS 256
#define KM_FOLD 16        // tiles between folds of the f32 private sums into the f64 partial

// partial layout per workgroup: [k*P sums][k weights][k withinss][1 changed]
__host__ __device__ inline long long km_part_stride(int k, int P) { return (long long)k * P + 2LL * k + 1; }

template <int KT, int MAXV, bool ACC>
__global__ __launch_bounds__(KM_THREADS) void kmeans_lloyd_kernel(
    const float* __restrict__ X, const float* __restrict__ w, long long N, int P, const float* __restrict__ Cin,
    const float* __restrict__ cn, int k, int* assign, const int* assign_old,
    float* __restrict__ dmin_out, double* __restrict__ part, int vrg_in, float fx_scale, int dbg) {
  extern __shared__ __align__(16) float lds[];
  const int P16 = (P + 15) & ~15;            // k-range padded so each lane group gets a float4 multiple
  const int S = P16 + 4;                     // LDS row stride (dwords)
  const int nq = (k + 15) >> 4;              // 16-center chunks in use (<= KT)
  const int KP = nq * 16;                    // centers padded to the MFMA tile
  float* Xs = lds;                           // [64][S]
  float* Cs = Xs + KM_ROWS * S;              // [KP][S]
  float* cns = Cs + KP * S;                  // [KP]
  // per-cluster sums: vrg private copies [vrg][k][P]; thread (vh, vc) owns
  // column vc of copy vh, so the read-modify-writes need no atomics
  const int vpr = P <= 64 ? 64 : (P <= 128 ? 128 : 256);
  const int vrg = vrg_in;
  const int vc = (int)threadIdx.x % vpr, vh = (int)threadIdx.x / vpr;
  // vrg == 0: one [k][P] copy of 64-bit fixed-point sums (returnless
  // ds_add_u64: ~5 per CU-clock vs 0.33 for ds_add_f32, scripts/lds_atomic_mb.hip)
  const int sum_f = vrg == 0 ? 2 * k * P : vrg * k * P;   // floats of LDS for the sums
  float* Ssum = cns + KP;                    // [vrg][k][P] f32, or [k][P] u64 (ACC)
  float* Swt = Ssum + (ACC ? sum_f : 0);     // [k]
  float* Sss = Swt + (ACC ? k : 0);          // [k]
  float* xsq = Sss + (ACC ? k : 0);          // [64]
  float* dmn = xsq + KM_ROWS;                // [64]
  int* asg = (int*)(dmn + KM_ROWS);          // [64]
  float* wts = (float*)(asg + KM_ROWS);      // [64] row weights of the tile
  __shared__ int changed_s;
  double* o = ACC ? part + (long long)blockIdx.x * km_part_stride(k, P) : nullptr;
  double wacc[2] = {0.0, 0.0};               // f64 weights / within-SS of entries tid, tid + 256 of [Swt | Sss]
  int nfold = 0;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int g = lane >> 4;                   // k-group of this lane
  const int li = lane & 15;
  const int Pq = P16 >> 2;                   // k-range per lane group (multiple of 4)

  // centers -> LDS (padded rows: zeros, |c|^2 = +inf never wins)
  for (int e = tid; e < KP * S; e += KM_THREADS) {
    const int j = e / S, c = e - j * S;
    Cs[e] = (j < k && c < P) ? Cin[(long long)j * P + c] : 0.f;
  }
  for (int j = tid; j < KP; j += KM_THREADS) cns[j] = j < k ? cn[j] : INFINITY;
  if (ACC) {
    for (int e = tid; e < sum_f + 2 * k; e += KM_THREADS) Ssum[e] = 0.f;   // Ssum, Swt, Sss contiguous
  }
  if (tid == 0) changed_s = 0;
  if (ACC && vrg > 0)
    for (int e = tid; e < k * P; e += KM_THREADS) o[e] = 0.0;   // folded f32 sums land here
  // X tile columns P..P16 stay zero (the staging below writes only c < P)
  for (int e = tid; e < KM_ROWS * S; e += KM_THREADS) Xs[e] = 0.f;

  const long long ntiles = (N + KM_ROWS - 1) / KM_ROWS;
  const int G = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, G);
  // each thread moves up to MAXV float4 of a tile; their LDS offsets are the
  // same for every tile (computed once: no divisions in the loop)
  const int nv4 = (KM_ROWS * P) >> 2;
  int xo[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int v = tid + i * KM_THREADS;
    const int e = v * 4;
    const int r = e / P;                     // P % 4 == 0: a float4 never straddles rows
    xo[i] = v < nv4 ? r * S + (e - r * P) : -1;
  }
  // prefetch set of a tile: its X floats + (threads < 64) row weight and old assignment
  f32x4 pre[MAXV];
  float pre_w = 1.f;
  int pre_a = -1;
  auto load_tile = [&](long long t) {
    const long long r0 = t * KM_ROWS;
    const long long lim = (N - r0) * P;      // valid floats in this tile
    const f32x4* src = (const f32x4*)(X + r0 * P);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int v = tid + i * KM_THREADS;
      f32x4 q = {0.f, 0.f, 0.f, 0.f};
      if (!(dbg & 8) && xo[i] >= 0 && 4LL * v < lim) q = src[v];
      pre[i] = q;
    }
    if (tid < KM_ROWS && r0 + tid < N) {
      if (ACC && w) pre_w = w[r0 + tid];
      if (ACC && assign_old) pre_a = assign_old[r0 + tid];
    }
  };
  // per-row results of the previous tile, stored just before the next prefetch
  long long out_r = -1;
  int out_a = 0;
  float out_d = 0.f;

  long long t = bid;
  if (t < ntiles) load_tile(t);
  __syncthreads();

  for (; t < ntiles; t += G) {
    const long long r0 = t * KM_ROWS;
    // registers -> LDS (row-strided) + the rows' scalars
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
      if (!(dbg & 16) && xo[i] >= 0) *(f32x4*)(Xs + xo[i]) = pre[i];
    int cur_a = pre_a;
    if (tid < KM_ROWS) wts[tid] = r0 + tid < N ? pre_w : 0.f;   // tail rows weigh nothing
    __syncthreads();
    if (t + G < ntiles) load_tile(t + G);    // next tile in flight during the math
    // previous tile's row outputs: issued right behind the prefetch, they
    // drain during this tile's math (the next top-of-loop wait covers both)
    if (out_r >= 0) {
      if (assign) assign[out_r] = out_a;
      if (dmin_out) dmin_out[out_r] = out_d;
      out_r = -1;
    }

    // ---- distances: wave wv owns rows 16*wv .. 16*wv+15
    f32x4 acc[KT];
#pragma unroll
    for (int q = 0; q < KT; ++q) acc[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const float* xa = Xs + (16 * wv + li) * S + g * Pq;
    const float* cb = Cs + li * S + g * Pq;
    float sq = 0.f;
    for (int s = 0; s < ((dbg & 1) ? 0 : Pq); s += 4) {
      const f32x4 a4 = *(const f32x4*)(xa + s);
      sq += a4[0] * a4[0] + a4[1] * a4[1] + a4[2] * a4[2] + a4[3] * a4[3];
#pragma unroll
      for (int q = 0; q < KT; ++q) {
        if (q < nq) {
          const f32x4 b4 = *(const f32x4*)(cb + q * 16 * S + s);
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[0], b4[0], acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[1], b4[1], acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[2], b4[2], acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[3], b4[3], acc[q], 0, 0, 0);
        }
      }
    }
    // |x|^2 of row li: sum over the 4 lane groups
    sq += __shfl_xor(sq, 16, 64);
    sq += __shfl_xor(sq, 32, 64);
    if (g == 0) xsq[16 * wv + li] = sq;
    // arg-min: lane holds rows 4g+r (r = reg), center q*16+li
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float best = INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int q = 0; q < KT; ++q) {
        const int j = q * 16 + li;
        const float d = q < nq ? cns[j] - 2.f * acc[q][r] : INFINITY;
        if (d < best) { best = d; bi = j; }
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
      }
      if (li == 0) {
        const int row = 16 * wv + 4 * g + r;
        dmn[row] = best;
        asg[row] = bi < k ? bi : 0;
      }
    }
    __syncthreads();
    // ---- per-row results + per-cluster weights / within-SS
    if (!(dbg & 4) && tid < KM_ROWS && r0 + tid < N) {
      const int a = asg[tid];
      const float d2 = fmaxf(xsq[tid] + dmn[tid], 0.f);
      if (ACC && assign_old && cur_a != a) atomicAdd(&changed_s, 1);
      out_r = r0 + tid;
      out_a = a;
      out_d = d2;
      if (ACC) {
        const float wr = wts[tid];
        if (wr != 0.f) {
          lds_add(Swt + a, wr);
          lds_add(Sss + a, wr * d2);
        }
      }
    }
    if (ACC && !(dbg & 2) && vrg == 0) {
      // ---- per-cluster sums as 64-bit fixed point: thread -> (row, column)
      // pairs, columns fastest (consecutive lanes, consecutive words)
      unsigned long long* S64 = reinterpret_cast<unsigned long long*>(Ssum);
      const long long nrow = min((long long)KM_ROWS, N - r0);
      const int tot = (int)nrow * P;
      int r = tid / P, c = tid - (tid / P) * P;
      const int dr = KM_THREADS / P, dc = KM_THREADS - (KM_THREADS / P) * P;
      for (int e = tid; e < tot; e += KM_THREADS) {
        const float v = wts[r] * Xs[r * S + c];
        if (v != 0.f)
          __hip_atomic_fetch_add(S64 + asg[r] * P + c, (unsigned long long)__float2ll_rn(v * fx_scale),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        r += dr; c += dc;
        if (c >= P) { c -= P; ++r; }
      }
    }
    if (ACC && !(dbg & 2) && vrg > 0 && vh < vrg && vc < P) {
      // ---- per-cluster sums: thread (vh, vc) walks rows vh, vh+vrg, ... four
      // at a time: the four sums are read first (one LDS round trip), rows
      // of the same cluster are merged in registers, each distinct cluster
      // written back once.  No atomics: a returnless ds_add_f32 per
      // (row, column) measured 5x slower than the rest of the pass.
      float* Sv = Ssum + vh * k * P + vc;
      for (int r = vh; r < KM_ROWS; r += 4 * vrg) {
        int a[4];
        float x[4], v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int rr = r + u * vrg;
          const bool ok = rr < KM_ROWS;
          a[u] = ok ? asg[rr] : asg[r];
          x[u] = ok ? wts[rr] * Xs[rr * S + vc] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = Sv[a[u] * P];
#pragma unroll
        for (int u = 1; u < 4; ++u) {
          // fold row u into the first earlier row of the same cluster
          if (a[u] == a[0]) { x[0] += x[u]; a[u] = -1; }
          else if (u > 1 && a[u] == a[1]) { x[1] += x[u]; a[u] = -1; }
          else if (u > 2 && a[u] == a[2]) { x[2] += x[u]; a[u] = -1; }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (a[u] >= 0) Sv[a[u] * P] = v[u] + x[u];
      }
    }
    __syncthreads();
    if (ACC) {
      // weights / within-SS of this tile: f32 LDS -> f64 registers, LDS re-zeroed
      // (the next tile's row stats are written only after the next barrier)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = tid + h * KM_THREADS;
        if (e < 2 * k) { wacc[h] += (double)Swt[e]; Swt[e] = 0.f; }
      }
      if (vrg > 0 && ++nfold == KM_FOLD) {
        nfold = 0;
        for (int e = tid; e < k * P; e += KM_THREADS) {
          float sv = 0.f;
          for (int h = 0; h < vrg; ++h) { sv += Ssum[h * k * P + e]; Ssum[h * k * P + e] = 0.f; }
          o[e] += (double)sv;
        }
      }
    }
  }
  if (out_r >= 0) {
    if (assign) assign[out_r] = out_a;
    if (dmin_out) dmin_out[out_r] = out_d;
  }
  if (ACC) {
    if (vrg == 0) {
      const unsigned long long* S64 = reinterpret_cast<const unsigned long long*>(Ssum);
      const double inv = 1.0 / (double)fx_scale;
      for (int e = tid; e < k * P; e += KM_THREADS) o[e] = (double)(long long)S64[e] * inv;
    } else {
      for (int e = tid; e < k * P; e += KM_THREADS) {
        float sv = 0.f;
        for (int h = 0; h < vrg; ++h) sv += Ssum[h * k * P + e];
        o[e] += (double)sv;
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = tid + h * KM_THREADS;
      if (e < 2 * k) o[k * P + e] = wacc[h];   // Swt, Sss contiguous
    }
    if (tid == 0) o[k * P + 2 * k] = (double)changed_s;
  }
}

// Large-k assignment pass (split path, first half): WAVE-persistent, X in
// registers, only the centers in LDS.
//
// The fused / acc=0 Lloyd kernel stages a 64-row X tile in LDS next to the
// centers; at k >= 64 that is 89 KB at P = 100, one 4-wave workgroup per CU,
// i.e. one wave per SIMD feeding dependent MFMA chains.  Here each wave owns
// 16-row tiles on its own (no barriers in the loop): lane (row li, k-group
// g) loads its row's k-range [g*Pq, (g+1)*Pq) straight from HBM as float4
// (the next tile is prefetched into a second register set), the centers sit
// in LDS for the whole pass (KP x (P16 + 4) floats: 59 KB at k = 128,
// P = 100), so 2 workgroups = 8 waves share a CU.  The MFMA loop interleaves
// the KT independent 16-center accumulators (the four k-slices of a float4
// outermost) so consecutive v_mfma never depend on each other.  Distances,
// arg-min (ties to the lowest index) and d2 = |x|^2 + min_j(|c_j|^2 - 2 x.c_j)
// as in the fused kernel; writes assign[N] and d2[N].
// MODE 1 (skinny GEMM, PCA / SVD projections): the same MFMA tiles write the
// dot products out[row][j] = x_row . c_j (f32, row-major [N][k]) instead of
// the arg-min -- X read once, no library GEMM.
// NW waves per workgroup; PF (NW == 4): the next tile is prefetched into a
// second register set, else (NW == 6, 3 waves per SIMD) occupancy hides the
// loads and the register set is dropped.
template <int KT, int MAXNV, int MODE = 0, int NW = 4>
__global__ __launch_bounds__(64 * NW) void kmeans_assign_kernel(const float* __restrict__ X, long long N, int P,
                                                            const float* __restrict__ Cin,
                                                            const float* __restrict__ cn, int k,
                                                            int* __restrict__ assign, float* __restrict__ d2out) {
  extern __shared__ __align__(16) float ldsa[];
  const int P16 = (P + 15) & ~15;
  const int S = P16 + 4;
  const int nq = (k + 15) >> 4;
  const int KP = nq * 16;
  float* Cs = ldsa;                          // [KP][S]
  float* cns = Cs + KP * S;                  // [KP]
  const int tid = threadIdx.x;
  constexpr bool PF = NW == 4;
  for (int e = tid; e < KP * S; e += 64 * NW) {
    const int j = e / S, c = e - j * S;
    Cs[e] = (j < k && c < P) ? Cin[(long long)j * P + c] : 0.f;
  }
  for (int j = tid; j < KP; j += 64 * NW) cns[j] = (j < k && cn != nullptr) ? cn[j] : INFINITY;
  __syncthreads();
  const int lane = tid & 63, wv = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int Pq = P16 >> 2;                   // k-range per lane group (multiple of 4)
  const int nv = Pq >> 2;                    // float4 per lane
  const long long ntiles = (N + 15) >> 4;
  const long long nwaves = (long long)gridDim.x * NW;
  long long t = (long long)xcd_remap(blockIdx.x, gridDim.x) * NW + wv;
  const float* cb = Cs + li * S + g * Pq;
  f32x4 A[MAXNV], B[PF ? MAXNV : 1];
  auto load = [&](long long tt, f32x4* R) {
    const long long row = tt * 16 + li;
    const bool okr = row < N;
    const float* src = X + row * (long long)P + g * Pq;
#pragma unroll
    for (int v = 0; v < MAXNV; ++v) {
      f32x4 q = {0.f, 0.f, 0.f, 0.f};
      if (v < nv && okr && g * Pq + 4 * v < P) q = *(const f32x4*)(src + 4 * v);
      R[v] = q;
    }
  };
  if (PF && t < ntiles) load(t, A);
  for (; t < ntiles; t += nwaves) {
    const bool more = t + nwaves < ntiles;
    if constexpr (PF) {
      if (more) load(t + nwaves, B);         // next tile in flight during the MFMAs
    } else {
      load(t, A);
    }
    f32x4 acc[KT];
#pragma unroll
    for (int q = 0; q < KT; ++q) acc[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float sq = 0.f;
    // Branch-free step loop: steps v >= nv and tiles q >= nq multiply zeros
    // (a4 is zero-filled by load(), b4 by the select), so the accumulators
    // never flow through control-flow joins -- with per-step `if`s the
    // compiler shuffles the KT accumulators between AGPRs and VGPRs at every
    // join (30k v_accvgpr moves, 412-444 VGPRs at KT = 8).  The dispatcher
    // picks KT / MAXNV close to nq / nv, so the padding MFMAs are few.
#pragma unroll
    for (int v = 0; v < MAXNV; ++v) {
      const f32x4 a4 = A[v];
      sq += a4[0] * a4[0] + a4[1] * a4[1] + a4[2] * a4[2] + a4[3] * a4[3];
      const bool vin = v < nv;
      f32x4 b4[KT];
#pragma unroll
      for (int q = 0; q < KT; ++q) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        b4[q] = (vin && q < nq) ? *(const f32x4*)(cb + q * 16 * S + 4 * v) : z;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < KT; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[j], b4[q][j], acc[q], 0, 0, 0);
    }
    sq += __shfl_xor(sq, 16, 64);
    sq += __shfl_xor(sq, 32, 64);            // |x|^2 of row li on every lane group
    const long long r0 = t * 16;
    if (MODE == 1) {
      // lane holds rows 4g + r, column q*16 + li of every 16-column block
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long row = r0 + 4 * g + r;
        if (row < N) {
#pragma unroll
          for (int q = 0; q < KT; ++q) {
            const int j = q * 16 + li;
            if (q < nq && j < k) d2out[row * k + j] = acc[q][r];
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < (MODE == 0 ? 4 : 0); ++r) {
      float best = INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int q = 0; q < KT; ++q) {
        const int j = q * 16 + li;
        const float d = q < nq ? cns[j] - 2.f * acc[q][r] : INFINITY;
        if (d < best) { best = d; bi = j; }
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
      }
      const float xs = __shfl(sq, 4 * g + r, 64);   // |x|^2 of row 4g + r
      const long long row = r0 + 4 * g + r;
      if (li == 0 && row < N) {
        assign[row] = bi < k ? bi : 0;
        d2out[row] = fmaxf(xs + best, 0.f);
      }
    }
    if constexpr (PF) {
      if (more) {
#pragma unroll
        for (int v = 0; v < MAXNV; ++v) A[v] = B[v];
      }
    }
  }
}

// Two 16-row tiles per wave (the default at KT >= 4; H2O3_KM_RT=1 selects the
// one-tile kernel above): every center
// float4 read from LDS feeds the MFMAs of both tiles, so the LDS traffic per
// MFMA halves and each step has 2 x KT independent accumulators in flight;
// no register prefetch (the second tile's registers take its place).
// 100M x 100: k = 128 44.1 ms per Lloyd iteration (46.9 one-tile), k = 64 29.0 (29.9).
template <int KT, int MAXNV>
__global__ __launch_bounds__(256) void kmeans_assign2_kernel(const float* __restrict__ X, long long N, int P,
                                                             const float* __restrict__ Cin,
                                                             const float* __restrict__ cn, int k,
                                                             int* __restrict__ assign, float* __restrict__ d2out) {
  extern __shared__ __align__(16) float ldsa[];
  const int P16 = (P + 15) & ~15;
  const int S = P16 + 4;
  const int nq = (k + 15) >> 4;
  const int KP = nq * 16;
  float* Cs = ldsa;
  float* cns = Cs + KP * S;
  const int tid = threadIdx.x;
  for (int e = tid; e < KP * S; e += 256) {
    const int j = e / S, c = e - j * S;
    Cs[e] = (j < k && c < P) ? Cin[(long long)j * P + c] : 0.f;
  }
  for (int j = tid; j < KP; j += 256) cns[j] = (j < k && cn != nullptr) ? cn[j] : INFINITY;
  __syncthreads();
  const int lane = tid & 63, wv = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int Pq = P16 >> 2;
  const int nv = Pq >> 2;
  const long long ntiles = (N + 15) >> 4;
  const long long npairs = (ntiles + 1) >> 1;
  const long long nwaves = (long long)gridDim.x * 4;
  const float* cb = Cs + li * S + g * Pq;
  auto load = [&](long long tt, f32x4* R) {
    const long long row = tt * 16 + li;
    const bool okr = row < N;
    const float* src = X + row * (long long)P + g * Pq;
#pragma unroll
    for (int v = 0; v < MAXNV; ++v) {
      f32x4 q = {0.f, 0.f, 0.f, 0.f};
      if (v < nv && okr && g * Pq + 4 * v < P) q = *(const f32x4*)(src + 4 * v);
      R[v] = q;
    }
  };
  auto finish = [&](const f32x4* acc, float sq, long long r0) {
    sq += __shfl_xor(sq, 16, 64);
    sq += __shfl_xor(sq, 32, 64);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float best = INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int q = 0; q < KT; ++q) {
        const int j = q * 16 + li;
        const float d = q < nq ? cns[j] - 2.f * acc[q][r] : INFINITY;
        if (d < best) { best = d; bi = j; }
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
      }
      const float xs = __shfl(sq, 4 * g + r, 64);
      const long long row = r0 + 4 * g + r;
      if (li == 0 && row < N) {
        assign[row] = bi < k ? bi : 0;
        d2out[row] = fmaxf(xs + best, 0.f);
      }
    }
  };
  for (long long tp = (long long)xcd_remap(blockIdx.x, gridDim.x) * 4 + wv; tp < npairs; tp += nwaves) {
    f32x4 A0[MAXNV], A1[MAXNV];
    load(2 * tp, A0);
    load(2 * tp + 1, A1);
    f32x4 acc0[KT], acc1[KT];
#pragma unroll
    for (int q = 0; q < KT; ++q) { acc0[q] = (f32x4){0.f, 0.f, 0.f, 0.f}; acc1[q] = acc0[q]; }
    float sq0 = 0.f, sq1 = 0.f;
#pragma unroll
    for (int v = 0; v < MAXNV; ++v) {
      const f32x4 a = A0[v], b = A1[v];
      sq0 += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
      sq1 += b[0] * b[0] + b[1] * b[1] + b[2] * b[2] + b[3] * b[3];
      const bool vin = v < nv;
      f32x4 b4[KT];
#pragma unroll
      for (int q = 0; q < KT; ++q) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        b4[q] = (vin && q < nq) ? *(const f32x4*)(cb + q * 16 * S + 4 * v) : z;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < KT; ++q) {
          acc0[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b4[q][j], acc0[q], 0, 0, 0);
          acc1[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j], b4[q][j], acc1[q], 0, 0, 0);
        }
    }
    finish(acc0, sq0, 2 * tp * 16);
    finish(acc1, sq1, (2 * tp + 1) * 16);
  }
}

static int km_assign_rt() {   // row tiles per wave: 2 (default), H2O3_KM_RT=1 for the one-tile kernel
  static int rt = -1;
  if (rt < 0) {
    const char* e = getenv("H2O3_KM_RT");
    rt = (e != nullptr && atoi(e) == 1) ? 1 : 2;
  }
  return rt;
}

template <int KT, int MAXNV, int MODE, int NW>
static int ka_launch3(const float* X, long long N, int P, const float* C, const float* cn, int k, int* assign,
                      float* d2, int G, hipStream_t s, int* per_cu_out) {
  const int P16 = (P + 15) & ~15, KP = ((k + 15) >> 4) * 16;
  const size_t lds = ((size_t)KP * (P16 + 4) + KP) * sizeof(float);
  auto kern = (MODE == 0 && KT >= 4 && km_assign_rt() == 2) ? kmeans_assign2_kernel<KT, MAXNV>
                                                             : kmeans_assign_kernel<KT, MAXNV, MODE, NW>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  if (per_cu_out) {
    int pc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, kern, 64 * NW, lds) != hipSuccess) return -1;
    *per_cu_out = pc;
    return 0;
  }
  hipLaunchKernelGGL(kern, dim3(G), dim3(64 * NW), lds, s, X, N, P, C, cn, k, assign, d2);
  H2O_CHECK_LAUNCH();
}

template <int KT, int MAXNV, int MODE = 0>
static int ka_launch2(const float* X, long long N, int P, const float* C, const float* cn, int k, int* assign,
                      float* d2, int G, hipStream_t s, int* per_cu_out) {
  // NW = 6 (3 waves per SIMD, no register prefetch) measured slower at
  // k = 128: 56.9 vs 47.0 ms per Lloyd iteration (profiles/README.md round 6)
  return ka_launch3<KT, MAXNV, MODE, 4>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
}

template <int KT, int MODE>
static int ka_launch(const float* X, long long N, int P, const float* C, const float* cn, int k, int* assign,
                     float* d2, int G, hipStream_t s, int* per_cu_out) {
  const int nv = ((P + 15) & ~15) >> 4;      // float4 per lane = P16 / 16
  // exact step counts up to 8 float4 (P <= 128): the padding steps of a
  // larger MAXNV would be MFMAs on zeros (the loop is branch-free)
  if (nv <= 2) return ka_launch2<KT, 2, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (nv <= 3) return ka_launch2<KT, 3, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (nv <= 4) return ka_launch2<KT, 4, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (nv <= 5) return ka_launch2<KT, 5, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (nv <= 6) return ka_launch2<KT, 6, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (nv <= 7) return ka_launch2<KT, 7, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (nv <= 8) return ka_launch2<KT, 8, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (nv <= 12) return ka_launch2<KT, 12, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  return ka_launch2<KT, 16, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
}

template <int MODE = 0>
static int ka_dispatch(const float* X, long long N, int P, const float* C, const float* cn, int k, int* assign,
                       float* d2, int G, hipStream_t s, int* per_cu_out) {
  if (P <= 0 || P > 256 || (P & 3) || k <= 0 || k > 256) return (int)hipErrorInvalidValue;
  const int P16 = (P + 15) & ~15, KP = ((k + 15) >> 4) * 16;
  if (((size_t)KP * (P16 + 4) + KP) * sizeof(float) > 160 * 1024) return (int)hipErrorInvalidValue;
  const int kt = (k + 15) >> 4;
  if (kt <= 1 && MODE == 1) return ka_launch<1, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (kt <= 2) return ka_launch<2, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (kt <= 4) return ka_launch<4, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (kt <= 6) return ka_launch<6, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (kt <= 8) return ka_launch<8, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  if (kt <= 12) return ka_launch<12, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
  return ka_launch<16, MODE>(X, N, P, C, cn, k, assign, d2, G, s, per_cu_out);
}

extern "C" int h2o_kmeans_assign_resident_per_cu(int k, int P) {
  int pc = 0;
  if (ka_dispatch(nullptr, 0, P, nullptr, nullptr, k, nullptr, nullptr, 0, nullptr, &pc) != 0) return 0;
  return pc;
}

// Assignment pass of the split path: assign[N] (int32) and d2[N] (f32,
// squared distance to the chosen center).  G workgroups of 4 waves.
extern "C" int h2o_kmeans_assign(const float* X, long long N, int P, const float* C, const float* cn, int k,
                                 int* assign, float* d2, int G, hipStream_t s) {
  if (N <= 0) return 0;
  if (G <= 0 || !assign || !d2) return (int)hipErrorInvalidValue;
  return ka_dispatch<0>(X, N, P, C, cn, k, assign, d2, G, s, nullptr);
}

// out [N][k] f32 = X [N][P] . V^T with V given as [k][P] rows (k <= 256,
// P % 4 == 0): the projections of PCA / SVD (X v_j) on the f32 matrix cores,
// X read once.  G workgroups of 4 waves (h2o_xv_resident_per_cu per CU).
extern "C" int h2o_xv_resident_per_cu(int k, int P) {
  int pc = 0;
  if (ka_dispatch<1>(nullptr, 0, P, nullptr, nullptr, k, nullptr, nullptr, 0, nullptr, &pc) != 0) return 0;
  return pc;
}

extern "C" int h2o_xv(const float* X, long long N, int P, const float* V, int k, float* out, int G, hipStream_t s) {
  if (N <= 0) return 0;
  if (G <= 0 || !out) return (int)hipErrorInvalidValue;
  return ka_dispatch<1>(X, N, P, V, nullptr, k, nullptr, out, G, s, nullptr);
}

// out[e] = sum_g part[g][e] in f64 (e over the whole partial record)
__global__ __launch_bounds__(256) void kmeans_reduce_kernel(const double* __restrict__ part, int G, long long stride,
                                                            double* __restrict__ out) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= stride) return;
  double s = 0.0;
  for (int gi = 0; gi < G; ++gi) s += part[(long long)gi * stride + e];
  out[e] = s;
}

// Large-k split path, second half: per-cluster sums of an assignment that
// the Lloyd kernel (acc = 0) already wrote.  At large k the fused kernel's
// LDS (X tile + centers + sums) allows one resident workgroup per CU and
// the whole pass runs latency-bound (profiles/kmeans_100m_k64_phase_mb.txt:
// 89 ms at k = 64, 49 ms of it in the sums).  Here the assignment pass keeps
// only X tile + centers in LDS, and this kernel keeps only the [k][P] 64-bit
// fixed-point sums: consecutive lanes take consecutive columns of a tile
// (coalesced 4-B loads, consecutive u64 LDS words: at most 2 lanes per bank
// pair, no same-address collisions within a wave-instruction), one
// returnless ds_add_u64 per (row, column).  Row weights / within-SS / changed
// assignments as in the fused kernel; one f64 partial per workgroup.
#define KMS_THREADS 1024   // sums pass: 16 waves per workgroup at one workgroup per CU
#define KMS_MAXJ 16        // X elements per thread per 64-row tile (64 * 256 / 1024)
// Software-pipelined: while the u64 atomics of tile t run, the X elements
// (and row assignment / weight / d2) of tile t + 1 are already in flight in
// registers, so each tile costs one HBM latency overlapped with LDS work
// instead of ~7 dependent load -> atomic round trips (the round-5 loop ran
// 29 ms at 100M x 100, k = 128, against ~7 ms of loads).  The per-row
// weight / within-SS go to f64 LDS sums (ds_add_f64, no per-tile f32 fold),
// and the tile's assignment / weight arrays are double-buffered: ONE barrier
// per tile.
__global__ __launch_bounds__(KMS_THREADS) void kmeans_sums_kernel(
    const float* __restrict__ X, const float* __restrict__ w, long long N, int P, int k,
    const int* __restrict__ asg, const int* __restrict__ asg_old, const float* __restrict__ d2,
    double* __restrict__ part, float fx_scale) {
  extern __shared__ __align__(16) unsigned long long S64[];   // [k][P]
  double* Swt = (double*)(S64 + (size_t)k * P);                 // [k]
  double* Sss = Swt + k;                                         // [k]
  int* tasg = (int*)(Sss + k);                                   // [2][64]
  float* tw = (float*)(tasg + 2 * KM_ROWS);                      // [2][64]
  __shared__ int changed_s;
  const int tid = threadIdx.x;
  for (int e = tid; e < k * P; e += KMS_THREADS) S64[e] = 0ull;
  for (int e = tid; e < 2 * k; e += KMS_THREADS) Swt[e] = 0.0;
  if (tid == 0) changed_s = 0;
  const long long ntiles = (N + KM_ROWS - 1) / KM_ROWS;
  const int G = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, G);
  // this thread's fixed (row, column) slots of a tile
  int rj[KMS_MAXJ], cj[KMS_MAXJ];
#pragma unroll
  for (int j = 0; j < KMS_MAXJ; ++j) {
    const int e = tid + j * KMS_THREADS;
    rj[j] = e / P;
    cj[j] = e - (e / P) * P;
  }
  float xv[KMS_MAXJ];
  int ra = 0, rold = 0;
  float rw = 0.f, rd = 0.f;
  auto fetch = [&](long long t) {
    const long long r0 = t * KM_ROWS;
    const int tot = (int)min((long long)KM_ROWS, N - r0) * P;
    const float* src = X + r0 * P;
#pragma unroll
    for (int j = 0; j < KMS_MAXJ; ++j) {
      const int e = tid + j * KMS_THREADS;
      xv[j] = e < tot ? src[e] : 0.f;
    }
    if (tid < KM_ROWS) {
      const long long r = r0 + tid;
      if (r < N) {
        ra = asg[r];
        rw = w ? w[r] : 1.f;
        rd = d2[r];
        rold = asg_old ? asg_old[r] : ra;
      } else {
        ra = 0; rw = 0.f; rd = 0.f; rold = 0;
      }
    }
  };
  __syncthreads();
  long long t = bid;
  if (t < ntiles) fetch(t);
  for (int it = 0; t < ntiles; t += G, ++it) {
    const int b = it & 1;
    if (tid < KM_ROWS) {
      if (rold != ra) atomicAdd(&changed_s, 1);
      if (rw != 0.f) {
        atomicAdd(Swt + ra, (double)rw);
        atomicAdd(Sss + ra, (double)rw * (double)rd);
      }
      tasg[b * KM_ROWS + tid] = ra;
      tw[b * KM_ROWS + tid] = rw;
    }
    __syncthreads();
    float cur[KMS_MAXJ];
#pragma unroll
    for (int j = 0; j < KMS_MAXJ; ++j) cur[j] = xv[j];
    if (t + G < ntiles) fetch(t + G);        // next tile in flight during this tile's atomics
    const int* ta = tasg + b * KM_ROWS;
    const float* twb = tw + b * KM_ROWS;
#pragma unroll
    for (int j = 0; j < KMS_MAXJ; ++j) {
      if (rj[j] < KM_ROWS) {
        const float v = twb[rj[j]] * cur[j];
        if (v != 0.f)
          __hip_atomic_fetch_add(S64 + ta[rj[j]] * P + cj[j], (unsigned long long)__float2ll_rn(v * fx_scale),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  __syncthreads();
  double* o = part + (long long)blockIdx.x * km_part_stride(k, P);
  const double inv = 1.0 / (double)fx_scale;
  for (int e = tid; e < k * P; e += KMS_THREADS) o[e] = (double)(long long)S64[e] * inv;
  for (int e = tid; e < 2 * k; e += KMS_THREADS) o[(long long)k * P + e] = Swt[e];
  if (tid == 0) o[(long long)k * P + 2 * k] = (double)changed_s;
}

static size_t km_sums_lds_bytes(int k, int P) {
  return (size_t)k * P * 8 + (size_t)2 * k * 8 + 2 * 2 * KM_ROWS * 4;
}

static int km_kt(int k) {   // the template instance a given k runs on
  const int kt = (k + 15) / 16;
  return kt <= 1 ? 1 : kt <= 2 ? 2 : kt <= 4 ? 4 : kt <= 8 ? 8 : 16;
}

static size_t km_lds_bytes(int KT, int k, int P, bool acc, int vrg) {
  (void)KT;
  const int P16 = (P + 15) & ~15, S = P16 + 4, KP = ((k + 15) / 16) * 16;
  const size_t sum_f = vrg == 0 ? 2 * (size_t)k * P : (size_t)vrg * k * P;
  size_t f = (size_t)KM_ROWS * S + (size_t)KP * S + KP + (acc ? sum_f + 2 * k : 0) + 4 * KM_ROWS;
  return f * 4;
}

// sums layout: 0 = one 64-bit fixed-point copy (when a scale is given and
// it fits), else private f32 copies per workgroup -- every thread busy
// (256 / vpr row groups) when the LDS allows, else fewer
static int km_vrg(int k, int P, bool acc, float fx_scale) {
  if (acc && fx_scale > 0.f && km_lds_bytes(0, k, P, acc, 0) <= 96 * 1024) return 0;
  const int vpr = P <= 64 ? 64 : (P <= 128 ? 128 : 256);
  int vrg = KM_THREADS / vpr;
  while (vrg > 1 && km_lds_bytes(0, k, P, acc, vrg) > 96 * 1024) vrg >>= 1;
  return vrg;
}

static int g_km_dbg = 0;   // microbenchmark phase-skip flags (h2o_kmeans_set_debug); 0 in production

template <int KT, int MAXV, bool ACC>
static int km_launch2(const float* X, const float* w, long long N, int P, const float* C, const float* cn, int k,
                      int* assign, const int* assign_old, float* dmin, double* part, int G, float fx, hipStream_t s) {
  const int vrg = km_vrg(k, P, ACC, fx);
  const size_t lds = km_lds_bytes(KT, k, P, ACC, vrg);
  auto kern = kmeans_lloyd_kernel<KT, MAXV, ACC>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(kern, dim3(G), dim3(KM_THREADS), lds, s, X, w, N, P, C, cn, k, assign, assign_old, dmin, part,
                     vrg, fx, g_km_dbg);
  H2O_CHECK_LAUNCH();
}

template <int KT>
static int km_launch(const float* X, const float* w, long long N, int P, const float* C, const float* cn, int k,
                     int* assign, const int* assign_old, float* dmin, double* part, int G, int acc, float fx,
                     hipStream_t s) {
  // MAXV = float4 per thread per 64-row tile = ceil(P / 16)
  if (P <= 64) return acc ? km_launch2<KT, 4, true>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, fx, s)
                          : km_launch2<KT, 4, false>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, fx, s);
  if (P <= 128) return acc ? km_launch2<KT, 8, true>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, fx, s)
                           : km_launch2<KT, 8, false>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, fx, s);
  return acc ? km_launch2<KT, 16, true>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, fx, s)
             : km_launch2<KT, 16, false>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, fx, s);
}

template <int KT, int MAXV, bool ACC>
static int km_resident2(int k, int P, float fx) {
  int per_cu = 0;
  const size_t lds = km_lds_bytes(KT, k, P, ACC, km_vrg(k, P, ACC, fx));
  auto kern = kmeans_lloyd_kernel<KT, MAXV, ACC>;
  if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, KM_THREADS, lds) != hipSuccess) return 0;
  return per_cu;
}

template <int KT>
static int km_resident(int k, int P, int acc, float fx) {
  if (P <= 64) return acc ? km_resident2<KT, 4, true>(k, P, fx) : km_resident2<KT, 4, false>(k, P, fx);
  if (P <= 128) return acc ? km_resident2<KT, 8, true>(k, P, fx) : km_resident2<KT, 8, false>(k, P, fx);
  return acc ? km_resident2<KT, 16, true>(k, P, fx) : km_resident2<KT, 16, false>(k, P, fx);
}

extern "C" {

// Largest k the fused kernel takes for a given P (LDS limit); 0 = unsupported P.
int h2o_kmeans_max_k(int P, int acc) {
  if (P <= 0 || P > 256 || (P & 3)) return 0;
  int best = 0;
  for (int k = 16; k <= 256; k += 16) {
    if (km_lds_bytes(km_kt(k), k, P, acc != 0, km_vrg(k, P, acc != 0, 0.f)) <= 160 * 1024) best = k;
  }
  return best;
}

long long h2o_kmeans_part_stride(int k, int P) { return km_part_stride(k, P); }

// Phase-skip flags for scripts/kmeans_mb.py (1 MFMA, 2 sums, 4 row stats,
// 8 global loads, 16 LDS staging).  Results are wrong with any flag set.
void h2o_kmeans_set_debug(int flags) { g_km_dbg = flags; }

// Workgroups of the Lloyd kernel resident per CU for (k, P, acc): the
// persistent grid is sized to exactly fill the chip (no tail of late
// workgroups walking a full share of tiles alone).
int h2o_kmeans_resident_per_cu(int k, int P, int acc, float fx_scale) {
  if (P <= 0 || P > 256 || (P & 3) || k <= 0 || k > 256) return 0;
  const int kt = km_kt(k);
  if (kt <= 1) return km_resident<1>(k, P, acc, fx_scale);
  if (kt <= 2) return km_resident<2>(k, P, acc, fx_scale);
  if (kt <= 4) return km_resident<4>(k, P, acc, fx_scale);
  if (kt <= 8) return km_resident<8>(k, P, acc, fx_scale);
  return km_resident<16>(k, P, acc, fx_scale);
}

// One Lloyd pass.  X [N, P] f32 row-major (P % 4 == 0, P <= 256), C [k, P]
// f32, cn [k] = |c|^2.  fx_scale > 0: per-cluster sums as 64-bit fixed point
// x * fx_scale (the caller bounds sum |w x| * fx_scale < 2^62 per workgroup).  acc=1: per-workgroup partials into part
// [G, km_part_stride] (then h2o_kmeans_reduce); acc=0: assignment only.
// assign / assign_old / dmin / w may be null.  Returns a hipError_t.
int h2o_kmeans_lloyd(const float* X, const float* w, long long N, int P, const float* C, const float* cn, int k,
                     int* assign, const int* assign_old, float* dmin, double* part, int G, int acc, float fx_scale,
                     hipStream_t s) {
  if (N <= 0) return 0;
  if (P <= 0 || P > 256 || (P & 3) || k <= 0 || k > 256 || G <= 0) return (int)hipErrorInvalidValue;
  const int kt = km_kt(k);
  if (km_lds_bytes(kt, k, P, acc != 0, km_vrg(k, P, acc != 0, fx_scale)) > 160 * 1024) return (int)hipErrorInvalidValue;
  if (acc && !part) return (int)hipErrorInvalidValue;
  if (kt <= 1) return km_launch<1>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, acc, fx_scale, s);
  if (kt <= 2) return km_launch<2>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, acc, fx_scale, s);
  if (kt <= 4) return km_launch<4>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, acc, fx_scale, s);
  if (kt <= 8) return km_launch<8>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, acc, fx_scale, s);
  return km_launch<16>(X, w, N, P, C, cn, k, assign, assign_old, dmin, part, G, acc, fx_scale, s);
}

// Large-k split path: LDS bytes / resident workgroups per CU of the sums
// kernel, and the launch.  asg: the new assignment (Lloyd kernel, acc = 0),
// asg_old: the previous one (changed count; may be null), d2: the per-row
// squared distances it wrote (dmin), fx_scale > 0 as for h2o_kmeans_lloyd.
int h2o_kmeans_sums_resident_per_cu(int k, int P) {
  const size_t lds = km_sums_lds_bytes(k, P);
  if (lds > 160 * 1024) return 0;
  if (hipFuncSetAttribute((const void*)kmeans_sums_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess)
    return 0;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kmeans_sums_kernel, KMS_THREADS, lds) != hipSuccess)
    return 0;
  return per_cu;
}

int h2o_kmeans_sums(const float* X, const float* w, long long N, int P, int k, const int* asg, const int* asg_old,
                    const float* d2, double* part, int G, float fx_scale, hipStream_t s) {
  if (N <= 0) return 0;
  if (P <= 0 || P > 256 || k <= 0 || k > 256 || G <= 0 || !part || !asg || !d2 || !(fx_scale > 0.f))
    return (int)hipErrorInvalidValue;
  const size_t lds = km_sums_lds_bytes(k, P);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)kmeans_sums_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(kmeans_sums_kernel, dim3(G), dim3(KMS_THREADS), lds, s, X, w, N, P, k, asg, asg_old, d2, part,
                     fx_scale);
  H2O_CHECK_LAUNCH();
}

int h2o_kmeans_reduce(const double* part, int G, long long stride, double* out, hipStream_t s) {
  if (G <= 0 || stride <= 0) return 0;
  const long long nb = (stride + 255) / 256;
  hipLaunchKernelGGL(kmeans_reduce_kernel, dim3((unsigned)nb), dim3(256), 0, s, part, G, stride, out);
  H2O_CHECK_LAUNCH();
}

}  // extern "C"
