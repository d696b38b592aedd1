// Weighted Gram matrix G = X^T diag(w) X on the f32 matrix cores.
//
// Reference: hex/gram/Gram.java (GramTask: per-row dense/sparse rank-1
// updates accumulated in double, one MRTask per IRLS iteration) and
// hex/glm/GLMTask.GLMIterationTask.
//
// MI355X design: X is a dense row-major f32 [N, P] in HBM (P padded to a
// multiple of 32).  A workgroup of 4 waves owns one 32x32 output tile pair
// (ti <= tj, only the upper triangle is computed) and a contiguous row
// range; every wave runs v_mfma_f32_32x32x2_f32 (exact f32 products, f32
// accumulate) straight from global memory — lane l of a 2-row K-step loads
// X[r0 + (l>>5)][col0 + (l&31)], so each half-wave reads one 128-byte
// segment of a row, fully coalesced, no LDS staging needed.  The diagonal
// weights w (IRLS working weights) are fused into the B operand.  Every 512
// rows the f32 accumulator is folded into an f64 accumulator (precision of
// the reference's double Gram at f32-MFMA speed); waves are reduced through
// LDS and each block writes an f64 partial tile that the host sums.
#include "common.h"
#include <type_traits>
#include <utility>
#include <cstdlib>
#include <algorithm>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void gram_kernel(const float* __restrict__ X, const float* __restrict__ w,
                                                   long long N, int P, const int2* __restrict__ pairs,
                                                   int rows_per_block, double* __restrict__ out) {
  const int pair = blockIdx.x;
  const int split = blockIdx.y;
  const int2 tp = pairs[pair];
  const int ci = tp.x * 32, cj = tp.y * 32;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const long long rb0 = (long long)split * rows_per_block;
  const long long rb1 = min((long long)N, rb0 + rows_per_block);
  // wave wv handles rows rb0 + 2*(wv + 4*t) .. (interleaved 2-row steps)
  const int kr = lane >> 5;
  const int cc = lane & 31;
  double acc64[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc64[i] = 0.0;
  f32x16 acc = {0};
  int since = 0;
  for (long long r = rb0 + 2 * wv + kr; r < rb1 + kr; r += 8) {
    float a = 0.f, b = 0.f;
    if (r < rb1) {
      const float* row = X + r * (long long)P;
      a = row[ci + cc];
      const float wr = w ? w[r] : 1.f;
      b = wr * (ci == cj ? a : row[cj + cc]);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    if (++since == 256) {
#pragma unroll
      for (int i = 0; i < 16; ++i) { acc64[i] += (double)acc[i]; acc[i] = 0.f; }
      since = 0;
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) acc64[i] += (double)acc[i];
  // reduce the 4 waves through LDS (f64): 32x32 doubles = 8 KB per wave
  __shared__ double red[4][32 * 32];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
    const int col = lane & 31;
    red[wv][row * 32 + col] = acc64[i];
  }
  __syncthreads();
  double* o = out + ((size_t)split * gridDim.x + pair) * 1024;
  for (int e = threadIdx.x; e < 1024; e += 256) {
    o[e] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
  }
}

extern "C" int h2o_gram(const float* X, const float* w, long long N, int P, const int* pairs, int n_pairs,
                        int n_splits, int rows_per_block, double* out, hipStream_t s) {
  if (N <= 0 || n_pairs <= 0) return 0;
  if (P % 32 != 0) return -1;
  dim3 grid(n_pairs, n_splits);
  hipLaunchKernelGGL(gram_kernel, grid, dim3(256), 0, s, X, w, N, P, (const int2*)pairs, rows_per_block, out);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused GLM IRLS pass: ONE read of X per iteration.
//
// Reference: hex/glm/GLMTask.java GLMIterationTask.map (per row: eta = x.b,
// mu = linkinv(eta), w = prior*d^2/var, z = eta + (y-mu)/d, Gram += w x x',
// xy += w z x, likelihood += dev) and hex/gram/Gram.java.
//
// MI355X design: a 256-thread workgroup streams 64-row chunks of X through
// LDS (row stride S = P + 16 (mod 64) so the four row-quarters of an MFMA
// operand read hit disjoint banks).  Per chunk: (1) the four waves compute
// eta = x.beta for 16 rows each (beta held in registers, 64-lane dot + DPP
// reduce); (2) wave 0 evaluates the family/link for its 64 rows (mu, IRLS
// weight W, working response z, deviance) and overwrites two padding
// columns of the staged chunk with 1 and z — so the SAME MFMA sweep also
// produces X'W1, X'Wz, sum W and sum Wz (the augmented Gram [X 1 z]'W[X 1 z]);
// (3) every wave runs v_mfma_f32_16x16x4f32 for up to 9 upper-triangle
// 16x16 tile pairs straight out of LDS (P=128: 36 pairs = 4 waves x 9,
// perfectly balanced over the SIMDs; less diagonal waste than 32x32), folding f32 -> f32 -> f64 every 256 / 16K
// rows.  Each block owns an f64 partial tile (no atomics -> deterministic;
// the caller zero-fills `out`).
// Mode EXTERNAL (W, z supplied by the caller) serves families / links the
// fused path does not cover and the plain weighted Gram (z == nullptr).
// ---------------------------------------------------------------------------
#define GI_RC 64
#define GI_PPW 9   // 16x16 tile pairs per wave (36 per workgroup: P=128 is one exact group)

struct GlmFamArgs {
  int link;     // 0 identity 1 logit 2 log 3 inverse
  int var;      // 0 gaussian 1 binomial 2 poisson 3 gamma 4 tweedie 5 negbin
  float tvp;    // tweedie variance power
  float theta;  // negative-binomial dispersion
  int dbg;      // perf experiments only: bit0 skip MFMA sweep, bit1 skip HBM loads of X,
                // bit2 skip y/w/offset loads, bit3 skip the eta dot products, bit4 eta and
                // sqrt(W) by ds_bpermute instead of DPP + LDS (ws kernel)
  int signed_w; // external weights may be negative (no sqrt(W) pre-scaling)
  int bf3;      // P = 128 ws path: 1 bf16x3 MFMA operands instead of f32, 2 one-MFMA bf16 (fused + gradient)
  int grad_f64; // exact-gradient channel: f64 products (1) or f32 products summed per chunk, f64 beyond (0)
};

__device__ __forceinline__ float gi_linkinv(int link, float eta) {
  switch (link) {
    case 1: return __frcp_rn(1.f + __expf(-eta));   // v_rcp_f32: no IEEE division sequence per row
    case 2: return __expf(fminf(eta, 80.f));
    case 3: return 1.f / (fabsf(eta) < 1e-10f ? (eta < 0.f ? -1e-10f : 1e-10f) : eta);
    default: return eta;
  }
}
__device__ __forceinline__ float gi_dmu(int link, float mu) {
  switch (link) {
    case 1: return fmaxf(mu * (1.f - mu), 1e-10f);
    case 2: return fmaxf(mu, 1e-10f);
    case 3: return -(mu * mu);
    default: return 1.f;
  }
}
__device__ __forceinline__ float gi_var(const GlmFamArgs& f, float mu) {
  switch (f.var) {
    case 1: return fmaxf(mu * (1.f - mu), 1e-10f);
    case 2: return fmaxf(mu, 1e-10f);
    case 3: return fmaxf(mu * mu, 1e-10f);
    case 4: return powf(fmaxf(mu, 1e-10f), f.tvp);
    case 5: return fmaxf(mu + f.theta * mu * mu, 1e-10f);
    default: return 1.f;
  }
}
__device__ __forceinline__ float gi_dev(const GlmFamArgs& f, float y, float mu) {
  switch (f.var) {
    case 1: {
      const float m = fminf(fmaxf(mu, 1e-15f), 1.f - 1e-7f);
      const float t1 = y > 0.f ? y * __logf(y / m) : 0.f;
      const float t2 = y < 1.f ? (1.f - y) * __logf((1.f - y) / (1.f - m)) : 0.f;
      return 2.f * (t1 + t2);
    }
    case 2: {
      const float t = y > 0.f ? y * __logf(y / fmaxf(mu, 1e-30f)) : 0.f;
      return 2.f * (t - (y - mu));
    }
    case 3: return 2.f * (-__logf(fmaxf(y, 1e-30f) / mu) + (y - mu) / mu);
    case 4: {
      const float p = f.tvp;
      if (p == 0.f) return (y - mu) * (y - mu);
      if (p == 1.f) { const float t = y > 0.f ? y * __logf(y / mu) : 0.f; return 2.f * (t - (y - mu)); }
      if (p == 2.f) return 2.f * (-__logf(fmaxf(y, 1e-30f) / mu) + (y - mu) / mu);
      const float a = y > 0.f ? powf(y, 2.f - p) / ((1.f - p) * (2.f - p)) : 0.f;
      return 2.f * (a - y * powf(mu, 1.f - p) / (1.f - p) + powf(mu, 2.f - p) / (2.f - p));
    }
    case 5: {
      const float th = f.theta;
      const float t1 = y > 0.f ? y * __logf(y / mu) : 0.f;
      const float t2 = (y + 1.f / th) * __logf((1.f + th * y) / (1.f + th * mu));
      return 2.f * (t1 - t2);
    }
    default: return (y - mu) * (y - mu);
  }
}

// upper-triangle pair p of T tiles -> (i, j), same order as linalg_ops._pairs
__host__ __device__ constexpr int gi_pair_i(int T, int p) {
  int i = 0;
  while (p >= T - i) { p -= T - i; ++i; }
  return i;
}
__host__ __device__ constexpr int gi_pair_j(int T, int p) {
  int i = 0;
  while (p >= T - i) { p -= T - i; ++i; }
  return i + p;
}

template <int T, int SL, int Q>
__device__ __forceinline__ void gi_mfma_q(const float* xr, const float* xw, f32x4* acc) {
  constexpr int pp = SL + 4 * Q;
  if constexpr (pp < T * (T + 1) / 2) {
    constexpr int ti = gi_pair_i(T, pp), tj = gi_pair_j(T, pp);
    acc[Q] = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[ti], xw[tj], acc[Q], 0, 0, 0);
  }
}
template <int T, int SL, int... Q>
__device__ __forceinline__ void gi_mfma_all(std::integer_sequence<int, Q...>, const float* xr, const float* xw,
                                            f32x4* acc) {
  (gi_mfma_q<T, SL, Q>(xr, xw, acc), ...);
}

// quad_perm DPP move (0xB1: lane ^ 1, 0x4E: lane ^ 2), a VALU op instead of ds_bpermute
template <int CTRL>
__device__ __forceinline__ float gi_dpp(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}

// bf16x3 path: every staged value is split x = hi + lo (hi = bf16(x), lo =
// bf16(x - hi)) and each f32 product is rebuilt from hi*hi + hi*lo + lo*hi on
// the 16x16x32 bf16 MFMA (lo*lo ~ 2^-16 relative is dropped): 3 bf16 MFMAs of
// 16 cycles replace 8 f32 16x16x4 MFMAs of 32 cycles for the same 32 rows.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// XOR swizzle of the 8-row k-blocks of feature f in the bf16x3 LDS image
// (glm_irls_ws_kernel): conflict-free producer b128 stores and consumer b128
// operand reads (searched over pads / swizzles against the gfx950 lane groups)
__device__ __forceinline__ int gi_swz(int f) { return (f ^ (f >> 2)) & 7; }

template <int T, int SL, int Q, int M>
__device__ __forceinline__ void gi_mfma3_q(const bf16x8* ah, const bf16x8* al, f32x4* acc) {
  constexpr int pp = SL + 4 * Q;
  if constexpr (pp < T * (T + 1) / 2) {
    constexpr int ti = gi_pair_i(T, pp), tj = gi_pair_j(T, pp);
    if constexpr (M == 0) acc[Q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ti], ah[tj], acc[Q], 0, 0, 0);
    if constexpr (M == 1) acc[Q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ti], al[tj], acc[Q], 0, 0, 0);
    if constexpr (M == 2) acc[Q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[ti], ah[tj], acc[Q], 0, 0, 0);
  }
}
// one-MFMA bf16 tier (hi*hi only, ~2^-9 relative per product)
template <int T, int SL, int... Q>
__device__ __forceinline__ void gi_mfma1_all(std::integer_sequence<int, Q...>, const bf16x8* ah, f32x4* acc) {
  (gi_mfma3_q<T, SL, Q, 0>(ah, ah, acc), ...);
}
// all hi*hi first, then the two cross terms: consecutive MFMAs hit different
// accumulators
template <int T, int SL, int... Q>
__device__ __forceinline__ void gi_mfma3_all(std::integer_sequence<int, Q...>, const bf16x8* ah, const bf16x8* al,
                                             f32x4* acc) {
  (gi_mfma3_q<T, SL, Q, 0>(ah, al, acc), ...);
  (gi_mfma3_q<T, SL, Q, 1>(ah, al, acc), ...);
  (gi_mfma3_q<T, SL, Q, 2>(ah, al, acc), ...);
}

// Chunk rows (multiple of 4 = one 16x16x4 k-step); the staging registers hold
// NV = ceil(RC*PP/1024) float4 per thread.
template <int PP>
struct GiCfg {
  static constexpr int RC = PP <= 128 ? 64 : ((8192 / PP) / 4 * 4 < 16 ? 16 : (8192 / PP) / 4 * 4);
  static constexpr int P4 = PP / 4;                        // float4 per row
  static constexpr int NV = (RC * P4 + 255) / 256;         // float4 per thread
  static constexpr bool EXACT = (RC * P4) % 256 == 0;
  static constexpr int FOLD = RC >= 256 ? 1 : 256 / RC;   // chunks per f32 fold (~256 rows)
  static constexpr int RPP = 256 / P4 > 0 ? 256 / P4 : 1;  // rows per staging pass
  static constexpr bool POW2 = (PP & (PP - 1)) == 0;
};

template <int PP, bool FUSED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void glm_irls_kernel(
    const float* __restrict__ X, long long N, const int2* __restrict__ pairs, int n_pairs, int rows_per_block,
    const float* __restrict__ beta, float b0, const float* __restrict__ y, const float* __restrict__ wprior,
    const float* __restrict__ offset, GlmFamArgs fam, const float* __restrict__ Wext,
    const float* __restrict__ zext, int aug, double* __restrict__ out, double* __restrict__ dev_out) {
  using C = GiCfg<PP>;
  constexpr int RC = C::RC, P4 = C::P4, NV = C::NV;
  // row stride: the 4 row-quarters of an MFMA operand read land 16 banks apart
  constexpr int S = PP + ((16 - (PP % 64)) & 63);
  static_assert(!FUSED || C::POW2, "fused path needs a power-of-two padded width");
  __shared__ float L[RC * S];
  __shared__ float wr[RC];
  __shared__ float eta_s[2][RC];
  const int split = blockIdx.x;
  const int grp = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int kr = lane >> 4, cc = lane & 15;
  const long long rb0 = (long long)split * rows_per_block;
  const long long rb1 = min(N, rb0 + rows_per_block);

  // tile pairs of this wave; the slot rotates with the block id so that the
  // co-resident blocks of a CU spread the 3-pair slots over all four SIMDs
  int ci[GI_PPW], cj[GI_PPW];
  bool pv[GI_PPW];
  const int slot = __builtin_amdgcn_readfirstlane((wv + split) & 3);  // wave-uniform -> SGPRs
#pragma unroll
  for (int q = 0; q < GI_PPW; ++q) {
    const int p = grp * (4 * GI_PPW) + slot + 4 * q;
    pv[q] = p < n_pairs;
    const int2 t = pv[q] ? pairs[p] : make_int2(0, 0);
    ci[q] = __builtin_amdgcn_readfirstlane(t.x * 16);
    cj[q] = __builtin_amdgcn_readfirstlane(t.y * 16);
  }
  int npv = 0;
#pragma unroll
  for (int q = 0; q < GI_PPW; ++q) npv += pv[q] ? 1 : 0;
  // fused: every thread always stages the same 4 columns (POW2 width), so
  // its slice of beta lives in 4 registers and eta is reduced from the
  // staging registers before they ever reach LDS
  const int c4 = threadIdx.x % P4;
  float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (FUSED) b4 = *reinterpret_cast<const float4*>(beta + 4 * c4);

  // mid-level f32 accumulators live in LDS (this wave's own slice, lane-major:
  // conflict-free) to keep the VGPR budget for the MFMA pipeline
  __shared__ float midL[4][GI_PPW * 4][64];
  f32x4 acc[GI_PPW];
#pragma unroll
  for (int q = 0; q < GI_PPW; ++q) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { midL[wv][4 * q + i][lane] = 0.f; acc[q][i] = 0.f; }
  }
  double dev = 0.0;

  f32x4 V[NV];
  float sy = 0.f, sw = 0.f, so = 0.f;  // wave 0: per-row scalars of the staged chunk
  auto load_chunk = [&](long long r0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int ee = (C::EXACT || e < RC * P4) ? e : RC * P4 - 1;  // tail lanes re-load the last vector
      const int rr = ee / P4, cq = ee - rr * P4;
      const long long g = min(r0 + rr, N - 1);
      V[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(X + g * (long long)PP) + cq);
    }
    if (wv == 0 && lane < RC) {
      const long long g = min(r0 + lane, N - 1);
      if (FUSED) {
        sy = y[g];
        sw = wprior ? wprior[g] : 1.f;
        so = offset ? offset[g] : 0.f;
      } else {
        sw = Wext ? Wext[g] : 1.f;
        sy = zext ? zext[g] : 0.f;
      }
    }
  };

  int since = 0;
  if (rb0 < rb1) load_chunk(rb0);
  for (long long r0 = rb0; r0 < rb1; r0 += RC) {
    // (0) registers -> LDS (+ eta partial sums straight from the registers)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int ee = (C::EXACT || e < RC * P4) ? e : RC * P4 - 1;  // duplicate store of identical data
      const int rr = ee / P4, cq = ee - rr * P4;
      *reinterpret_cast<f32x4*>(L + rr * S + 4 * cq) = V[i];
      if (FUSED) {
        float s = V[i].x * b4.x + V[i].y * b4.y + V[i].z * b4.z + V[i].w * b4.w;
        constexpr int G = P4 < 64 ? P4 : 64;
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((threadIdx.x & (G - 1)) == 0) eta_s[(threadIdx.x % P4) / 64][rr] = s;
      }
    }
    __syncthreads();
    // (1) wave 0: family / link -> IRLS weight W and working response z
    if (wv == 0 && lane < RC) {
      const long long r = r0 + lane;
      float W = 0.f, z = 0.f;
      if (r < rb1) {
        if (FUSED) {
          const float eta = eta_s[0][lane] + (P4 > 64 ? eta_s[1][lane] : 0.f) + b0 + so;
          const float mu = gi_linkinv(fam.link, eta);
          if (fam.link == 0 && fam.var == 0) {
            W = sw;
            z = sy - so;
          } else {
            const float d = gi_dmu(fam.link, mu);
            W = sw * d * d / gi_var(fam, mu);
            z = (eta - so) + (sy - mu) / d;
          }
          if (sw != 0.f) dev += (double)(sw * gi_dev(fam, sy, mu));
        } else {
          W = sw;
          z = sy;
        }
      }
      wr[lane] = W;
      if (aug >= 0) {
        L[lane * S + aug] = 1.f;
        L[lane * S + aug + 1] = z;
      }
    }
    // (2) prefetch the next chunk while this one is on the matrix cores
    if (r0 + RC < rb1) load_chunk(r0 + RC);
    __syncthreads();
    // (3) MFMA sweep; the pair count is wave-uniform, so branch once outside
    // the loop and keep the body branch-free (LDS loads run ahead of MFMAs)
    auto sweep = [&](auto npv_tag) {
      constexpr int NPV = decltype(npv_tag)::value;
#pragma unroll 2
      for (int k = 0; k < RC / 4; ++k) {
        const int rr = 4 * k + kr;
        const float w = wr[rr];
        const float* row = L + rr * S;
#pragma unroll
        for (int q = 0; q < NPV; ++q) {
          const float a = row[ci[q] + cc];
          const float b = w * row[cj[q] + cc];
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[q], 0, 0, 0);
        }
      }
    };
    // P <= 128 (one pair group): the wave's pairs are compile-time, so each
    // k-step reads every 16-column tile ONCE (T <= 8 LDS reads instead of
    // 2 per pair) and weights it once; the 9 MFMAs then run from registers.
    auto sweep_ct = [&](auto slot_tag) {
      constexpr int SL = decltype(slot_tag)::value;
      constexpr int T = PP / 16;
#pragma unroll 2
      for (int k = 0; k < RC / 4; ++k) {
        const int rr = 4 * k + kr;
        const float w = wr[rr];
        const float* row = L + rr * S + cc;
        float xr[T], xw[T];
#pragma unroll
        for (int t = 0; t < T; ++t) xr[t] = row[16 * t];
#pragma unroll
        for (int t = 0; t < T; ++t) xw[t] = w * xr[t];
        gi_mfma_all<T, SL>(std::make_integer_sequence<int, GI_PPW>{}, xr, xw, acc);
      }
    };
    if constexpr (PP <= 128) {
      switch (slot) {
        case 0: sweep_ct(std::integral_constant<int, 0>{}); break;
        case 1: sweep_ct(std::integral_constant<int, 1>{}); break;
        case 2: sweep_ct(std::integral_constant<int, 2>{}); break;
        default: sweep_ct(std::integral_constant<int, 3>{}); break;
      }
    } else switch (npv) {
      case 9: sweep(std::integral_constant<int, 9>{}); break;
      case 8: sweep(std::integral_constant<int, 8>{}); break;
      case 7: sweep(std::integral_constant<int, 7>{}); break;
      case 6: sweep(std::integral_constant<int, 6>{}); break;
      case 5: sweep(std::integral_constant<int, 5>{}); break;
      case 4: sweep(std::integral_constant<int, 4>{}); break;
      case 3: sweep(std::integral_constant<int, 3>{}); break;
      case 2: sweep(std::integral_constant<int, 2>{}); break;
      case 1: sweep(std::integral_constant<int, 1>{}); break;
      default: break;
    }
    ++since;
    const bool last = r0 + RC >= rb1;
    if (since % C::FOLD == 0 || last) {
#pragma unroll
      for (int q = 0; q < GI_PPW; ++q) {
#pragma unroll
        for (int i = 0; i < 4; ++i) { midL[wv][4 * q + i][lane] += acc[q][i]; acc[q][i] = 0.f; }
      }
    }
    if (since >= 64 * C::FOLD || last) {
#pragma unroll
      for (int q = 0; q < GI_PPW; ++q) {
        if (!pv[q]) continue;
        const int p = grp * (4 * GI_PPW) + slot + 4 * q;
        double* o = out + ((size_t)split * n_pairs + p) * 256;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          o[(4 * kr + i) * 16 + cc] += (double)midL[wv][4 * q + i][lane];  // D[i][j]: i = 4*(lane/16)+v, j = lane%16
          midL[wv][4 * q + i][lane] = 0.f;
        }
      }
      since = 0;
    }
    __syncthreads();
  }
  if (FUSED && grp == 0 && wv == 0) {
    dev = wave_sum(dev);
    if (lane == 0) dev_out[split] = dev;
  }
}


// ---------------------------------------------------------------------------
// Warp-specialised variant for padded widths <= 128 (the 100-column bench
// shape): 512-thread workgroups, waves 0-3 are MFMA consumers, waves 4-7 are
// producers.  LDS holds TWO 64-row chunks; while the consumers sweep chunk i
// the producers write chunk i+1 (loaded from HBM one iteration earlier, so a
// sweep of latency hiding; two chunks stay in flight), evaluate the family for their own 16 rows
// (each producer wave owns whole rows: eta is a pure in-wave shuffle reduce)
// and issue the loads of chunk i+3.  One barrier per chunk.  Consumers keep
// the MFMA accumulators in registers (f32 over <= 1024 rows) and fold them
// into the block's own f64 tile (no atomics, deterministic).
// ---------------------------------------------------------------------------
//
// Exact-gradient channel (FUSED + SQW, grad_out != nullptr): the producers
// also accumulate g = X' r with r = W (z - eta + offset) = w (y - mu) dmu/deta
// / var on the VALU as exact f64 products x r (an f32 x f32 product fits a
// double) summed in f64, folded into per-wave f64 LDS slots every chunk, and
// the block writes grad_out[split][PP + 1] (column PP = sum r, the intercept).
// f64 products matter for ill-conditioned designs: independent f32 product
// roundings of two near-collinear columns do not cancel along their weak
// difference direction, and the Newton step divides by that eigenvalue.
// The host then forms the IRLS right-hand side as G beta + g, so the Newton
// step beta + G^-1 g has an exact fixed point (g = 0) whatever the precision
// of the bf16x3 Hessian G: its precision only sets the convergence rate.
// Reference: hex/glm/GLMTask.java:1507 (GLMIterationTask, double _xy) and
// hex/gram/Gram.java:17 (double _xx).
// LO = false (with BF3): the one-MFMA bf16 Hessian tier -- no lo plane, one
// 16x16x32 MFMA per product instead of three (Newton on the exact gradient
// still converges to the exact-gradient fixed point; the tier is chosen from
// the condition number, glm.py _TIER_LIMITS)
template <int PP, bool FUSED, bool SQW, bool BF3, bool LO = true>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void glm_irls_ws_kernel(
    const float* __restrict__ X, long long N, int ldx, int n_pairs, int rows_per_block,
    const float* __restrict__ beta, float b0, const float* __restrict__ y, const float* __restrict__ wprior,
    const float* __restrict__ offset, GlmFamArgs fam, const float* __restrict__ Wext,
    const float* __restrict__ zext, int aug, double* __restrict__ out, double* __restrict__ dev_out,
    double* __restrict__ grad_out) {
  constexpr int RC = 64;
  constexpr int P4 = PP / 4;
  constexpr int T = PP / 16;
  constexpr int S = PP + ((16 - (PP % 64)) & 63);
  constexpr int RPW = 16;              // rows owned by one producer wave
  constexpr int NVP = RPW * P4 / 64;   // float4 per producer lane per chunk
  constexpr int RPV = 64 / P4;         // rows covered by one float4 slot of a wave
  static_assert(PP <= 128 && (PP & (PP - 1)) == 0, "ws kernel: power-of-two width <= 128");
  // BF3 LDS image: feature-major [feature][KS] bf16 hi and lo planes; the 64
  // chunk rows are permuted (producer wave pw, lane half par, slot v ->
  // k = 16 pw + 8 par + v) so each producer lane writes 8 rows of one feature
  // as one 16-byte store and each consumer lane reads its 16x16x32 operand
  // (8 consecutive k of one feature) as one ds_read_b128.  The 8-row k-blocks
  // of feature f sit XOR-swizzled at block (kb ^ swz(f)), swz(f) = (f ^ f>>2)
  // & 7, KS = 64: the 8 lanes of a ds_write_b128 group (8 consecutive
  // features) and the 16 lanes of a ds_read_b128 group (16 features x 2
  // k-blocks) land on distinct bank quads.  PMC with the padded KS = 72
  // layout: 6.35 bank-conflict cycles per LDS instruction (4-way on the
  // producer stores, 2-way on the operand reads).
  constexpr int KS = 64;
  static_assert(!BF3 || (PP == 128 && SQW), "bf16x3 path: P = 128, sqrt(W)-scaled rows");
  __shared__ float L[2][BF3 ? 4 : RC * S];
  __shared__ __attribute__((aligned(16))) __bf16 LB[2][LO ? 2 : 1][BF3 ? PP * KS : 8];
  __shared__ float wr[2][RC];
  __shared__ double dsum[4];
  // P = 128 producer scratch: eta partials [wave][row 16][quad 8] and the
  // per-row sqrt(W) [wave][16] (replaces 48 + 8 ds_bpermute per chunk)
  constexpr bool QRED = P4 == 32;
  __shared__ __attribute__((aligned(16))) float es[QRED ? 4 : 1][QRED ? 128 : 4];
  __shared__ __attribute__((aligned(16))) float sqs[QRED ? 4 : 1][QRED ? 16 : 4];
  // exact-gradient channel: per producer lane 4 f64 feature slots, per wave the
  // per-row residuals r laid out like sqs
  constexpr bool GRAD = FUSED && SQW;
  __shared__ __attribute__((aligned(16))) double gs[GRAD ? 4 : 1][GRAD ? P4 : 1][GRAD ? 4 : 1];
  __shared__ __attribute__((aligned(16))) float rqs[GRAD ? 4 : 1][GRAD ? 16 : 4];
  __shared__ double gsum_s[4];
  const bool want_grad = GRAD && grad_out != nullptr;
  const int split = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const long long rb0 = (long long)split * rows_per_block;
  const long long rb1 = min(N, rb0 + rows_per_block);
  const int nchunks = rb1 > rb0 ? (int)((rb1 - rb0 + RC - 1) / RC) : 0;

  if (wv >= 4) {
    // ============================ producers ============================
    const int pw = wv - 4;
    const int cq = lane % P4;
    f32x4 b4 = {0.f, 0.f, 0.f, 0.f};
    if (FUSED) b4 = *reinterpret_cast<const f32x4*>(beta + 4 * cq);
    struct Stage {
      f32x4 V[NVP];
      float sy, sw, so;
    };
    // non-fused: two chunks in flight per producer lane; fused keeps one (the
    // eta / family registers would otherwise spill at the 128-VGPR budget)
    constexpr bool DEEP = !FUSED;
    Stage A, B;
    double dev = 0.0;
    double gsum = 0.0;   // lanes < 16: sum of r over this wave's rows (intercept gradient)
    if (want_grad && lane < P4) {
#pragma unroll
      for (int e = 0; e < 4; ++e) gs[pw][lane][e] = 0.0;
    }
    // exact-gradient channel: the lane's NVP rows (row v RPV + lane / P4) times
    // its 4 features as exact f64 products (f32 x f32 fits a double), summed in
    // f64 over the lanes holding the same features, folded into LDS by lanes < P4
    auto grad_acc = [&](const f32x4* V, float rres, bool qred) __attribute__((always_inline)) {
      float rv[NVP];
      if (QRED && qred) {
        float* Q = rqs[pw];
        if (lane < RPW) Q[(lane & 1) * 8 + (lane >> 1)] = rres;
        const int par = lane / P4;
        const f32x4 q0 = *reinterpret_cast<const f32x4*>(Q + par * 8);
        const f32x4 q1 = *reinterpret_cast<const f32x4*>(Q + par * 8 + 4);
        rv[0] = q0.x; rv[1] = q0.y; rv[2] = q0.z; rv[3] = q0.w;
        rv[4] = q1.x; rv[5] = q1.y; rv[6] = q1.z; rv[7] = q1.w;
      } else {
#pragma unroll
        for (int v = 0; v < NVP; ++v) rv[v] = __shfl(rres, v * RPV + lane / P4, 64);
      }
      if (fam.grad_f64) {
        // exact products: ill-conditioned designs (the f32 / f64 Hessian tiers)
        double a[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = 0.0;
#pragma unroll
          for (int v = 0; v < NVP; ++v) a[e] = fma((double)V[v][e], (double)rv[v], a[e]);
        }
#pragma unroll
        for (int o = P4; o < 64; o <<= 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) a[e] += __shfl_xor(a[e], o, 64);
        }
        if (lane < P4) {
#pragma unroll
          for (int e = 0; e < 4; ++e) gs[pw][lane][e] += a[e];
        }
      } else {
        // f32 products over the lane's rows of the chunk, f64 beyond (the
        // bf16x3 tier: condition number < 2e3, product rounding is harmless)
        float a[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = 0.f;
#pragma unroll
          for (int v = 0; v < NVP; ++v) a[e] = fmaf(V[v][e], rv[v], a[e]);
        }
#pragma unroll
        for (int o = P4; o < 64; o <<= 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) a[e] += __shfl_xor(a[e], o, 64);
        }
        if (lane < P4) {
#pragma unroll
          for (int e = 0; e < 4; ++e) gs[pw][lane][e] += (double)a[e];
        }
      }
    };
    auto load = [&](int c, Stage& st) {
      f32x4* V = st.V;
      float& sy = st.sy;
      float& sw = st.sw;
      float& so = st.so;
      const long long r0 = rb0 + (long long)c * RC + pw * RPW;
      if (fam.dbg & 2) {
#pragma unroll
        for (int v = 0; v < NVP; ++v) V[v] = f32x4{0.f, 0.f, 0.f, (float)c};
      } else {
        // X rows are ldx floats (ldx <= PP, ldx % 4 == 0): the PP - ldx
        // padding columns never leave HBM, their lanes stage zeros
        const bool live = 4 * cq < ldx;
#pragma unroll
        for (int v = 0; v < NVP; ++v) {
          const long long g = min(r0 + v * RPV + lane / P4, N - 1);
          V[v] = live ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(X + g * (long long)ldx) + cq)
                      : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      if (lane < RPW && (fam.dbg & 4)) {
        sy = 0.f; sw = 1.f; so = 0.f;
      } else if (lane < RPW) {
        const long long g = min(r0 + lane, N - 1);
        if (FUSED) {
          sy = y[g];
          sw = wprior ? wprior[g] : 1.f;
          so = offset ? offset[g] : 0.f;
        } else {
          sw = Wext ? Wext[g] : 1.f;
          sy = zext ? zext[g] : 0.f;
        }
      }
    };
    auto store = [&](int c, Stage& st) {
      const f32x4* V = st.V;
      const float sy = st.sy, sw = st.sw, so = st.so;
      float* Lb = L[c & 1];
      float etav = 0.f;
      const bool qred = QRED && !(fam.dbg & 16);
      if (FUSED && qred) {
        if (!(fam.dbg & 8)) {
          // lane-local 4-feature dot products of its 8 rows, quad sums by DPP,
          // then the 8 quad partials of a row meet in LDS: row j's lane (< 16)
          // reads them back as two b128 (eta lands where the family runs)
          float ps[NVP];
#pragma unroll
          for (int v = 0; v < NVP; ++v) ps[v] = V[v].x * b4.x + V[v].y * b4.y + V[v].z * b4.z + V[v].w * b4.w;
#pragma unroll
          for (int v = 0; v < NVP; ++v) ps[v] += gi_dpp<0xB1>(ps[v]);
#pragma unroll
          for (int v = 0; v < NVP; ++v) ps[v] += gi_dpp<0x4E>(ps[v]);
          const int r = lane & 3, q = (lane >> 2) & 7, par = lane >> 5;
          float* S = es[pw];
#pragma unroll
          for (int m = 0; m < NVP / 4; ++m) {
            const float val = r == 0 ? ps[4 * m] : r == 1 ? ps[4 * m + 1] : r == 2 ? ps[4 * m + 2] : ps[4 * m + 3];
            S[(2 * (r + 4 * m) + par) * 8 + q] = val;
          }
          if (lane < RPW) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(S + lane * 8);
            const f32x4 b = *reinterpret_cast<const f32x4*>(S + lane * 8 + 4);
            etav = (a.x + a.y) + (a.z + a.w) + ((b.x + b.y) + (b.z + b.w));
          }
        }
      } else if (FUSED && !(fam.dbg & 8)) {
#pragma unroll
        for (int v = 0; v < NVP; ++v) {
          float sdot = V[v].x * b4.x + V[v].y * b4.y + V[v].z * b4.z + V[v].w * b4.w;
#pragma unroll
          for (int o = P4 / 2; o > 0; o >>= 1) sdot += __shfl_xor(sdot, o, 64);
          // lane j (< 16) collects the eta of its row j = v*RPV + src/P4
          const float got = __shfl(sdot, (lane % RPV) * P4, 64);
          if (lane / RPV == v) etav = got;
        }
      }
      float W = 0.f, z = 0.f, rres = 0.f;
      if (lane < RPW) {
        const long long r = rb0 + (long long)c * RC + pw * RPW + lane;
        if (r < rb1) {
          if (FUSED) {
            const float eta = etav + b0 + so;
            const float mu = gi_linkinv(fam.link, eta);
            if (fam.link == 0 && fam.var == 0) {
              W = sw;
              z = sy - so;
              rres = sw * (sy - eta);
              if (sw != 0.f) dev += (double)(sw * gi_dev(fam, sy, mu));
            } else if (fam.link == 1 && fam.var == 1) {
              // canonical binomial: dmu/deta == variance, so W = w d and one
              // reciprocal; 0/1 responses need one log for the deviance
              const float d = fmaxf(mu * (1.f - mu), 1e-10f);
              W = sw * d;
              z = (eta - so) + (sy - mu) * __frcp_rn(d);
              rres = sw * (sy - mu);
              if (sw != 0.f) {
                const float m = fminf(fmaxf(mu, 1e-15f), 1.f - 1e-7f);
                const float dv = sy == 1.f ? -2.f * __logf(m) : sy == 0.f ? -2.f * __logf(1.f - m)
                                                                         : gi_dev(fam, sy, mu);
                dev += (double)(sw * dv);
              }
            } else {
              const float d = gi_dmu(fam.link, mu);
              const float wd = sw * d / gi_var(fam, mu);
              W = wd * d;
              z = (eta - so) + (sy - mu) / d;
              rres = wd * (sy - mu);
              if (sw != 0.f) dev += (double)(sw * gi_dev(fam, sy, mu));
            }
          } else {
            W = sw;
            z = sy;
          }
        }
        if (want_grad) gsum += (double)rres;
      }
      // SQW: rows are staged pre-scaled by sqrt(W) so the consumers' MFMA
      // operands come straight from LDS (no VALU between LDS and MFMA)
      const float sq = SQW ? sqrtf(fmaxf(W, 0.f)) : 1.f;
      if constexpr (BF3) {
        __bf16* Hb = LB[c & 1][0];
        __bf16* Lb2 = LB[c & 1][LO ? 1 : 0];
        const int par = lane / P4;
        // row j = 2 v + par: lanes < 16 publish sqrt(W) as [par][v], every
        // lane reads its 8 rows' factors as two broadcast b128
        float sv[NVP];
        if (qred) {
          float* Q = sqs[pw];
          if (lane < RPW) Q[(lane & 1) * 8 + (lane >> 1)] = sq;
          const f32x4 q0 = *reinterpret_cast<const f32x4*>(Q + par * 8);
          const f32x4 q1 = *reinterpret_cast<const f32x4*>(Q + par * 8 + 4);
          sv[0] = q0.x; sv[1] = q0.y; sv[2] = q0.z; sv[3] = q0.w;
          sv[4] = q1.x; sv[5] = q1.y; sv[6] = q1.z; sv[7] = q1.w;
        } else {
#pragma unroll
          for (int v = 0; v < NVP; ++v) sv[v] = __shfl(sq, v * RPV + par, 64);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bf16x8 h, l;
#pragma unroll
          for (int v = 0; v < NVP; ++v) {
            const float x = V[v][e] * sv[v];
            const __bf16 hb = (__bf16)x;
            h[v] = hb;
            if constexpr (LO) l[v] = (__bf16)(x - (float)hb);
          }
          const int f = 4 * cq + e;
          const int off = f * KS + (((2 * pw + par) ^ gi_swz(f)) << 3);
          *reinterpret_cast<bf16x8*>(Hb + off) = h;
          if constexpr (LO) *reinterpret_cast<bf16x8*>(Lb2 + off) = l;
        }
        if constexpr (GRAD) {
          if (want_grad) grad_acc(V, rres, qred);   // after the bf16 stores: the sqrt(W) factors are dead
        }
        if (lane < RPW && aug >= 0) {
          const int k = pw * RPW + (lane % RPV) * 8 + lane / RPV;
          const float a0 = sq, a1 = sq * z;
          const __bf16 h0 = (__bf16)a0, h1 = (__bf16)a1;
          const int k0 = aug * KS + ((((k >> 3) ^ gi_swz(aug)) << 3) | (k & 7));
          const int k1 = (aug + 1) * KS + ((((k >> 3) ^ gi_swz(aug + 1)) << 3) | (k & 7));
          Hb[k0] = h0;
          Hb[k1] = h1;
          if constexpr (LO) {
            Lb2[k0] = (__bf16)(a0 - (float)h0);
            Lb2[k1] = (__bf16)(a1 - (float)h1);
          }
        }
        return;
      }
#pragma unroll
      for (int v = 0; v < NVP; ++v) {
        const int rl = pw * RPW + v * RPV + lane / P4;
        f32x4 val = V[v];
        if (SQW) val *= __shfl(sq, v * RPV + lane / P4, 64);
        *reinterpret_cast<f32x4*>(Lb + rl * S + 4 * cq) = val;
      }
      if constexpr (GRAD) {
        if (want_grad) grad_acc(V, rres, qred);
      }
      if (lane < RPW) {
        const int rl = pw * RPW + lane;
        if (!SQW) wr[c & 1][rl] = W;
        if (aug >= 0) {
          Lb[rl * S + aug] = sq;
          Lb[rl * S + aug + 1] = sq * z;
        }
      }
    };
    if (nchunks > 0) {
      load(0, A);
      store(0, A);
      if (nchunks > 1) load(1, A);
      if (DEEP && nchunks > 2) load(2, B);
    }
    __syncthreads();
    // iteration i stores chunk i+1 (stage A for even i, B for odd) and
    // refills that stage with chunk i+3: two chunks always in flight
    for (int i = 0; i < nchunks; ++i) {
      if (!DEEP) {
        if (i + 1 < nchunks) {
          store(i + 1, A);
          if (i + 2 < nchunks) load(i + 2, A);
        }
      } else if (i + 1 < nchunks) {
        if ((i & 1) == 0) {
          store(i + 1, A);
          if (i + 3 < nchunks) load(i + 3, A);
        } else {
          store(i + 1, B);
          if (i + 3 < nchunks) load(i + 3, B);
        }
      }
      __syncthreads();
    }
    if (FUSED) {
      dev = wave_sum(dev);
      if (lane == 0) dsum[pw] = dev;
    }
    if (want_grad) {
      gsum = wave_sum(gsum);
      if (lane == 0) gsum_s[pw] = gsum;
    }
    __syncthreads();
    if (FUSED && threadIdx.x == 256) dev_out[split] = dsum[0] + dsum[1] + dsum[2] + dsum[3];
    if constexpr (GRAD) {
      if (want_grad) {
        // feature f = 4 cq + e: slot [cq][e] of every producer wave
        const int t = threadIdx.x - 256;
        if (t < PP) {
          const int cq2 = t >> 2, e = t & 3;
          const double g = (gs[0][cq2][e] + gs[1][cq2][e]) + (gs[2][cq2][e] + gs[3][cq2][e]);
          grad_out[(size_t)split * (PP + 1) + t] = g;
        } else if (t == PP) {
          grad_out[(size_t)split * (PP + 1) + PP] = gsum_s[0] + gsum_s[1] + gsum_s[2] + gsum_s[3];
        }
      }
    }
  } else {
    // ============================ consumers ============================
    const int slot = __builtin_amdgcn_readfirstlane((wv + split) & 3);
    const int kr = lane >> 4, cc = lane & 15;
    f32x4 acc[GI_PPW];
#pragma unroll
    for (int q = 0; q < GI_PPW; ++q) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[q][e] = 0.f;
    }
    auto flush = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < GI_PPW; ++q) {
        const int p = slot + 4 * q;
        if (p < n_pairs) {
          double* o = out + ((size_t)split * n_pairs + p) * 256;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[(4 * kr + e) * 16 + cc] += (double)acc[q][e];
            acc[q][e] = 0.f;
          }
        }
      }
    };
    // the slot switch sits OUTSIDE the chunk loop (one register assignment for
    // the accumulators); operands of k-step k+1 are loaded from LDS before the
    // MFMAs of step k are issued (register double-buffer)
    auto run = [&](auto slot_tag) __attribute__((always_inline)) {
      constexpr int SL = decltype(slot_tag)::value;
      __syncthreads();
      for (int i = 0; i < nchunks; ++i) {
        const float* Lb = L[i & 1] + kr * S + cc;
        const float* wb = wr[i & 1] + kr;
        if constexpr (BF3) {
          if (!(fam.dbg & 1)) {
            const __bf16* Hb = LB[i & 1][0];
            const __bf16* Lo = LB[i & 1][LO ? 1 : 0];
            // feature f = 16 t + cc, k-block kr + 4 ks: gi_swz(f) = s0 ^ 4 (t & 1)
            // with s0 = gi_swz(cc), so the swizzled offset is one of two
            // per-lane bases (k-block bit 2 flipped by ks ^ t) + 16 t KS
            const int s0 = gi_swz(cc);
            const int B0 = cc * KS + ((kr ^ s0) << 3);
            const int B1 = B0 ^ 32;
#pragma unroll 1
            for (int ks = 0; ks < RC / 32; ++ks) {
              bf16x8 ah[T], al[T];
              const int Be = ks ? B1 : B0, Bo = ks ? B0 : B1;
#pragma unroll
              for (int t = 0; t < T; ++t) {
                const int off = 16 * t * KS + ((t & 1) ? Bo : Be);
                ah[t] = *reinterpret_cast<const bf16x8*>(Hb + off);
                if constexpr (LO) al[t] = *reinterpret_cast<const bf16x8*>(Lo + off);
              }
              if constexpr (LO) gi_mfma3_all<T, SL>(std::make_integer_sequence<int, GI_PPW>{}, ah, al, acc);
              else gi_mfma1_all<T, SL>(std::make_integer_sequence<int, GI_PPW>{}, ah, acc);
            }
          }
        } else if (!(fam.dbg & 1)) {
          float xr[T], xn[T], xw[T];
          float w = SQW ? 1.f : wb[0];
#pragma unroll
          for (int t = 0; t < T; ++t) xr[t] = Lb[16 * t];
#pragma unroll 2
          for (int k = 0; k < RC / 4; ++k) {
            const int kn = k + 1 < RC / 4 ? k + 1 : k;
            const float wn = SQW ? 1.f : wb[4 * kn];
#pragma unroll
            for (int t = 0; t < T; ++t) xn[t] = Lb[4 * kn * S + 16 * t];
            if (SQW) {
              gi_mfma_all<T, SL>(std::make_integer_sequence<int, GI_PPW>{}, xr, xr, acc);
            } else {
#pragma unroll
              for (int t = 0; t < T; ++t) xw[t] = w * xr[t];
              gi_mfma_all<T, SL>(std::make_integer_sequence<int, GI_PPW>{}, xr, xw, acc);
            }
#pragma unroll
            for (int t = 0; t < T; ++t) xr[t] = xn[t];
            w = wn;
          }
        }
        if ((i & 15) == 15 || i + 1 == nchunks) flush();  // f32 over <= 1024 rows, then f64
        __syncthreads();
      }
    };
    switch (slot) {
      case 0: run(std::integral_constant<int, 0>{}); break;
      case 1: run(std::integral_constant<int, 1>{}); break;
      case 2: run(std::integral_constant<int, 2>{}); break;
      default: run(std::integral_constant<int, 3>{}); break;
    }
    __syncthreads();
  }
}

template <int PP>
static void gi_launch(bool fused, dim3 grid, hipStream_t s, const float* X, long long N, int ldx, const int2* pairs,
                      int n_pairs, int rpb, const float* beta, float b0, const float* y, const float* wprior,
                      const float* offset, GlmFamArgs fam, const float* Wext, const float* zext, int aug,
                      double* out, double* dev_out, double* grad_out) {
  if constexpr (PP <= 128 && (PP & (PP - 1)) == 0) {
    // IRLS weights are >= 0 -> sqrt(W) pre-scaling; caller-signed weights
    // (e.g. X'r for lambda_max) take the explicit-multiply path
    if constexpr (PP == 128) {
      if (fam.bf3 == 2 && !fam.signed_w && fused) {
        // plain-bf16 Hessian tier (needs the exact gradient channel)
        hipLaunchKernelGGL((glm_irls_ws_kernel<PP, true, true, true, false>), dim3(grid.x), dim3(512), 0, s, X, N,
                           ldx, n_pairs, rpb, beta, b0, y, wprior, offset, fam, Wext, zext, aug, out, dev_out,
                           grad_out);
        return;
      }
      if (fam.bf3 && !fam.signed_w) {
        if (fused)
          hipLaunchKernelGGL((glm_irls_ws_kernel<PP, true, true, true>), dim3(grid.x), dim3(512), 0, s, X, N, ldx,
                             n_pairs, rpb, beta, b0, y, wprior, offset, fam, Wext, zext, aug, out, dev_out, grad_out);
        else
          hipLaunchKernelGGL((glm_irls_ws_kernel<PP, false, true, true>), dim3(grid.x), dim3(512), 0, s, X, N, ldx,
                             n_pairs, rpb, beta, b0, y, wprior, offset, fam, Wext, zext, aug, out, dev_out, nullptr);
        return;
      }
    }
    if (fused)
      hipLaunchKernelGGL((glm_irls_ws_kernel<PP, true, true, false>), dim3(grid.x), dim3(512), 0, s, X, N, ldx, n_pairs,
                         rpb, beta, b0, y, wprior, offset, fam, Wext, zext, aug, out, dev_out, grad_out);
    else if (!fam.signed_w)
      hipLaunchKernelGGL((glm_irls_ws_kernel<PP, false, true, false>), dim3(grid.x), dim3(512), 0, s, X, N, ldx, n_pairs,
                         rpb, beta, b0, y, wprior, offset, fam, Wext, zext, aug, out, dev_out, nullptr);
    else
      hipLaunchKernelGGL((glm_irls_ws_kernel<PP, false, false, false>), dim3(grid.x), dim3(512), 0, s, X, N, ldx, n_pairs,
                         rpb, beta, b0, y, wprior, offset, fam, Wext, zext, aug, out, dev_out, nullptr);
    return;
  }
  if constexpr (GiCfg<PP>::POW2) {
    if (fused) {
      hipLaunchKernelGGL((glm_irls_kernel<PP, true>), grid, dim3(256), 0, s, X, N, pairs, n_pairs, rpb, beta, b0, y,
                         wprior, offset, fam, Wext, zext, aug, out, dev_out);
      return;
    }
  }
  hipLaunchKernelGGL((glm_irls_kernel<PP, false>), grid, dim3(256), 0, s, X, N, pairs, n_pairs, rpb, beta, b0, y,
                     wprior, offset, fam, Wext, zext, aug, out, dev_out);
}

// H2O3_GLM_BF3: 1 (default) bf16x3 MFMA for the P = 128 ws path, 0 f32 MFMA
// (read per call: one getenv per IRLS pass; a caller's bf3 >= 0 overrides it)
static int gi_bf3() {
  const char* e = getenv("H2O3_GLM_BF3");
  return e ? atoi(e) : 1;
}

static int gi_dbg() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("H2O3_GI_DBG");
    v = e ? atoi(e) : 0;
  }
  return v;
}

// rows_per_block must be a multiple of h2o_glm_irls_chunk(P).
extern "C" int h2o_glm_irls_chunk(int P) {
  const int r = (8192 / P) / 4 * 4;
  return P <= 128 ? 64 : (r < 16 ? 16 : r);
}

extern "C" int h2o_glm_irls(const float* X, long long N, int P, int ldx, const int* pairs, int n_pairs, int n_splits,
                            int rows_per_block, const float* beta, float b0, const float* y, const float* wprior,
                            const float* offset, int link, int var, float tvp, float theta, const float* Wext,
                            const float* zext, int aug, int signed_w, double* out, double* dev_out,
                            double* grad_out, int bf3, int grad_f64, hipStream_t s) {
  if (N <= 0 || n_pairs <= 0) return 0;
  if (P % 32 != 0 || P > 512) return -1;
  // narrow row storage (ldx < P) only on the warp-specialised path
  if (ldx % 4 != 0 || ldx > P || (ldx < P && (P > 128 || (P & (P - 1)) != 0))) return -5;
  if (aug >= 0 && aug + 1 >= P) return -2;
  if (beta && (P & (P - 1)) != 0) return -3;
  if (rows_per_block % h2o_glm_irls_chunk(P) != 0) return -4;
  const int groups = (n_pairs + 4 * GI_PPW - 1) / (4 * GI_PPW);
  dim3 grid(n_splits, groups);
  GlmFamArgs fam{link, var, tvp, theta, gi_dbg(), signed_w, bf3 < 0 ? gi_bf3() : bf3, grad_f64};
  if (fam.bf3 == 2 && !grad_out) fam.bf3 = 1;   // the plain-bf16 Hessian only beside the exact gradient
  const bool fused = beta != nullptr;
  // the exact-gradient channel rides the fused ws kernel (P <= 128, power of
  // two) only (grad_out: [n_splits][P + 1] doubles)
  if (grad_out && !(fused && P <= 128 && (P & (P - 1)) == 0 && !signed_w)) return -6;
  const int2* pr = (const int2*)pairs;
#define GI_CASE(pp)                                                                                          \
  case pp:                                                                                                   \
    gi_launch<pp>(fused, grid, s, X, N, ldx, pr, n_pairs, rows_per_block, beta, b0, y, wprior, offset, fam, Wext, \
                  zext, aug, out, dev_out, grad_out);                                                        \
    break;
  switch (P) {
    GI_CASE(32) GI_CASE(64) GI_CASE(96) GI_CASE(128) GI_CASE(160) GI_CASE(192) GI_CASE(224) GI_CASE(256)
    GI_CASE(288) GI_CASE(320) GI_CASE(352) GI_CASE(384) GI_CASE(416) GI_CASE(448) GI_CASE(480) GI_CASE(512)
    default: return -1;
  }
#undef GI_CASE
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Wide GLMs (P > 512): one streaming pass turns the augmented, sqrt(W)-scaled
// rows a = sqrt(W) [x | 1 | z | 0 ...] (Pa columns) into bf16 hi / lo halves
// stored side by side, HL[r] = [hi(a) | lo(a)] (row stride 2 Pa).  The Gram
// then needs ONE library GEMM: C = hi^T [hi | lo] (bf16 in, f32 out) holds
// hi'hi and hi'lo, and lo'hi = (hi'lo)^T by symmetry, so
// G = C[:, :Pa] + C[:, Pa:] + C[:, Pa:]^T -- two bf16 GEMM blocks per Gram
// instead of one f32 GEMM at 1/16 of the bf16 matrix rate (lo*lo, ~2^-16
// relative, is dropped).  One thread per 4 columns of a row: a float4 load,
// two 8-byte stores.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void gram_split_kernel(const float* __restrict__ X, int ldx, int P, int Pa,
                                                         const float* __restrict__ W, const float* __restrict__ z,
                                                         long long rows, __bf16* __restrict__ HL) {
  const int q4 = Pa / 4;
  const long long total = rows * q4;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const long long r = t / q4;
    const int c = (int)(t - r * q4) * 4;
    const float s = sqrtf(fmaxf(W ? W[r] : 1.f, 0.f));
    f32x4 v;
    if (c + 3 < P && (ldx & 3) == 0) {
      v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(X + r * ldx + c));
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int cc = c + e;
        v[e] = cc < P ? X[r * ldx + cc] : cc == P ? 1.f : (cc == P + 1 && z) ? z[r] : 0.f;
      }
    }
    bf16x4 h, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = v[e] * s;
      h[e] = (__bf16)a;
      l[e] = (__bf16)(a - (float)h[e]);
    }
    __bf16* o = HL + r * (2LL * Pa) + c;
    *reinterpret_cast<bf16x4*>(o) = h;
    *reinterpret_cast<bf16x4*>(o + Pa) = l;
  }
}

extern "C" int h2o_gram_split(const float* X, int ldx, int P, int Pa, const float* W, const float* z,
                              long long rows, void* HL, hipStream_t s) {
  if (rows <= 0) return 0;
  if (Pa % 4 != 0 || Pa < P + 2 || ldx < P) return -1;
  const long long work = rows * (Pa / 4);
  const int grid = (int)std::min<long long>((work + 255) / 256, 256LL * 64);
  hipLaunchKernelGGL(gram_split_kernel, dim3(grid), dim3(256), 0, s, X, ldx, P, Pa, W, z, rows, (__bf16*)HL);
  return (int)hipGetLastError();
}

// Fused wide IRLS pass: one wave per row (the row's Pa <= 1024 columns sit in
// 16 registers per lane), eta = x.beta by a wave reduction, the family's
// IRLS weight / working response / deviance on every lane (wave-uniform), and
// the [hi | lo] split of sqrt(W) [x | 1 | z] -- X is read from HBM once per
// IRLS iteration; the library GEMM that follows reads only the bf16 halves.
// Deviance: one f64 partial per block (deterministic; the host sums).
#define WIDE_GFOLD 64
template <int NQ, int RW, bool HASHL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RW == 1 ? 4 : 1))) void glm_wide_split_kernel(
    const float* __restrict__ X, int ldx, int P, int Pa, long long rows, const float* __restrict__ beta, float b0,
    const float* __restrict__ y, const float* __restrict__ wprior, const float* __restrict__ offset,
    GlmFamArgs fam, __bf16* __restrict__ HL, double* __restrict__ dev_out, double* __restrict__ grad_out,
    float* __restrict__ wout) {
  // HL null: no bf16 planes; wout[r] = the row's IRLS weight instead (the
  // fused wide Gram kernel below reads X and these weights).
  // grad_out (optional): [gridDim.x][Pa] f64, this block's slot += X' r over
  // its rows of the chunk (r = w (y - mu) dmu/deta / var: the exact-gradient
  // channel, see glm_irls_ws_kernel); column P holds sum r.  Each lane's f32
  // products are folded into its own f64 LDS slots every WIDE_GFOLD rows, so
  // one launch can sweep any number of rows at the stated precision.
  __shared__ double dsum[4];
  __shared__ double gsh[4][NQ * 256];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  if (grad_out) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) gsh[wv][4 * (lane + 64 * q) + e] = 0.0;
  }
  int since = 0;
  f32x4 b[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int c = 4 * (lane + 64 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) b[q][e] = c + e < P ? beta[c + e] : 0.f;
  }
  double dev = 0.0;
  f32x4 ga[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) ga[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gi = 0.f;
  // RW consecutive rows per wave per step: their loads are all issued before
  // the first dot-product reduction (RW x 4 KB in flight per wave instead of
  // one row, whose reduction and family math stalled the next row's loads)
  const long long nw = (long long)gridDim.x * 4 * RW;
  for (long long r0 = ((long long)blockIdx.x * 4 + wv) * RW; r0 < rows; r0 += nw) {
    f32x4 v[RW][NQ];
    float dot[RW];
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      const long long r = r0 + j < rows ? r0 + j : rows - 1;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int c = 4 * (lane + 64 * q);
        if (c + 3 < P) {
          v[j][q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(X + r * ldx + c));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[j][q][e] = c + e < P ? X[r * ldx + c + e] : 0.f;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      dot[j] = 0.f;
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        dot[j] += v[j][q].x * b[q].x + v[j][q].y * b[q].y + v[j][q].z * b[q].z + v[j][q].w * b[q].w;
    }
#pragma unroll
    for (int j = 0; j < RW; ++j) dot[j] = wave_sum(dot[j]);
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      const long long r = r0 + j;
      if (r >= rows) break;
      const float sy = y[r], sw = wprior ? wprior[r] : 1.f, so = offset ? offset[r] : 0.f;
      const float eta = dot[j] + b0 + so;
      const float mu = gi_linkinv(fam.link, eta);
      float W, z, rres;
      if (fam.link == 0 && fam.var == 0) {
        W = sw;
        z = sy - so;
        rres = sw * (sy - eta);
      } else {
        const float d = gi_dmu(fam.link, mu);
        const float wd = sw * d / gi_var(fam, mu);
        W = wd * d;
        z = (eta - so) + (sy - mu) / d;
        rres = wd * (sy - mu);
      }
      if (lane == 0 && sw != 0.f) dev += (double)(sw * gi_dev(fam, sy, mu));
      if (grad_out) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) ga[q] += v[j][q] * rres;
        gi += rres;
        if (++since == WIDE_GFOLD) {
          since = 0;
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const int c = 4 * (lane + 64 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e) gsh[wv][c + e] += (double)(c + e == P ? gi : ga[q][e]);
            ga[q] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
          gi = 0.f;
        }
      }
      if constexpr (!HASHL) {
        if (lane == 0) wout[r] = fmaxf(W, 0.f);
        continue;
      }
      const float s = sqrtf(fmaxf(W, 0.f));
      __bf16* o = HL + r * (2LL * Pa);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int c = 4 * (lane + 64 * q);
        if (c >= Pa) break;
        f32x4 a = v[j][q];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (c + e == P) a[e] = 1.f;
          if (c + e == P + 1) a[e] = z;
        }
        bf16x4 h, l;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float t = a[e] * s;
          h[e] = (__bf16)t;
          l[e] = (__bf16)(t - (float)h[e]);
        }
        *reinterpret_cast<bf16x4*>(o + c) = h;
        *reinterpret_cast<bf16x4*>(o + Pa + c) = l;
      }
    }
  }
  dev = wave_sum(dev);
  if (lane == 0) dsum[wv] = dev;
  if (grad_out) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int c = 4 * (lane + 64 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) gsh[wv][c + e] += (double)(c + e == P ? gi : ga[q][e]);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) dev_out[blockIdx.x] = dsum[0] + dsum[1] + dsum[2] + dsum[3];
  if (grad_out) {
    for (int c = threadIdx.x; c < Pa; c += 256)
      grad_out[(size_t)blockIdx.x * Pa + c] +=
          (gsh[0][c] + gsh[1][c]) + (gsh[2][c] + gsh[3][c]);
  }
}

// Workgroups that fill the chip once for the weight-only pass (resident
// blocks per CU x CUs): a grid of whole rounds, no partial last round.
extern "C" int h2o_glm_wide_split_grid(int Pa) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  const void* k = Pa <= 256 ? (const void*)glm_wide_split_kernel<1, 1, false>
                  : Pa <= 512 ? (const void*)glm_wide_split_kernel<2, 1, false>
                              : (const void*)glm_wide_split_kernel<4, 1, false>;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, 0) != hipSuccess) return 0;
  return per_cu * cus;
}

// Pa <= 1024 (P <= 1022), Pa % 4 == 0; dev_out holds `blocks` doubles.
#ifndef WIDE_RW
#define WIDE_RW 1
#endif
extern "C" int h2o_glm_wide_split(const float* X, int ldx, int P, int Pa, long long rows, const float* beta, float b0,
                                  const float* y, const float* wprior, const float* offset, int link, int var,
                                  float tvp, float theta, void* HL, double* dev_out, int blocks, double* grad_out,
                                  float* wout, hipStream_t s) {
  if (rows <= 0) return 0;
  if (Pa % 4 != 0 || Pa < P + 2 || ldx < P || blocks <= 0 || (!HL && !wout)) return -1;
  GlmFamArgs fam{link, var, tvp, theta, 0, 0, 0, 0};
#define WIDE_SPLIT(NQ, RW, H)                                                                                    \
  hipLaunchKernelGGL((glm_wide_split_kernel<NQ, RW, H>), dim3(blocks), dim3(256), 0, s, X, ldx, P, Pa, rows, beta, \
                     b0, y, wprior, offset, fam, (__bf16*)HL, dev_out, grad_out, wout)
  if (HL) {
    if (Pa <= 256) WIDE_SPLIT(1, 2, true);
    else if (Pa <= 512) WIDE_SPLIT(2, 2, true);
    else if (Pa <= 1024) WIDE_SPLIT(4, 2, true);
    else return -2;
  } else {
    // weight-only pass of the fused wide IRLS: rows in flight per wave
    // (H2O3_WIDE_RW = 1 / 2 / 4, default WIDE_RW; at 12.5M x 1000 the pass
    // takes 10.5 / 12.5 / 12.4 ms: more rows per wave lowers occupancy
    // (129 -> 155 -> 195 VGPRs) and does not raise the read rate)
    static const int rw = getenv("H2O3_WIDE_RW") ? atoi(getenv("H2O3_WIDE_RW")) : WIDE_RW;
    if (Pa <= 256) WIDE_SPLIT(1, 1, false);
    else if (Pa <= 512) WIDE_SPLIT(2, 1, false);
    else if (Pa > 1024) return -2;
    else if (rw == 1) WIDE_SPLIT(4, 1, false);
    else if (rw == 4) WIDE_SPLIT(4, 4, false);
    else WIDE_SPLIT(4, 2, false);
  }
#undef WIDE_SPLIT
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused wide weighted Gram: C = [X | 1]' diag(w) [X | 1] straight from the
// f32 rows of X (no bf16 planes in HBM, no library GEMM).
//
// Tiles: 128 x 128 blocks (bi <= bj) of the (NB*128)^2 Gram, column P is the
// intercept's 1, columns past it are 0.  A workgroup owns one tile pair and
// one row slice: chunks of 64 rows c = s, s + S, s + 2S, ...  The npairs
// workgroups of a slice are consecutive logical ids after the XCD remap, so
// they run on one XCD at the same time and read each 64-row chunk of X from
// HBM once, then from that XCD's L2.
//
// Per chunk every thread loads eight 8-row column vectors (coalesced: a wave
// reads 64 consecutive columns of one row per load), scales the A panel by
// the row weights, splits x = hi + lo (bf16) and stores them k-contiguous in
// LDS ([column][row], pitch 72 bf16: conflict-free b128 operand reads); the
// next chunk's loads are issued before this chunk's MFMAs.  Each wave owns a
// 64 x 64 quarter of the tile: 16 accumulators of v_mfma_f32_16x16x32_bf16,
// three MFMAs per product (hi hi + hi lo + lo hi, the lo lo term ~2^-16
// relative dropped).  The f32 accumulators are folded into the workgroup's
// own f64 slot every `fold` chunks (64 K rows at fold 1024) and at the end;
// the host sums the slices in f64.
// ---------------------------------------------------------------------------
#define WG_T 128
#define WG_KR 64
#define WG_PITCH 72

__device__ __forceinline__ void wg_pair(int p, int NB, int* bi, int* bj) {
  int i = 0;
  while (p >= NB - i) {
    p -= NB - i;
    ++i;
  }
  *bi = i;
  *bj = i + p;
}

__global__ __launch_bounds__(256, 2) void glm_wide_gram_kernel(const float* __restrict__ X, int ldx, int P,
                                                               long long N, const float* __restrict__ Wr, int NB,
                                                               int npairs, int S, int fold,
                                                               double* __restrict__ part, int dbg) {
  extern __shared__ __bf16 wg_lds[];
  __bf16* sAh = wg_lds;
  __bf16* sAl = sAh + WG_T * WG_PITCH;
  __bf16* sBh = sAl + WG_T * WG_PITCH;
  __bf16* sBl = sBh + WG_T * WG_PITCH;
  float* sW = reinterpret_cast<float*>(sBl + WG_T * WG_PITCH);   // the chunk's 64 row weights
  const int nblk = npairs * S;
  const int L = xcd_remap(blockIdx.x, nblk);
  const int sl = L / npairs, pr = L - sl * npairs;
  int bi, bj;
  wg_pair(pr, NB, &bi, &bj);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int mi = wv >> 1, ni = wv & 1;
  const long long nchunk = (N + WG_KR - 1) / WG_KR;
  // loader slots: q = 0..7 -> panel q >> 2 (A = bi, B = bj), column
  // tid & 127, row group ((tid >> 7) + 2 q) & 7 -- wave-uniform, so the row
  // offsets are scalar and the weights scalar loads; X through a buffer
  // descriptor rebased per chunk (rows past N read as 0 by the range check)
  const int t7 = __builtin_amdgcn_readfirstlane(tid >> 7);
  const int colb = tid & 127;
  const int gcA = bi * WG_T + colb, gcB = bj * WG_T + colb;
  const float fillA = gcA == P ? 1.f : 0.f, fillB = gcB == P ? 1.f : 0.f;
  const bool inA = gcA < P, inB = gcB < P;
  float xr[8][8];
  float wpre = 0.f;
  // issue-only: the raw values land in xr / wpre while this chunk's MFMAs
  // run; the column fill and the row weights are applied in store()
  auto load = [&](long long c) {
    const long long row0 = c * WG_KR;
    const int nr = (int)((N - row0) < WG_KR ? (N - row0) : WG_KR);
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void*)(X + row0 * ldx), (short)0, (dbg & 1) ? 0 : nr * ldx * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)(Wr + row0), (short)0, nr * 4, 0x00020000);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int pan = q >> 2;
      const int rg = (t7 + 2 * q) & 7;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        xr[q][e] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, (pan ? gcB : gcA) * 4, (rg * 8 + e) * ldx * 4, 0));
    }
    if (tid < WG_KR) wpre = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, tid * 4, 0, 0));  // 0 past N
  };
  auto store = [&]() {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int pan = q >> 2, col = colb, rg = (t7 + 2 * q) & 7;
      bf16x8 h, l;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = (pan ? inB : inA) ? xr[q][e] : (pan ? fillB : fillA);
        if (!pan) x *= sW[rg * 8 + e];
        h[e] = (__bf16)x;
        l[e] = (__bf16)(x - (float)h[e]);
      }
      const int off = col * WG_PITCH + rg * 8;
      *reinterpret_cast<bf16x8*>((pan ? sBh : sAh) + off) = h;
      *reinterpret_cast<bf16x8*>((pan ? sBl : sAl) + off) = l;
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  double* my = part + (size_t)L * (WG_T * WG_T);
  auto fold_out = [&]() {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 64 * mi + 16 * a + 4 * (lane >> 4) + r, j = 64 * ni + 16 * b + (lane & 15);
          my[i * WG_T + j] += (double)acc[a][b][r];
        }
        acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
  };
  long long c = sl;
  if (c < nchunk) load(c);
  int since = 0;
  long long cfold = c + (long long)fold * S;   // fold once the chunk index passes this
  while (c < nchunk) {
    __syncthreads();  // the previous chunk's operand / weight reads are done
    if (tid < WG_KR) sW[tid] = wpre;
    __syncthreads();
    store();
    __syncthreads();
    const long long cn = c + S;
    if (cn < nchunk) load(cn);  // in flight during this chunk's MFMAs
#pragma unroll
    for (int ks = 0; ks < WG_KR / 32; ++ks) {
      const int ko = ks * 32 + 8 * (lane >> 4);
      bf16x8 ah[4], al[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int off = (64 * mi + 16 * a + (lane & 15)) * WG_PITCH + ko;
        ah[a] = *reinterpret_cast<const bf16x8*>(sAh + off);
        al[a] = *reinterpret_cast<const bf16x8*>(sAl + off);
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        // one B column tile at a time (8 registers); the 12 MFMAs on four
        // accumulators keep dependent issues 4 apart
        const int off = (64 * ni + 16 * b + (lane & 15)) * WG_PITCH + ko;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(sBh + off);
        const bf16x8 bl = *reinterpret_cast<const bf16x8*>(sBl + off);
#pragma unroll
        for (int a = 0; a < 4; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[a], bh, acc[a][b], 0, 0, 0);
#pragma unroll
        for (int a = 0; a < 4; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[a], bl, acc[a][b], 0, 0, 0);
#pragma unroll
        for (int a = 0; a < 4; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[a], bh, acc[a][b], 0, 0, 0);
      }
    }
    ++since;
    c = cn;
    if (c >= cfold) {
      fold_out();
      since = 0;
      cfold = c + (long long)fold * S;
    }
  }
  if (since) fold_out();
}

// part: [npairs * S][128][128] f64, zeroed by the caller; slot L holds
// pair L % npairs (bi <= bj, row-major over the upper triangle of the NB x NB
// tile grid) for slice L / npairs.  NB = ceil((P + 1) / 128).
// dbg bit 0 (timing only): the X descriptor gets zero records, so every X
// load is dropped by the range check while the instruction stream stays.
extern "C" int h2o_glm_wide_gram(const float* X, int ldx, int P, long long N, const float* Wr, int S, int fold,
                                 double* part, int dbg, hipStream_t s) {
  if (N <= 0) return 0;
  if (ldx < P || S <= 0 || fold <= 0) return -1;
  const int NB = (P + 1 + WG_T - 1) / WG_T;
  const int npairs = NB * (NB + 1) / 2;
  const size_t lds = 4 * WG_T * WG_PITCH * sizeof(__bf16) + WG_KR * sizeof(float);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)glm_wide_gram_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(glm_wide_gram_kernel, dim3(npairs * S), dim3(256), lds, s, X, ldx, P, N, Wr, NB, npairs, S, fold,
                     part, dbg);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// 256 x 256 tile version (default): one workgroup of 8 waves per CU, each
// wave a 128 x 64 piece on v_mfma_f32_32x32x16_bf16 (8 accumulators of 16
// registers).  LDS holds two chunk buffers: while the MFMAs read chunk t,
// the same waves convert and store chunk t + 1 (its f32 values arrived in
// registers during the previous chunk) into the other buffer -- one barrier
// per chunk, and the VALU conversion interleaves with the MFMA stream
// instead of running in a phase of its own (PMC of the single-buffer
// version: MFMA busy 36%, 35% of wave cycles parked at barriers / waits).
// Columns are stored k-contiguous, pitch 32 bf16, with the 8-row k-blocks
// XOR-swizzled by (column >> 2) & 3: conflict-free b128 stores and operand
// reads.  Diagonal tiles skip their lower-left quarter (the transpose of the
// upper-right one).
// ---------------------------------------------------------------------------
#define WG2_T 256
// KR rows per chunk: 32 for bf16x3 (4 planes per buffer), 32 or 64 for the
// one-MFMA bf16 tier (2 planes; 64 halves the barriers and weight loads per
// row).  k-blocks of 8 are XOR-swizzled so that the 8 lanes of a b128 access
// (8 consecutive columns, one k-block) land in 8 different 16-B bank groups
// of the 256-B bank row: pitch 64 B -> swizzle by column >> 2, pitch 128 B
// -> by column >> 1.
template <int KR, int SWZ = 0>
__device__ __forceinline__ int wg2_off(int col, int kb) {
  // SWZ (KR = 64 A/B only): 0 (col >> 1) & 7, 1 ((col >> 1) ^ (col >> 4)) & 7, 2 (col >> 2) & 7
  const int x = KR == 32 ? (col >> 2) & 3
                         : (SWZ == 1 ? ((col >> 1) ^ (col >> 4)) & 7 : SWZ == 2 ? (col >> 2) & 7 : (col >> 1) & 7);
  return col * KR + ((kb ^ x) << 3);
}

template <bool BF3, int KR, int SWZ = 0>
__global__ __launch_bounds__(512, 1) void glm_wide_gram256_kernel(const float* __restrict__ X, int ldx, int P,
                                                                  long long N, const float* __restrict__ Wr, int NB,
                                                                  int npairs, int S, int fold,
                                                                  double* __restrict__ part, int dbg) {
  constexpr int NPL = BF3 ? 4 : 2;                 // planes: A hi, (A lo), B hi, (B lo)
  constexpr int BUF = NPL * WG2_T * KR;            // bf16 per chunk buffer
  constexpr int PBH = BF3 ? 2 : 1;                 // plane index of B hi
  constexpr int NRG = KR / 8;                      // 8-row groups per chunk
  constexpr int NQ = NRG;                          // (panel, row group) slices per thread: 2 panels x NRG / 2
  extern __shared__ __bf16 wg2_lds[];
  const int nblk = npairs * S;
  const int L = xcd_remap(blockIdx.x, nblk);
  const int sl = L / npairs, pr = L - sl * npairs;
  int bi, bj;
  wg_pair(pr, NB, &bi, &bj);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int mi = wv >> 2, nq = wv & 3;      // rows 128 mi .., columns 64 nq ..
  const bool skip = bi == bj && mi == 1 && nq < 2;  // lower-left quarter of a diagonal tile
  const long long nchunk = (N + KR - 1) / KR;
  // chunks of this slice: c = sl + t S, t = 0 .. nt - 1
  const long long nt = sl < nchunk ? (nchunk - 1 - sl) / S + 1 : 0;
  // loader: thread = column tid & 255 of panel q / (NQ / 2), row group
  // (tid >> 8) + 2 (q % (NQ / 2)) -- wave-uniform
  const int t8 = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int colb = tid & 255;
  const int gcA = bi * WG2_T + colb, gcB = bj * WG2_T + colb;
  const float fillA = gcA == P ? 1.f : 0.f, fillB = gcB == P ? 1.f : 0.f;
  const bool inA = gcA < P, inB = gcB < P;
  float xr[NQ][8];
  // row weights of the panel-A row groups of the chunk being converted next:
  // wave-uniform, so they come in by scalar loads (no LDS staging, no LDS
  // wait inside the MFMA stream).  Wr holds N rounded up to KR, zero past N.
  typedef float f32x8 __attribute__((ext_vector_type(8)));
  f32x8 wq[NQ / 2];
  const long long npad = (N + KR - 1) / KR * KR;
  auto load_wq = [&](long long t) __attribute__((always_inline)) {
    long long row0 = (sl + t * S) * KR;
    row0 = row0 < npad ? row0 : 0;                 // prefetch past the last chunk: any in-bounds rows
#pragma unroll
    for (int q = 0; q < NQ / 2; ++q)
      wq[q] = *reinterpret_cast<const f32x8*>(Wr + row0 + (t8 + 2 * q) * 8);
  };
  auto load_x = [&](long long t) __attribute__((always_inline)) {
    const long long row0 = (sl + t * S) * KR;
    const long long left = N - row0;
    const int nr = (int)(left < KR ? (left > 0 ? left : 0) : KR);   // past N: every load reads 0
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void*)(X + row0 * ldx), (short)0, (dbg & 1) ? 0 : nr * ldx * 4, 0x00020000);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int pan = q / (NQ / 2), rg = t8 + 2 * (q % (NQ / 2));
#pragma unroll
      for (int e = 0; e < 8; ++e)
        xr[q][e] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, (pan ? gcB : gcA) * 4, (rg * 8 + e) * ldx * 4, 0));
    }
  };
  // FULL (wave-uniform): every column of this wave's loader slice is < P in
  // both panels, so the conversion needs no per-element fill select
  auto store_q = [&](int buf, int q, auto fullc) __attribute__((always_inline)) {
    __bf16* base = wg2_lds + buf * BUF;
    const int pan = q / (NQ / 2), rg = t8 + 2 * (q % (NQ / 2));
    bf16x8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x;
      if constexpr (decltype(fullc)::value) x = xr[q][e];
      else x = (pan ? inB : inA) ? xr[q][e] : (pan ? fillB : fillA);
      if (!pan) x *= wq[q][e];
      h[e] = (__bf16)x;
      if constexpr (BF3) l[e] = (__bf16)(x - (float)h[e]);
    }
    const int off = wg2_off<KR, SWZ>(colb, rg);
    *reinterpret_cast<bf16x8*>(base + (pan ? PBH : 0) * WG2_T * KR + off) = h;
    if constexpr (BF3) *reinterpret_cast<bf16x8*>(base + (pan ? 3 : 1) * WG2_T * KR + off) = l;
  };
  auto store = [&](int buf, auto fullc) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) store_q(buf, q, fullc);
  };
  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  double* my = part + (size_t)L * (WG2_T * WG2_T);
  auto fold_out = [&]() __attribute__((always_inline)) {
    // opaque copies: the 128 fold addresses are not loop-invariant for the
    // compiler, so they are not hoisted out of the chunk loop into registers
    const unsigned long long mu = (unsigned long long)my;
    double* mb = (double*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(mu >> 32)) << 32) |
                           (unsigned)__builtin_amdgcn_readfirstlane((unsigned)mu));
    int ln = lane;
    asm volatile("" : "+s"(mb), "+v"(ln));
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          // 32x32 C layout: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
          const int i = 128 * mi + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
          const int j = 64 * nq + 32 * b + (ln & 31);
          gbl_add(mb + i * WG2_T + j, (double)acc[a][b][r]);   // no-return atomic: nothing to hold in registers
          acc[a][b][r] = 0.f;
        }
      }
  };
  // one chunk's MFMAs on buffer `buf`, with the conversion + store of the
  // next chunk's q-th slice into buffer `nbuf` after each (ks, b) sub-step:
  // straight-line code, so the scheduler interleaves VALU with the MFMAs
  auto compute_store = [&](int buf, int nbuf, auto fullc) __attribute__((always_inline)) {
    const __bf16* sAh = wg2_lds + buf * BUF;
    const __bf16* sAl = sAh + WG2_T * KR;
    const __bf16* sBh = sAh + PBH * WG2_T * KR;
    const __bf16* sBl = sAh + 3 * WG2_T * KR;
#pragma unroll
    for (int ks = 0; ks < KR / 16; ++ks) {
      const int kb = 2 * ks + (lane >> 5);
      bf16x8 ah[4], al[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int off = wg2_off<KR, SWZ>(128 * mi + 32 * a + (lane & 31), kb);
        ah[a] = *reinterpret_cast<const bf16x8*>(sAh + off);
        if constexpr (BF3) al[a] = *reinterpret_cast<const bf16x8*>(sAl + off);
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int off = wg2_off<KR, SWZ>(64 * nq + 32 * b + (lane & 31), kb);
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(sBh + off);
#pragma unroll
        for (int a = 0; a < 4; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh, acc[a][b], 0, 0, 0);
        if constexpr (BF3) {
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(sBl + off);
#pragma unroll
          for (int a = 0; a < 4; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl, acc[a][b], 0, 0, 0);
#pragma unroll
          for (int a = 0; a < 4; ++a) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh, acc[a][b], 0, 0, 0);
        }
        store_q(nbuf, 2 * ks + b, fullc);
      }
    }
  };
  if (nt == 0) return;
  const int wbase = (tid & 255) & ~63;              // this wave's first loader column
  const bool full = bi * WG2_T + wbase + 63 < P && bj * WG2_T + wbase + 63 < P;
  auto run = [&](auto fullc) __attribute__((always_inline)) {
    // prologue: chunk 0 in buffer 0, chunk 1's values and weights in flight
    load_wq(0);
    load_x(0);
    store(0, fullc);
    __syncthreads();
    if (nt > 1) load_x(1);
    load_wq(1);
    // chunk groups of `fold` with the fold between them; every chunk runs
    // the same straight-line body (a diagonal tile's skipped quarter computes
    // and is never folded; the store past the last chunk writes the unused
    // buffer), so MFMA and conversion interleave within one basic block
    for (long long t0 = 0; t0 < nt; t0 += fold) {
      const long long t1 = t0 + fold < nt ? t0 + fold : nt;
      for (long long t = t0; t < t1; ++t) {
        const int cur = (int)(t & 1);
        compute_store(cur, cur ^ 1, fullc);
        __syncthreads();
        load_x(t + 2);
        load_wq(t + 2);
      }
      if (!skip) fold_out();
    }
  };
  if (__builtin_amdgcn_readfirstlane(full ? 1 : 0)) run(std::true_type{});
  else run(std::false_type{});
}

// bf3 = 0: one bf16 MFMA per product (hi * hi, ~2^-9 relative): the
// Hessian of a well-conditioned system, whose Newton step on the exact
// gradient still converges to the exact-gradient fixed point
extern "C" int h2o_glm_wide_gram256(const float* X, int ldx, int P, long long N, const float* Wr, int S, int fold,
                                    double* part, int dbg, int bf3, hipStream_t s) {
  if (N <= 0) return 0;
  if (ldx < P || S <= 0 || fold <= 0) return -1;
  const int NB = (P + 1 + WG2_T - 1) / WG2_T;
  const int npairs = NB * (NB + 1) / 2;
  // bf16 tier chunk rows (H2O3_WIDE_KR = 32 / 64, default 64)
  static const int kr16 = getenv("H2O3_WIDE_KR") && atoi(getenv("H2O3_WIDE_KR")) == 32 ? 32 : 64;
  const int KR = bf3 ? 32 : kr16;
  const size_t lds = 2 * (size_t)(bf3 ? 4 : 2) * WG2_T * KR * sizeof(__bf16);
  static bool attr = false;
  if (!attr) {
    const size_t l3 = 2 * 4 * WG2_T * 32 * sizeof(__bf16);
    const size_t l32 = 2 * 2 * WG2_T * 32 * sizeof(__bf16);
    const size_t l64 = 2 * 2 * WG2_T * 64 * sizeof(__bf16);
    (void)hipFuncSetAttribute((const void*)glm_wide_gram256_kernel<true, 32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)l3);
    (void)hipFuncSetAttribute((const void*)glm_wide_gram256_kernel<false, 32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)l32);
    (void)hipFuncSetAttribute((const void*)glm_wide_gram256_kernel<false, 64>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)l64);
    attr = true;
  }
  if (bf3)
    hipLaunchKernelGGL((glm_wide_gram256_kernel<true, 32>), dim3(npairs * S), dim3(512), lds, s, X, ldx, P, N, Wr, NB,
                       npairs, S, fold, part, dbg);
  else if (KR == 32)
    hipLaunchKernelGGL((glm_wide_gram256_kernel<false, 32>), dim3(npairs * S), dim3(512), lds, s, X, ldx, P, N, Wr,
                       NB, npairs, S, fold, part, dbg);
  else {
    static const int swz = getenv("H2O3_WG2_SWZ") ? atoi(getenv("H2O3_WG2_SWZ")) : 0;   // A/B knob
    if (swz == 1) {
      (void)hipFuncSetAttribute((const void*)glm_wide_gram256_kernel<false, 64, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((glm_wide_gram256_kernel<false, 64, 1>), dim3(npairs * S), dim3(512), lds, s, X, ldx, P, N,
                         Wr, NB, npairs, S, fold, part, dbg);
    } else if (swz == 2) {
      (void)hipFuncSetAttribute((const void*)glm_wide_gram256_kernel<false, 64, 2>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((glm_wide_gram256_kernel<false, 64, 2>), dim3(npairs * S), dim3(512), lds, s, X, ldx, P, N,
                         Wr, NB, npairs, S, fold, part, dbg);
    } else {
      hipLaunchKernelGGL((glm_wide_gram256_kernel<false, 64>), dim3(npairs * S), dim3(512), lds, s, X, ldx, P, N, Wr,
                         NB, npairs, S, fold, part, dbg);
    }
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Exact f64 weighted Gram on the f64 matrix cores: G = Xa' diag(W) Xa with
// Xa = [X[:, :P] | 1] (the intercept column implicit), f32 storage widened
// exactly, f64 products and f64 accumulation -- the top GLM precision tier
// (ill-conditioned designs: RuleFit's 0/1 rule matrices, near-collinear
// columns), which ran as chunked f64 torch GEMMs over an f64 copy of X.
//
// Reference: hex/gram/Gram.java (GramTask: X'WX accumulated in double per
// chunk, reduced across nodes).
//
// Layout.  One workgroup = one 64 x 64 tile pair (I <= J) of the augmented
// Gram over one slab of rows; 4 waves, each a 32 x 32 quarter = 2 x 2
// v_mfma_f64_16x16x4_f64 blocks (A lane l: A[l&15][k=l>>4]; C/D: col=l&15,
// row=(l>>4)+4*reg).  Rows are staged 32 at a time through LDS as f64
// (A side pre-multiplied by W), the next 16 rows prefetched into registers
// while the MFMAs run (16-byte row loads when aligned).  Slab partials [S][npairs][64][64] are summed in a
// fixed order by the caller (deterministic).
#define GF_T 64
#define GF_KR 32

__device__ __forceinline__ double gf_load(const float* __restrict__ X, int ldx, int P, long long r, int c) {
  if (c < P) return (double)X[(size_t)r * ldx + c];
  return c == P ? 1.0 : 0.0;
}

// 4 consecutive columns c .. c+3 of row r of [X | 1 | 0...] as f64; VEC: one
// 16-byte load when all four are columns of X (rows 16-byte aligned).
typedef double gf_d4 __attribute__((ext_vector_type(4)));

template <bool VEC>
__device__ __forceinline__ gf_d4 gf_load4(const float* __restrict__ X, int ldx, int P, long long r, int c) {
  if (VEC && c + 3 < P) {
    const float4 q = *reinterpret_cast<const float4*>(X + (size_t)r * ldx + c);
    return gf_d4{(double)q.x, (double)q.y, (double)q.z, (double)q.w};
  }
  if (c + 3 < P) {
    const float* x = X + (size_t)r * ldx + c;
    return gf_d4{(double)x[0], (double)x[1], (double)x[2], (double)x[3]};
  }
  return gf_d4{gf_load(X, ldx, P, r, c), gf_load(X, ldx, P, r, c + 1), gf_load(X, ldx, P, r, c + 2),
               gf_load(X, ldx, P, r, c + 3)};
}

template <bool VEC>
__global__ __launch_bounds__(256) void gram_f64_kernel(const float* __restrict__ X, int ldx, int P, long long N,
                                                       const double* __restrict__ W, const int2* __restrict__ pairs,
                                                       int npairs, long long rows_per_slab,
                                                       double* __restrict__ part) {
  __shared__ double As[GF_KR][GF_T + 1];
  __shared__ double Bs[GF_KR][GF_T + 1];
  // blocks of one slab are consecutive: the tile pairs of a slab run
  // together and share its rows in L2
  const int p = blockIdx.x % npairs;
  const long long s = blockIdx.x / npairs;
  const int I0 = pairs[p].x * GF_T, J0 = pairs[p].y * GF_T;
  const bool diag = I0 == J0;
  const long long r0 = s * rows_per_slab;
  long long r1 = r0 + rows_per_slab;
  if (r1 > N) r1 = N;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wi = wv >> 1, wj = wv & 1;
  typedef double d4 __attribute__((ext_vector_type(4)));
  d4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  // staging map: quad e of thread t is row (t + 256 e) / 16, columns
  // 4 ((t + 256 e) % 16) .. +3 (16 threads cover one 64-column row)
  gf_d4 ra[2], rb[2];
  double wr[2];
  auto fetch = [&](long long base) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int q = t + 256 * e;
      const int rr = q >> 4, cc = (q & 15) * 4;
      const long long r = base + rr;
      const gf_d4 z = {0.0, 0.0, 0.0, 0.0};
      if (r < r1) {
        wr[e] = W[r];
        ra[e] = gf_load4<VEC>(X, ldx, P, r, I0 + cc);
        rb[e] = diag ? z : gf_load4<VEC>(X, ldx, P, r, J0 + cc);
      } else {
        wr[e] = 0.0;
        ra[e] = z;
        rb[e] = z;
      }
    }
  };
  if (r0 < r1) fetch(r0);
  for (long long base = r0; base < r1; base += GF_KR) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int q = t + 256 * e;
      const int rr = q >> 4, cc = (q & 15) * 4;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        As[rr][cc + u] = ra[e][u] * wr[e];
        Bs[rr][cc + u] = diag ? ra[e][u] : rb[e][u];
      }
    }
    __syncthreads();
    if (base + GF_KR < r1) fetch(base + GF_KR);   // overlaps the MFMAs below
#pragma unroll
    for (int ks = 0; ks < GF_KR / 4; ++ks) {
      const int k = 4 * ks + (lane >> 4);
      const double a0 = As[k][wi * 32 + (lane & 15)];
      const double a1 = As[k][wi * 32 + 16 + (lane & 15)];
      const double b0 = Bs[k][wj * 32 + (lane & 15)];
      const double b1 = Bs[k][wj * 32 + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
  double* out = part + ((size_t)s * npairs + p) * (GF_T * GF_T);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int row = wi * 32 + a * 16 + (lane >> 4) + 4 * reg;
        const int col = wj * 32 + b * 16 + (lane & 15);
        out[row * GF_T + col] = acc[a][b][reg];
      }
}

// X: f32 [N, ldx] (first P columns used), W: f64 [N]; pairs: int2 [npairs]
// tile pairs (I <= J) of the augmented Gram (P + 1 columns, 64-wide tiles);
// part: f64 [slabs, npairs, 64, 64].
extern "C" int h2o_gram_f64(const float* X, int ldx, int P, long long N, const double* W, const int* pairs,
                            int npairs, int slabs, long long rows_per_slab, double* part, hipStream_t s) {
  if (npairs <= 0 || slabs <= 0) return 0;
  if (P < 0 || ldx < P || rows_per_slab <= 0 || (long long)slabs * rows_per_slab < N) return -1;
  const long long blocks = (long long)slabs * npairs;
  if (blocks > 0x7fffffffLL) return -2;
  const bool vec = (ldx % 4 == 0) && ((uintptr_t)X % 16 == 0);
  if (vec)
    hipLaunchKernelGGL(gram_f64_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, X, ldx, P, N, W,
                       (const int2*)pairs, npairs, rows_per_slab, part);
  else
    hipLaunchKernelGGL(gram_f64_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, X, ldx, P, N, W,
                       (const int2*)pairs, npairs, rows_per_slab, part);
  return (int)hipGetLastError();
}

// The two f64 matrix-vector products of the same tier, straight from the f32
// rows: eta = X[:, :P] beta + b0 (one wave per row, coalesced along the row,
// f64 FMAs, wave sum) and the gradient partials X[:, :P]' r per row slab
// (thread per column, coalesced row reads, f64 register sums; slabs summed by
// the caller in a fixed order).
__global__ __launch_bounds__(256) void xv_f64_kernel(const float* __restrict__ X, int ldx, int P, long long N,
                                                     const double* __restrict__ beta, double b0,
                                                     double* __restrict__ eta) {
  const int lane = threadIdx.x & 63;
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= N) return;   // wave-uniform
  const float* xr = X + (size_t)r * ldx;
  double acc = 0.0;
  for (int c = lane; c < P; c += 64) acc += (double)xr[c] * beta[c];
  acc = wave_sum(acc);
  if (lane == 0) eta[r] = acc + b0;
}

__global__ __launch_bounds__(256) void xtr_f64_kernel(const float* __restrict__ X, int ldx, int P, long long N,
                                                      const double* __restrict__ rv, long long rows_per_slab,
                                                      double* __restrict__ part) {
  const long long r0 = (long long)blockIdx.y * rows_per_slab;
  long long r1 = r0 + rows_per_slab;
  if (r1 > N) r1 = N;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= P) return;
  double acc = 0.0;
  for (long long r = r0; r < r1; ++r) acc += (double)X[(size_t)r * ldx + c] * rv[r];
  part[(size_t)blockIdx.y * P + c] = acc;
}

extern "C" int h2o_xv_f64(const float* X, int ldx, int P, long long N, const double* beta, double b0, double* eta,
                          hipStream_t s) {
  if (N <= 0) return 0;
  if (P < 0 || ldx < P) return -1;
  const long long blocks = (N + 3) / 4;
  if (blocks > 0x7fffffffLL) return -2;
  hipLaunchKernelGGL(xv_f64_kernel, dim3((unsigned)blocks), dim3(256), 0, s, X, ldx, P, N, beta, b0, eta);
  return (int)hipGetLastError();
}

extern "C" int h2o_xtr_f64(const float* X, int ldx, int P, long long N, const double* r, int slabs,
                           long long rows_per_slab, double* part, hipStream_t s) {
  if (N <= 0 || P <= 0) return 0;
  if (ldx < P || slabs <= 0 || slabs > 65535 || (long long)slabs * rows_per_slab < N) return -1;
  hipLaunchKernelGGL(xtr_f64_kernel, dim3((unsigned)((P + 255) / 256), (unsigned)slabs), dim3(256), 0, s, X, ldx, P,
                     N, r, rows_per_slab, part);
  return (int)hipGetLastError();
}
