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

typedef float f32x16 __attribute__((ext_vector_type(16)));

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
// LDS (row stride S = P (+32) so the two half-waves of an MFMA operand read
// hit disjoint bank halves).  Per chunk: (1) the four waves compute
// eta = x.beta for 16 rows each (beta held in registers, 64-lane dot + DPP
// reduce); (2) wave 0 evaluates the family/link for its 64 rows (mu, IRLS
// weight W, working response z, deviance) and overwrites two padding
// columns of the staged chunk with 1 and z — so the SAME MFMA sweep also
// produces X'W1, X'Wz, sum W and sum Wz (the augmented Gram [X 1 z]'W[X 1 z]);
// (3) every wave runs v_mfma_f32_32x32x2f32 for up to PPW upper-triangle
// 32x32 tile pairs straight out of LDS, folding f32 -> f32 -> f64 every 256 / 16K
// rows.  Each block owns an f64 partial tile (no atomics -> deterministic;
// the caller zero-fills `out`).
// Mode EXTERNAL (W, z supplied by the caller) serves families / links the
// fused path does not cover and the plain weighted Gram (z == nullptr).
// ---------------------------------------------------------------------------
#define GI_RC 64
#define GI_PPW 3

struct GlmFamArgs {
  int link;     // 0 identity 1 logit 2 log 3 inverse
  int var;      // 0 gaussian 1 binomial 2 poisson 3 gamma 4 tweedie 5 negbin
  float tvp;    // tweedie variance power
  float theta;  // negative-binomial dispersion
};

__device__ __forceinline__ float gi_linkinv(int link, float eta) {
  switch (link) {
    case 1: return 1.f / (1.f + __expf(-eta));
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

template <bool FUSED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void glm_irls_kernel(
    const float* __restrict__ X, long long N, int P, int S, const int2* __restrict__ pairs, int n_pairs,
    int rows_per_block, const float* __restrict__ beta, float b0, const float* __restrict__ y,
    const float* __restrict__ wprior, const float* __restrict__ offset, GlmFamArgs fam,
    const float* __restrict__ Wext, const float* __restrict__ zext, int aug, double* __restrict__ out,
    double* __restrict__ dev_out) {
  extern __shared__ float L[];          // [GI_RC][S]
  __shared__ float wr[GI_RC];
  __shared__ float eta_s[GI_RC];
  const int split = blockIdx.x;
  const int grp = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int kr = lane >> 5, cc = lane & 31;
  const long long rb0 = (long long)split * rows_per_block;
  const long long rb1 = min(N, rb0 + rows_per_block);

  int ci[GI_PPW], cj[GI_PPW];
  bool pv[GI_PPW];
#pragma unroll
  for (int q = 0; q < GI_PPW; ++q) {
    const int p = grp * (4 * GI_PPW) + wv + 4 * q;
    pv[q] = p < n_pairs;
    const int2 t = pv[q] ? pairs[p] : make_int2(0, 0);
    ci[q] = t.x * 32;
    cj[q] = t.y * 32;
  }
  float bet[8];
  if (FUSED) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = lane + 64 * k;
      bet[k] = c < P ? beta[c] : 0.f;
    }
  }
  // three-level accumulation: MFMA f32 (256 rows) -> f32 mid (<=16K rows)
  // -> this block's own f64 output tile (plain read-modify-write, no atomics)
  f32x16 mid[GI_PPW];
  f32x16 acc[GI_PPW];
#pragma unroll
  for (int q = 0; q < GI_PPW; ++q) {
#pragma unroll
    for (int i = 0; i < 16; ++i) { mid[q][i] = 0.f; acc[q][i] = 0.f; }
  }
  double dev = 0.0;
  const int P4 = P >> 2;
  const int nvec = GI_RC * P4;
  int since = 0;
  for (long long r0 = rb0; r0 < rb1; r0 += GI_RC) {
    // (0) stage the chunk (clamped rows past N are zero-weighted below)
    for (int e = threadIdx.x; e < nvec; e += 256) {
      const int rr = e / P4, c4 = e - rr * P4;
      const long long g = min(r0 + rr, N - 1);
      const float4 v = *reinterpret_cast<const float4*>(X + g * (long long)P + 4 * c4);
      *reinterpret_cast<float4*>(L + rr * S + 4 * c4) = v;
    }
    __syncthreads();
    if (FUSED) {
      // (1) eta for 16 rows per wave
      for (int j = 0; j < GI_RC / 4; ++j) {
        const int rr = wv * (GI_RC / 4) + j;
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int c = lane + 64 * k;
          if (c < P) s += L[rr * S + c] * bet[k];
        }
        s = wave_sum(s);
        if (lane == 0) eta_s[rr] = s;
      }
      __syncthreads();
    }
    // (2) family / link on wave 0: IRLS weight + working response
    if (wv == 0) {
      const long long r = r0 + lane;
      float W = 0.f, z = 0.f;
      if (r < rb1) {
        if (FUSED) {
          const float off = offset ? offset[r] : 0.f;
          const float eta = eta_s[lane] + b0 + off;
          const float mu = gi_linkinv(fam.link, eta);
          const float yr = y[r];
          const float pw = wprior ? wprior[r] : 1.f;
          if (fam.link == 0 && fam.var == 0) {
            W = pw;
            z = yr - off;
          } else {
            const float d = gi_dmu(fam.link, mu);
            W = pw * d * d / gi_var(fam, mu);
            z = (eta - off) + (yr - mu) / d;
          }
          if (pw != 0.f) dev += (double)(pw * gi_dev(fam, yr, mu));
        } else {
          W = Wext ? Wext[r] : 1.f;
          z = zext ? zext[r] : 0.f;
        }
      }
      wr[lane] = W;
      if (aug >= 0) {
        L[lane * S + aug] = 1.f;
        L[lane * S + aug + 1] = z;
      }
    }
    __syncthreads();
    // (3) MFMA sweep over the chunk for this wave's tile pairs
#pragma unroll 4
    for (int k = 0; k < GI_RC / 2; ++k) {
      const int rr = 2 * k + kr;
      const float w = wr[rr];
      const float* row = L + rr * S;
#pragma unroll
      for (int q = 0; q < GI_PPW; ++q) {
        if (pv[q]) {
          const float a = row[ci[q] + cc];
          const float b = w * row[cj[q] + cc];
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[q], 0, 0, 0);
        }
      }
    }
    ++since;
    const bool last = r0 + GI_RC >= rb1;
    if ((since & 3) == 0 || last) {
#pragma unroll
      for (int q = 0; q < GI_PPW; ++q) {
#pragma unroll
        for (int i = 0; i < 16; ++i) { mid[q][i] += acc[q][i]; acc[q][i] = 0.f; }
      }
    }
    if (since == 256 || last) {
#pragma unroll
      for (int q = 0; q < GI_PPW; ++q) {
        if (!pv[q]) continue;
        const int p = grp * (4 * GI_PPW) + wv + 4 * q;
        double* o = out + ((size_t)split * n_pairs + p) * 1024;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = (i & 3) + 8 * (i >> 2) + 4 * kr;
          o[row * 32 + cc] += (double)mid[q][i];
          mid[q][i] = 0.f;
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

extern "C" int h2o_glm_irls(const float* X, long long N, int P, const int* pairs, int n_pairs, int n_splits,
                            int rows_per_block, const float* beta, float b0, const float* y, const float* wprior,
                            const float* offset, int link, int var, float tvp, float theta, const float* Wext,
                            const float* zext, int aug, double* out, double* dev_out, hipStream_t s) {
  if (N <= 0 || n_pairs <= 0) return 0;
  if (P % 32 != 0 || P > 512) return -1;
  if (aug >= 0 && aug + 1 >= P) return -2;
  const int S = (P % 64 == 0) ? P + 32 : P;
  const size_t lds = (size_t)GI_RC * S * sizeof(float);
  const int groups = (n_pairs + 4 * GI_PPW - 1) / (4 * GI_PPW);
  dim3 grid(n_splits, groups);
  GlmFamArgs fam{link, var, tvp, theta};
  if (beta) {
    hipLaunchKernelGGL(glm_irls_kernel<true>, grid, dim3(256), lds, s, X, N, P, S, (const int2*)pairs, n_pairs,
                       rows_per_block, beta, b0, y, wprior, offset, fam, Wext, zext, aug, out, dev_out);
  } else {
    hipLaunchKernelGGL(glm_irls_kernel<false>, grid, dim3(256), lds, s, X, N, P, S, (const int2*)pairs, n_pairs,
                       rows_per_block, beta, b0, y, wprior, offset, fam, Wext, zext, aug, out, dev_out);
  }
  return (int)hipGetLastError();
}
