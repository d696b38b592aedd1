// Deep Learning (MLP) kernels.  The training step of a dense MLP runs as
// three hand-written kernels (dl_mlp_*, f32 MFMA v_mfma_f32_16x16x4_f32 --
// exact f32 products, the reference's float arithmetic); the element-wise
// kernels below remain for the configurations the fused step does not take
// (maxout, autoencoders, non-Gaussian regression losses, sparsity /
// elastic-averaging terms) and for scoring, whose dense products use the
// library GEMM.
//
// Reference: hex/deeplearning/Neurons.java — fprop (gemv + bias + activation
// + Dropout.fillBytes unit masks, test-time activation scaling by
// (1 - hidden_dropout_ratio)), bprop (per neuron row: gradient with L1/L2,
// ADADELTA or momentum / Nesterov update, max_w2 row rescale, bias update
// with the row's mean squared weight gradient), Softmax / Linear output
// layers (setOutputLayerGradient).
//
// MI355X design: one mini-batch is [B, units] row-major in HBM.
//   * dl_fwd_kernel: A = act(Z + b) with the dropout decision recomputed
//     from a counter hash of (seed, row, unit) — no mask tensor, the
//     backward kernel recomputes the same bits;
//   * dl_bwd_kernel: dZ = dA * act'(A) * mask, and the bias gradient column
//     sums of the workgroup's row block folded into one global atomic per
//     (block, unit);
//   * dl_update_kernel: one workgroup per neuron row does the reference's
//     whole per-row bprop tail in one pass over the row — gradient + L1/L2,
//     ADADELTA accumulators (or momentum / Nesterov), the row's mean squared
//     gradient for the bias update, then the max_w2 rescale (second pass
//     over the row, still in cache);
//   * dl_softmax_kernel: output probabilities and dE/dnet = (p - t) w / n
//     (CrossEntropy) or the Quadratic softmax gradient, one wave per row.
#include "common.h"
#include <algorithm>
#include <cstdlib>
#include <cstring>

enum { ACT_LINEAR = 0, ACT_TANH = 1, ACT_RELU = 2, ACT_ELU = 3, ACT_MAXOUT = 4 };

__device__ __forceinline__ unsigned dl_hash(unsigned long long seed, unsigned row, unsigned unit) {
  // counter-based hash (splitmix64 finalizer) of (seed, row, unit)
  unsigned long long x = seed ^ (((unsigned long long)row << 32) | unit);
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (unsigned)(x >> 32);
}

// unit kept when hash >= ratio * 2^32 (Dropout: a unit is dropped with
// probability `ratio`)
__device__ __forceinline__ bool dl_keep(unsigned long long seed, unsigned row, unsigned unit, unsigned thr) {
  return thr == 0u || dl_hash(seed, row, unit) >= thr;
}

__device__ __forceinline__ float dl_act(int act, float z) {
  switch (act) {
    case ACT_TANH: return tanhf(z);
    case ACT_RELU: return fmaxf(z, 0.f);
    case ACT_ELU: return z > 0.f ? z : expm1f(z);
    default: return z;
  }
}

// derivative expressed through the activation value a = act(z)
__device__ __forceinline__ float dl_dact(int act, float a) {
  switch (act) {
    case ACT_TANH: return 1.f - a * a;
    case ACT_RELU: return a > 0.f ? 1.f : 0.f;
    case ACT_ELU: return a > 0.f ? 1.f : a + 1.f;
    default: return 1.f;
  }
}

// Z: [B, U*k] pre-activations (k = 2 for maxout, else 1), bias [U*k] added in
// place; A: [B, U].  mode: 0 = train (dropout masks), 1 = test (scale by
// test_scale = 1 - ratio for the reference's dropout activations).
__global__ __launch_bounds__(256) void dl_fwd_kernel(float* __restrict__ Z, const float* __restrict__ bias,
                                                     float* __restrict__ A, int B, int U, int act, unsigned thr,
                                                     unsigned long long seed, const unsigned long long* seed_dev,
                                                     int mode, float test_scale) {
  if (seed_dev) seed += *seed_dev;   // graph replays: the step seed lives in device memory
  const long long n = (long long)B * U;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int row = (int)(e / U), u = (int)(e - (long long)row * U);
    float a;
    if (act == ACT_MAXOUT) {
      float* z = Z + (long long)row * 2 * U + 2 * u;
      const float z0 = z[0] + (bias ? bias[2 * u] : 0.f), z1 = z[1] + (bias ? bias[2 * u + 1] : 0.f);
      z[0] = z0;
      z[1] = z1;
      a = fmaxf(z0, z1);
    } else {
      const float z = Z[e] + (bias ? bias[u] : 0.f);
      Z[e] = z;
      a = dl_act(act, z);
    }
    if (mode == 0) {
      if (!dl_keep(seed, row, u, thr)) a = 0.f;
    } else {
      a *= test_scale;
    }
    A[e] = a;
  }
}

// dZ = dA * act'(A) * mask; dbias[u(*k)] += sum over the block's rows.
// Grid: (ceil(U / 256), row blocks); each thread owns one unit column.
__global__ __launch_bounds__(256) void dl_bwd_kernel(const float* __restrict__ dA, const float* __restrict__ A,
                                                     const float* __restrict__ Z, float* __restrict__ dZ,
                                                     float* __restrict__ dbias, int B, int U, int act, unsigned thr,
                                                     unsigned long long seed, const unsigned long long* seed_dev,
                                                     int rows_per_block) {
  if (seed_dev) seed += *seed_dev;
  const int u = blockIdx.x * 256 + threadIdx.x;
  if (u >= U) return;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(B, r0 + rows_per_block);
  float s0 = 0.f, s1 = 0.f;
  for (int row = r0; row < r1; ++row) {
    const long long e = (long long)row * U + u;
    float g = dA[e];
    if (!dl_keep(seed, row, u, thr)) g = 0.f;
    if (act == ACT_MAXOUT) {
      const float z0 = Z[2 * e], z1 = Z[2 * e + 1];
      const float g0 = z0 >= z1 ? g : 0.f, g1 = z0 >= z1 ? 0.f : g;
      dZ[2 * e] = g0;
      dZ[2 * e + 1] = g1;
      s0 += g0;
      s1 += g1;
    } else {
      g *= dl_dact(act, A[e]);
      dZ[e] = g;
      s0 += g;
    }
  }
  if (act == ACT_MAXOUT) {
    gbl_add(dbias + 2 * u, s0);
    gbl_add(dbias + 2 * u + 1, s1);
  } else {
    gbl_add(dbias + u, s0);
  }
}

struct DLUpdate {
  float rho, eps;          // ADADELTA
  float rate, momentum;    // plain SGD: rate already * (1 - momentum) like the reference
  float l1, l2, max_w2;
  int ada, nesterov, has_momenta;
  float sparsity_beta, average_activation;  // autoencoder sparsity term on the bias
};

// Per-weight part of the reference's bprop: gradient + L1/L2, then ADADELTA
// or momentum / Nesterov.  Returns the new weight; *g2 gets grad^2 (ADADELTA).
__device__ __forceinline__ float dl_upd_weight(float wv, float gw, float* a2, float* m, const DLUpdate& p,
                                               float* g2) {
  const float grad = gw + (wv > 0.f ? p.l1 : (wv < 0.f ? -p.l1 : 0.f)) + wv * p.l2;
  float nw;
  *g2 = 0.f;
  if (p.ada) {
    const float gg = grad * grad;
    *g2 = gg;
    const float eg2 = p.rho * a2[1] + (1.f - p.rho) * gg;
    const float rate = sqrtf((a2[0] + p.eps) / (eg2 + p.eps));
    a2[1] = eg2;
    a2[0] = p.rho * a2[0] + (1.f - p.rho) * rate * rate * gg;
    nw = wv - rate * grad;
  } else if (!p.nesterov) {
    const float delta = -p.rate * grad;
    nw = wv + delta;
    if (p.has_momenta) {
      nw += p.momentum * m[0];
      m[0] = delta;
    }
  } else {
    float tmp = -grad;
    if (p.has_momenta) {
      m[0] = m[0] * p.momentum + tmp;
      tmp = m[0];
    }
    nw = wv + p.rate * tmp;
  }
  return nw;
}

// The bias update of a neuron row given the row's mean squared gradient.
__device__ __forceinline__ void dl_upd_bias(float* bias, const float* dbias, float* ada_b, float* mom_b,
                                            const float* avg_act, int row, float avg_g2, const DLUpdate& p) {
  const float bv = bias[row];
  const float pg = dbias[row] + (bv > 0.f ? p.l1 : (bv < 0.f ? -p.l1 : 0.f)) + bv * p.l2;
  float rate = p.rate;
  if (p.ada) {
    float* ab = ada_b + 2 * row;
    ab[1] = p.rho * ab[1] + (1.f - p.rho) * avg_g2;
    rate = sqrtf((ab[0] + p.eps) / (ab[1] + p.eps));
    ab[0] = p.rho * ab[0] + (1.f - p.rho) * rate * rate * avg_g2;
  }
  float nb;
  if (!p.nesterov || p.ada) {
    const float delta = -rate * pg;
    nb = bv + delta;
    if (p.has_momenta && !p.ada) {
      nb += p.momentum * mom_b[row];
      mom_b[row] = delta;
    }
  } else {
    float d = -pg;
    if (p.has_momenta) {
      mom_b[row] = mom_b[row] * p.momentum + d;
      d = mom_b[row];
    }
    nb = bv + rate * d;
  }
  if (avg_act && p.sparsity_beta > 0.f) nb -= rate * p.sparsity_beta * (avg_act[row] - p.average_activation);
  bias[row] = nb;
}

// One workgroup per neuron row: W [U, I], dW [U, I] (mean gradient over the
// mini-batch), ada [U, I, 2] = (E[dx^2], E[g^2]), mom [U, I], bias / dbias /
// ada_b [U, 2] / mom_b [U]; avg_act [U] (sparsity, may be null).
__global__ __launch_bounds__(256) void dl_update_kernel(float* __restrict__ W, const float* __restrict__ dW,
                                                        float* __restrict__ ada, float* __restrict__ mom,
                                                        float* __restrict__ bias, const float* __restrict__ dbias,
                                                        float* __restrict__ ada_b, float* __restrict__ mom_b,
                                                        const float* __restrict__ avg_act, int U, int I,
                                                        DLUpdate p) {
  const int row = blockIdx.x;
  if (row >= U) return;
  float* w = W + (long long)row * I;
  const float* gw = dW + (long long)row * I;
  float g2sum = 0.f;
  for (int c = threadIdx.x; c < I; c += 256) {
    float g2;
    w[c] = dl_upd_weight(w[c], gw[c], ada + 2 * ((long long)row * I + c), mom ? mom + (long long)row * I + c : nullptr,
                         p, &g2);
    g2sum += g2;
  }
  __shared__ float red[256];
  float r2 = 0.f;
  if (p.max_w2 < 3.0e38f) {
    __syncthreads();   // every lane's weight written before the rescale pass
    for (int c = threadIdx.x; c < I; c += 256) r2 += w[c] * w[c];
  }
  // block sums of g2sum and r2
  red[threadIdx.x] = g2sum;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float avg_g2 = red[0] / (float)max(I, 1);
  __syncthreads();
  red[threadIdx.x] = r2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float rsum = red[0];
  if (p.max_w2 < 3.0e38f && rsum > p.max_w2) {
    const float scale = sqrtf(p.max_w2 / rsum);
    for (int c = threadIdx.x; c < I; c += 256) w[c] *= scale;
  }
  if (threadIdx.x == 0) dl_upd_bias(bias, dbias, ada_b, mom_b, avg_act, row, avg_g2, p);
}

// Softmax output: Z [B, K] (+ bias in place) -> P [B, K]; with labels y
// (int64, < 0 = skip) and weights w: dZ = g(p, t) * w / n, loss_out[row] =
// -w log p_y.  loss: 0 CrossEntropy (p - t), 1 Quadratic ((p - t)(1 - p)p).
__global__ __launch_bounds__(256) void dl_softmax_kernel(float* __restrict__ Z, const float* __restrict__ bias,
                                                         float* __restrict__ P, const long long* __restrict__ y,
                                                         const float* __restrict__ w, float* __restrict__ dZ,
                                                         float* __restrict__ loss_out, int B, int K, float inv_n,
                                                         int loss) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  float* z = Z + (long long)row * K;
  float mx = -INFINITY;
  for (int j = lane; j < K; j += 64) {
    const float v = z[j] + bias[j];
    z[j] = v;
    mx = fmaxf(mx, v);
  }
  mx = wave_max(mx);
  float s = 0.f;
  for (int j = lane; j < K; j += 64) s += __expf(z[j] - mx);
  s = wave_sum(s);
  const float inv = 1.f / s;
  const long long t = y ? y[row] : -1;
  const float wr = (t < 0) ? 0.f : (w ? w[row] : 1.f);
  for (int j = lane; j < K; j += 64) {
    const float p = __expf(z[j] - mx) * inv;
    P[(long long)row * K + j] = p;
    if (dZ) {
      const float tt = (j == t) ? 1.f : 0.f;
      const float g = loss == 0 ? (p - tt) : (p - tt) * (1.f - p) * p;
      dZ[(long long)row * K + j] = g * wr * inv_n;
    }
    if (loss_out && j == t) loss_out[row] = -wr * __logf(fmaxf(p, 1e-30f));
  }
}

// ---------------------------------------------------------------------------
// Fused MLP training step (dense layers, tanh / rectifier / exprectifier /
// linear units with hashed dropout, softmax or Gaussian linear output).
//
//   dl_mlp_fb_kernel   one workgroup per 16 batch rows: gathers the rows
//                      (idx), input dropout, every layer's forward on f32
//                      MFMA with bias + activation + dropout fused into the
//                      epilogue, the output gradient, then the backward
//                      dA = dZ W (MFMA) with act' and the dropout mask fused.
//                      Activations and gradients stay in LDS between layers;
//                      the ones the weight gradient needs (A_l, dZ_l) are
//                      also written to HBM.
//   dl_mlp_dw_kernel   one workgroup per 16x16 tile of a dW_l = dZ_l^T A_l:
//                      8 waves split the batch rows, fold through LDS; the
//                      tiles of the first column also write db_l = sum dZ_l.
//   dl_mlp_upd_kernel  one wave per neuron row of every layer: the reference
//                      per-row bprop tail (dl_upd_weight / dl_upd_bias, the
//                      max_w2 rescale) and the step-seed advance.
//
// MFMA: v_mfma_f32_16x16x4_f32, lane l supplies A[l & 15][k = l >> 4] and
// B[k = l >> 4][l & 15], C[4 (l >> 4) + r][l & 15] in acc[r].  Each lane's
// k for a step s is k0 + 4 (l >> 4) + s, so one float4 LDS read feeds four
// MFMAs.  The f32 products are exact, as in the reference's float loops.
// ---------------------------------------------------------------------------
#define DL_MAXL 8
#define DL_ROWS 16
// forward/backward kernel: 8 waves, each a chunk of DL_TPW output tiles per
// pass (tiles wave, wave + 8, ...): a 200-unit layer is 13 tiles, two per
// wave, so the serial MFMA + load chain of each wave is half as long as
// with 4 waves of 4 tiles
#define DL_FB_WAVES 8
#define DL_FB_THREADS (64 * DL_FB_WAVES)
#define DL_TPW 2
typedef float dl_f32x4 __attribute__((ext_vector_type(4)));

struct DLNet {
  int nl, B, K, out_kind;        // out_kind: 0 softmax + CE, 1 softmax + quadratic, 2 linear + quadratic
  int ldx;
  float inv_n;
  int width[DL_MAXL + 1];        // width[0] = inputs, width[l + 1] = units of layer l
  int act[DL_MAXL];              // activation of the hidden layer l (its output is A_{l+1})
  unsigned thr[DL_MAXL + 1];     // dropout thresholds: [0] input, [l] of A_l
  int lds_a[DL_MAXL + 1];        // LDS offsets (floats) of A_l (l < nl) and of the logits (l = nl)
  int stride[DL_MAXL + 1];       // their row strides
  int lds_d0, lds_d1, ldsw;      // dZ ping-pong buffers and their row stride
  const float* W[DL_MAXL];       // [width[l+1], width[l]]
  const float* b[DL_MAXL];
  float* A[DL_MAXL];             // [B, width[l]] (A_0 = the input after dropout)
  float* dZ[DL_MAXL];            // [B, width[l+1]]
};

__device__ __forceinline__ dl_f32x4 dl_mfma4(float4 a, float4 b, dl_f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
  return c;
}

__device__ __forceinline__ unsigned long long dl_lcg(unsigned long long s) {
  return s * 6364136223846793005ull + 1442695040888963407ull;
}

__global__ __launch_bounds__(DL_FB_THREADS) void dl_mlp_fb_kernel(const DLNet net, const float* __restrict__ X,
                                                        const long long* __restrict__ idx,
                                                        const long long* __restrict__ ycls,
                                                        const float* __restrict__ yreg,
                                                        const float* __restrict__ wts, unsigned long long seed,
                                                        const unsigned long long* seed_dev, int advance) {
  extern __shared__ float lds[];
  if (seed_dev) seed += advance ? dl_lcg(*seed_dev) : *seed_dev;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g4 = 4 * (lane >> 4), c16 = lane & 15;
  const int r0 = blockIdx.x * DL_ROWS;
  const int B = net.B;
  // ---- input rows (gathered) with input dropout -> LDS A_0 and HBM A_0
  {
    const int P = net.width[0], S = net.stride[0];
    float* a0 = lds + net.lds_a[0];
    for (int e = tid; e < DL_ROWS * S; e += DL_FB_THREADS) {
      const int r = e / S, c = e - r * S;
      const int rg = r0 + r;
      float v = 0.f;
      if (rg < B && c < P) {
        const long long src = idx ? idx[rg] : (long long)rg;
        v = X[src * net.ldx + c];
        if (!dl_keep(seed + 0x5bd1e995ull, (unsigned)rg, (unsigned)c, net.thr[0])) v = 0.f;
        net.A[0][(long long)rg * P + c] = v;
      }
      a0[e] = v;
    }
  }
  __syncthreads();
  // ---- forward
  for (int l = 0; l < net.nl; ++l) {
    const int I = net.width[l], U = net.width[l + 1];
    const int Si = net.stride[l], So = net.stride[l + 1];
    const float* ain = lds + net.lds_a[l];
    float* aout = lds + net.lds_a[l + 1];
    const bool last = l == net.nl - 1;
    const int NT = (U + 15) >> 4, KP = (I + 15) & ~15;
    const float* __restrict__ W = net.W[l];
    const bool vec = (I & 3) == 0;
    const int act = last ? 0 : net.act[l];
    const unsigned thr = last ? 0u : net.thr[l + 1];
    const unsigned long long lseed = seed + 7919ull * (unsigned long long)(l + 1);
    const int nk = KP >> 4;
    // W float4 of tile t (output units t*16 + c16) at k step ks (-> k = 16 ks + g4)
    auto wload = [&](int t, int ks) -> float4 {
      float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
      const int u = t * 16 + c16, kk = ks * 16 + g4;
      if (t < NT && u < U) {
        const float* wr = W + (long long)u * I + kk;
        if (vec && kk + 3 < I) {
          w = *reinterpret_cast<const float4*>(wr);
        } else {
          w.x = kk < I ? wr[0] : 0.f;
          w.y = kk + 1 < I ? wr[1] : 0.f;
          w.z = kk + 2 < I ? wr[2] : 0.f;
          w.w = kk + 3 < I ? wr[3] : 0.f;
        }
      }
      return w;
    };
    for (int t0 = wave; t0 < NT; t0 += DL_FB_WAVES * DL_TPW) {
      dl_f32x4 acc[DL_TPW];
#pragma unroll
      for (int j = 0; j < DL_TPW; ++j) acc[j] = (dl_f32x4){0.f, 0.f, 0.f, 0.f};
      // 4-deep register ring of weight loads: the L2 latency of step ks + 4
      // hides behind the MFMAs of steps ks .. ks + 3
      float4 wq[4][DL_TPW];
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int j = 0; j < DL_TPW; ++j) wq[d][j] = d < nk ? wload(t0 + DL_FB_WAVES * j, d) : make_float4(0.f, 0.f, 0.f, 0.f);
      for (int kb = 0; kb < nk; kb += 4) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int ks = kb + d;
          if (ks < nk) {
            const float4 a = *reinterpret_cast<const float4*>(ain + c16 * Si + ks * 16 + g4);
#pragma unroll
            for (int j = 0; j < DL_TPW; ++j)
              if (t0 + DL_FB_WAVES * j < NT) acc[j] = dl_mfma4(a, wq[d][j], acc[j]);
            if (ks + 4 < nk) {
#pragma unroll
              for (int j = 0; j < DL_TPW; ++j) wq[d][j] = wload(t0 + DL_FB_WAVES * j, ks + 4);
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < DL_TPW; ++j) {
        const int t = t0 + DL_FB_WAVES * j;
        if (t < NT) {
          const int u = t * 16 + c16;
          const float bu = u < U ? net.b[l][u] : 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = g4 + r, rg = r0 + row;
            const float z = acc[j][r] + bu;
            if (last) {
              aout[row * So + u] = u < U ? z : 0.f;
            } else {
              float a = u < U ? dl_act(act, z) : 0.f;
              if (!dl_keep(lseed, (unsigned)rg, (unsigned)u, thr)) a = 0.f;
              aout[row * So + u] = a;
              if (rg < B && u < U) net.A[l + 1][(long long)rg * U + u] = a;
            }
          }
        }
      }
    }
    __syncthreads();
  }
  // ---- output gradient dE/dnet (already * w / n), rows in threads 0..15
  float* dcur = lds + net.lds_d0;
  float* dnext = lds + net.lds_d1;
  {
    const int K = net.K, So = net.stride[net.nl], Kp = (K + 15) & ~15;
    const float* zo = lds + net.lds_a[net.nl];
    if (tid < DL_ROWS) {
      const int row = tid, rg = r0 + row;
      float wr = 0.f;
      long long t = -1;
      float yv = 0.f;
      if (rg < B) {
        const long long src = idx ? idx[rg] : (long long)rg;
        wr = wts ? wts[src] : 1.f;
        if (net.out_kind < 2) {
          t = ycls[src];
          if (t < 0) wr = 0.f;
        } else {
          yv = yreg[src];
        }
      }
      float* dz = dcur + row * net.ldsw;
      float* gdz = net.dZ[net.nl - 1] + (long long)rg * K;
      if (net.out_kind < 2) {
        float mx = -INFINITY;
        for (int k = 0; k < K; ++k) mx = fmaxf(mx, zo[row * So + k]);
        float s = 0.f;
        for (int k = 0; k < K; ++k) s += __expf(zo[row * So + k] - mx);
        const float inv = 1.f / s;
        for (int k = 0; k < K; ++k) {
          const float p = __expf(zo[row * So + k] - mx) * inv;
          const float tt = (k == t) ? 1.f : 0.f;
          const float gk = (net.out_kind == 0 ? (p - tt) : (p - tt) * (1.f - p) * p) * wr * net.inv_n;
          dz[k] = gk;
          if (rg < B) gdz[k] = gk;
        }
      } else {
        const float gk = 2.f * (zo[row * So] - yv) * wr * net.inv_n;
        dz[0] = gk;
        if (rg < B) gdz[0] = gk;
      }
      for (int k = K; k < Kp; ++k) dz[k] = 0.f;
    }
  }
  __syncthreads();
  // ---- backward: dA_l = dZ_l W_l, dZ_{l-1} = dA_l act'(A_l) mask_l
  for (int l = net.nl - 1; l >= 1; --l) {
    const int U = net.width[l + 1], I = net.width[l];
    const int NT = (I + 15) >> 4, KP = (U + 15) & ~15;
    const float* __restrict__ W = net.W[l];
    const float* al = lds + net.lds_a[l];
    const int Sa = net.stride[l];
    const int act = net.act[l - 1];
    const unsigned thr = net.thr[l];
    const unsigned long long lseed = seed + 7919ull * (unsigned long long)l;
    const int nk = KP >> 4;
    // W column slice of tile t (inputs t*16 + c16) at k step ks: rows 16 ks + g4 .. +3
    auto wload = [&](int t, int ks) -> float4 {
      float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
      const int i = t * 16 + c16, kk = ks * 16 + g4;
      if (t < NT && i < I) {
        const float* wc = W + (long long)kk * I + i;
        w.x = kk < U ? wc[0] : 0.f;
        w.y = kk + 1 < U ? wc[I] : 0.f;
        w.z = kk + 2 < U ? wc[2 * I] : 0.f;
        w.w = kk + 3 < U ? wc[3 * I] : 0.f;
      }
      return w;
    };
    for (int t0 = wave; t0 < NT; t0 += DL_FB_WAVES * DL_TPW) {
      dl_f32x4 acc[DL_TPW];
#pragma unroll
      for (int j = 0; j < DL_TPW; ++j) acc[j] = (dl_f32x4){0.f, 0.f, 0.f, 0.f};
      float4 wq[4][DL_TPW];
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int j = 0; j < DL_TPW; ++j) wq[d][j] = d < nk ? wload(t0 + DL_FB_WAVES * j, d) : make_float4(0.f, 0.f, 0.f, 0.f);
      for (int kb = 0; kb < nk; kb += 4) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int ks = kb + d;
          if (ks < nk) {
            const float4 dv = *reinterpret_cast<const float4*>(dcur + c16 * net.ldsw + ks * 16 + g4);
#pragma unroll
            for (int j = 0; j < DL_TPW; ++j)
              if (t0 + DL_FB_WAVES * j < NT) acc[j] = dl_mfma4(dv, wq[d][j], acc[j]);
            if (ks + 4 < nk) {
#pragma unroll
              for (int j = 0; j < DL_TPW; ++j) wq[d][j] = wload(t0 + DL_FB_WAVES * j, ks + 4);
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < DL_TPW; ++j) {
        const int t = t0 + DL_FB_WAVES * j;
        if (t < NT) {
          const int i = t * 16 + c16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = g4 + r, rg = r0 + row;
            float g = 0.f;
            if (i < I && dl_keep(lseed, (unsigned)rg, (unsigned)i, thr)) g = acc[j][r] * dl_dact(act, al[row * Sa + i]);
            dnext[row * net.ldsw + i] = g;
            if (rg < B && i < I) net.dZ[l - 1][(long long)rg * I + i] = g;
          }
        }
      }
    }
    __syncthreads();
    float* tmp = dcur;
    dcur = dnext;
    dnext = tmp;
  }
}

struct DLGrad {
  int nl, B;
  int width[DL_MAXL + 1];
  int tiles_i[DL_MAXL];
  int tile_start[DL_MAXL + 1];
  const float* A[DL_MAXL];
  const float* dZ[DL_MAXL];
  float* dW[DL_MAXL];
  float* db[DL_MAXL];
};

__global__ __launch_bounds__(512) void dl_mlp_dw_kernel(const DLGrad g) {
  __shared__ float red[8][16][17];
  __shared__ float dbr[8][16];
  const int bid = blockIdx.x;
  int l = 0;
  while (l + 1 < g.nl && bid >= g.tile_start[l + 1]) ++l;
  const int local = bid - g.tile_start[l];
  const int ut = local / g.tiles_i[l], it = local - ut * g.tiles_i[l];
  const int U = g.width[l + 1], I = g.width[l], B = g.B;
  const float* __restrict__ dz = g.dZ[l];
  const float* __restrict__ a = g.A[l];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g4 = 4 * (lane >> 4), c16 = lane & 15;
  const int u = ut * 16 + c16, i = it * 16 + c16;
  const bool uok = u < U, iok = i < I, want_db = it == 0;
  dl_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float dbs = 0.f;
  // wave w takes the 16-row chunks q = w, w + 8, ...; a 4-deep ring of
  // chunk loads keeps the L2 latency behind the MFMAs
  const int nq = (B + 15) >> 4;
  auto ld = [&](int q, float4& x, float4& y) {
    const int rr = q * 16 + g4;
    x.x = (rr < B && uok) ? dz[(long long)rr * U + u] : 0.f;
    x.y = (rr + 1 < B && uok) ? dz[(long long)(rr + 1) * U + u] : 0.f;
    x.z = (rr + 2 < B && uok) ? dz[(long long)(rr + 2) * U + u] : 0.f;
    x.w = (rr + 3 < B && uok) ? dz[(long long)(rr + 3) * U + u] : 0.f;
    y.x = (rr < B && iok) ? a[(long long)rr * I + i] : 0.f;
    y.y = (rr + 1 < B && iok) ? a[(long long)(rr + 1) * I + i] : 0.f;
    y.z = (rr + 2 < B && iok) ? a[(long long)(rr + 2) * I + i] : 0.f;
    y.w = (rr + 3 < B && iok) ? a[(long long)(rr + 3) * I + i] : 0.f;
  };
  float4 xq[4], yq[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int q = wave + 8 * d;
    if (q < nq) ld(q, xq[d], yq[d]);
    else xq[d] = yq[d] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int qb = wave; qb < nq; qb += 32) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int q = qb + 8 * d;
      if (q < nq) {
        acc = dl_mfma4(xq[d], yq[d], acc);
        if (want_db) dbs += (xq[d].x + xq[d].y) + (xq[d].z + xq[d].w);
        if (q + 32 < nq) ld(q + 32, xq[d], yq[d]);
      }
    }
  }
  // C[m = u][n = i]: this lane holds u = ut*16 + g4 + r, i = it*16 + c16
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][g4 + r][c16] = acc[r];
  if (want_db) {
    dbs += __shfl_xor(dbs, 16, 64);
    dbs += __shfl_xor(dbs, 32, 64);
    if (lane < 16) dbr[wave][lane] = dbs;
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < 256) {
    const int m = t >> 4, n = t & 15;
    const int uu = ut * 16 + m, ii = it * 16 + n;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += red[w][m][n];
    if (uu < U && ii < I) g.dW[l][(long long)uu * I + ii] = v;
  }
  if (want_db && t < 16 && ut * 16 + t < U) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += dbr[w][t];
    g.db[l][ut * 16 + t] = v;
  }
}

struct DLUpdMulti {
  int nl;
  int width[DL_MAXL + 1];
  int row_start[DL_MAXL + 1];
  float* W[DL_MAXL];
  const float* dW[DL_MAXL];
  float* ada[DL_MAXL];
  float* mom[DL_MAXL];
  float* bias[DL_MAXL];
  const float* db[DL_MAXL];
  float* ada_b[DL_MAXL];
  float* mom_b[DL_MAXL];
  DLUpdate p[DL_MAXL];
};

__global__ __launch_bounds__(256) void dl_mlp_upd_kernel(const DLUpdMulti q, unsigned long long* seed_dev,
                                                         int advance) {
  const int lane = threadIdx.x & 63;
  const int grow = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (advance && seed_dev && grow == 0 && lane == 0) seed_dev[0] = dl_lcg(seed_dev[0]);
  if (grow >= q.row_start[q.nl]) return;
  int l = 0;
  while (l + 1 < q.nl && grow >= q.row_start[l + 1]) ++l;
  const int row = grow - q.row_start[l], I = q.width[l];
  const DLUpdate& p = q.p[l];
  float* w = q.W[l] + (long long)row * I;
  const float* gw = q.dW[l] + (long long)row * I;
  float* ada = q.ada[l];
  float* mom = q.mom[l];
  float g2sum = 0.f, r2 = 0.f;
  for (int c = lane; c < I; c += 64) {
    float g2;
    const float nw = dl_upd_weight(w[c], gw[c], ada + 2 * ((long long)row * I + c),
                                   mom ? mom + (long long)row * I + c : nullptr, p, &g2);
    w[c] = nw;
    g2sum += g2;
    r2 += nw * nw;
  }
  g2sum = wave_sum(g2sum);
  if (p.max_w2 < 3.0e38f) {
    r2 = wave_sum(r2);
    if (r2 > p.max_w2) {
      const float scale = sqrtf(p.max_w2 / r2);
      for (int c = lane; c < I; c += 64) w[c] *= scale;
    }
  }
  if (lane == 0) dl_upd_bias(q.bias[l], q.db[l], q.ada_b[l], q.mom_b[l], nullptr, row, g2sum / (float)max(I, 1), p);
}

extern "C" {

// Step-seed advance (an LCG step of the device seed): captured once in the
// training-step graph, so every replay draws new dropout masks.
__global__ void dl_seed_kernel(unsigned long long* s) {
  if (threadIdx.x == 0) s[0] = s[0] * 6364136223846793005ull + 1442695040888963407ull;
}

extern "C" int h2o_dl_seed_advance(unsigned long long* s, hipStream_t st) {
  hipLaunchKernelGGL(dl_seed_kernel, dim3(1), dim3(64), 0, st, s);
  H2O_CHECK_LAUNCH();
}

int h2o_dl_fwd(float* Z, const float* bias, float* A, int B, int U, int act, float drop_ratio,
               unsigned long long seed, const unsigned long long* seed_dev, int mode, float test_scale,
               hipStream_t s) {
  if (B <= 0 || U <= 0) return 0;
  const unsigned thr = drop_ratio <= 0.f ? 0u : (unsigned)fminf(drop_ratio * 4294967296.f, 4294967295.f);
  const long long n = (long long)B * U;
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(dl_fwd_kernel, dim3(grid), dim3(256), 0, s, Z, bias, A, B, U, act, thr, seed, seed_dev, mode,
                     test_scale);
  H2O_CHECK_LAUNCH();
}

// dbias must be zeroed by the caller (atomics accumulate into it)
int h2o_dl_bwd(const float* dA, const float* A, const float* Z, float* dZ, float* dbias, int B, int U, int act,
               float drop_ratio, unsigned long long seed, const unsigned long long* seed_dev, hipStream_t s) {
  if (B <= 0 || U <= 0) return 0;
  const unsigned thr = drop_ratio <= 0.f ? 0u : (unsigned)fminf(drop_ratio * 4294967296.f, 4294967295.f);
  const int gx = (U + 255) / 256;
  // enough row blocks to fill the chip (>= 1024 workgroups), >= 16 rows each
  int gy = std::max(1, std::min((B + 15) / 16, (2048 + gx - 1) / gx));
  const int rpb = (B + gy - 1) / gy;
  gy = (B + rpb - 1) / rpb;
  hipLaunchKernelGGL(dl_bwd_kernel, dim3(gx, gy), dim3(256), 0, s, dA, A, Z, dZ, dbias, B, U, act, thr, seed, seed_dev,
                     rpb);
  H2O_CHECK_LAUNCH();
}

int h2o_dl_update(float* W, const float* dW, float* ada, float* mom, float* bias, const float* dbias, float* ada_b,
                  float* mom_b, const float* avg_act, int U, int I, float rho, float eps, float rate, float momentum,
                  float l1, float l2, float max_w2, int use_ada, int nesterov, int has_momenta, float sparsity_beta,
                  float average_activation, hipStream_t s) {
  if (U <= 0) return 0;
  DLUpdate p{rho, eps, rate, momentum, l1, l2, max_w2, use_ada, nesterov, has_momenta, sparsity_beta,
             average_activation};
  hipLaunchKernelGGL(dl_update_kernel, dim3(U), dim3(256), 0, s, W, dW, ada, mom, bias, dbias, ada_b, mom_b, avg_act,
                     U, I, p);
  H2O_CHECK_LAUNCH();
}

int h2o_dl_softmax(float* Z, const float* bias, float* P, const long long* y, const float* w, float* dZ,
                   float* loss_out, int B, int K, float inv_n, int loss, hipStream_t s) {
  if (B <= 0 || K <= 0) return 0;
  hipLaunchKernelGGL(dl_softmax_kernel, dim3((B + 3) / 4), dim3(256), 0, s, Z, bias, P, y, w, dZ, loss_out, B, K,
                     inv_n, loss);
  H2O_CHECK_LAUNCH();
}

// Fused training step of a dense MLP (dl_mlp_* kernels).  Arrays are per
// layer (nl = hidden layers + output): width[nl + 1], act[nl - 1],
// drop[nl] ([0] input dropout, [l] of hidden layer l-1's output), W/b/A/dZ/
// dW/db/ada/mom/ada_b/mom_b[nl], ups[nl].  X [n, ldx] with idx [B] (int64,
// null = rows 0..B-1); ycls (int64, classification) or yreg (float);
// wts per row (may be null).  Returns -2 when the network does not fit the
// fused kernels (the caller runs the unfused step).
int h2o_dl_mlp_step(int nl, const int* width, const int* act, const float* drop, const float* const* W,
                    const float* const* b, float* const* A, float* const* dZ, float* const* dW, float* const* db,
                    float* const* ada, float* const* mom, float* const* ada_b, float* const* mom_b,
                    const DLUpdate* ups, const float* X, int ldx, const long long* idx, const long long* ycls,
                    const float* yreg, const float* wts, int B, int out_kind, float inv_n, unsigned long long seed,
                    unsigned long long* seed_dev, int advance, hipStream_t s) {
  if (nl < 1 || nl > DL_MAXL || B <= 0) return -2;
  DLNet net{};
  net.nl = nl;
  net.B = B;
  net.K = width[nl];
  net.out_kind = out_kind;
  net.ldx = ldx;
  net.inv_n = inv_n;
  int off = 0, maxw = 0;
  for (int l = 0; l <= nl; ++l) {
    net.width[l] = width[l];
    const int pw = (width[l] + 15) & ~15;
    net.lds_a[l] = off;
    net.stride[l] = pw + 4;
    off += DL_ROWS * (pw + 4);
    if (l >= 1) maxw = std::max(maxw, pw);
    if (l < nl) net.thr[l] = drop[l] <= 0.f ? 0u : (unsigned)fminf(drop[l] * 4294967296.f, 4294967295.f);
  }
  if (out_kind == 2 && width[nl] != 1) return -2;
  if (width[nl] > 64) return -2;
  net.ldsw = maxw + 4;
  net.lds_d0 = off;
  off += DL_ROWS * net.ldsw;
  net.lds_d1 = off;
  off += DL_ROWS * net.ldsw;
  const size_t lds_bytes = (size_t)off * sizeof(float);
  if (lds_bytes > 160 * 1024) return -2;
  for (int l = 0; l < nl; ++l) {
    if (l < nl - 1) net.act[l] = act[l];
    net.W[l] = W[l];
    net.b[l] = b[l];
    net.A[l] = A[l];
    net.dZ[l] = dZ[l];
  }
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)dl_mlp_fb_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(dl_mlp_fb_kernel, dim3((B + DL_ROWS - 1) / DL_ROWS), dim3(DL_FB_THREADS), lds_bytes, s, net, X, idx, ycls,
                     yreg, wts, seed, seed_dev, advance);
  DLGrad g{};
  g.nl = nl;
  g.B = B;
  int nt = 0;
  for (int l = 0; l < nl; ++l) {
    g.width[l] = width[l];
    g.tiles_i[l] = (width[l] + 15) >> 4;
    g.tile_start[l] = nt;
    nt += g.tiles_i[l] * ((width[l + 1] + 15) >> 4);
    g.A[l] = A[l];
    g.dZ[l] = dZ[l];
    g.dW[l] = dW[l];
    g.db[l] = db[l];
  }
  g.width[nl] = width[nl];
  g.tile_start[nl] = nt;
  hipLaunchKernelGGL(dl_mlp_dw_kernel, dim3(nt), dim3(512), 0, s, g);
  DLUpdMulti q{};
  q.nl = nl;
  int nr = 0;
  for (int l = 0; l < nl; ++l) {
    q.width[l] = width[l];
    q.row_start[l] = nr;
    nr += width[l + 1];
    q.W[l] = const_cast<float*>(W[l]);
    q.dW[l] = dW[l];
    q.ada[l] = ada[l];
    q.mom[l] = mom[l];
    q.bias[l] = const_cast<float*>(b[l]);
    q.db[l] = db[l];
    q.ada_b[l] = ada_b[l];
    q.mom_b[l] = mom_b[l];
    q.p[l] = ups[l];
  }
  q.width[nl] = width[nl];
  q.row_start[nl] = nr;
  hipLaunchKernelGGL(dl_mlp_upd_kernel, dim3((nr + 3) / 4), dim3(256), 0, s, q, seed_dev, advance);
  H2O_CHECK_LAUNCH();
}

}  // extern "C"


// ---------------------------------------------------------------------------
// Tiled f32-MFMA GEMM for the layers the LDS-resident fused step does not
// cover (wide hidden layers, maxout, autoencoders): C[M][N] = opA . opB with
// opA(m, k) = A[m * sam + k * sak] and opB(k, n) = B[k * sbk + n * sbn], so
// the three products of a training step -- Z = A W^T, dA = dZ W, dW = dZ^T A
// -- are one kernel with different strides (no library GEMM).  A 256-thread
// workgroup owns a 64 x 64 tile of C; each of its 4 waves a 32 x 32 quarter
// (2 x 2 blocks of v_mfma_f32_16x16x4f32: exact f32 products, f32
// accumulation like an f32 BLAS GEMM).  K advances in 32-wide slabs staged
// through LDS (double buffered: the next slab's global loads are in flight
// during the current slab's MFMAs); the loader walks the contiguous
// dimension of each operand so the global loads coalesce for every
// transpose.  Blocks are mapped XCD-aware.
// ---------------------------------------------------------------------------
#define DLG_TK 32
// BM x BN blocks of 16 x 16 per wave, 2 x 2 waves per workgroup: the
// workgroup tile is (32 BM) x (32 BN).  BM = BN = 2 (64 x 64) is the default;
// (2, 4) and (4, 4) trade grid size for operand reuse (H2O3_DL_GEMM_TILE).
template <int BM, int BN>
__global__ __launch_bounds__(256, BM * BN <= 4 ? 4 : 2) void dl_gemm_kernel(int M, int N, int K, const float* __restrict__ A, long long sam,
                                                         long long sak, const float* __restrict__ B, long long sbk,
                                                         long long sbn, float* __restrict__ C, int ntn, int ntiles,
                                                         int kchunk, float* __restrict__ Cw) {
  constexpr int TM = 32 * BM, TN = 32 * BN;
  constexpr int LA = TM * DLG_TK / 256, LB = TN * DLG_TK / 256;   // staged elements per thread
  // both operands k-inner in LDS (B transposed to [n][k]), rows padded to
  // 36 floats: one ds_read_b128 gives a lane 4 consecutive k of its row, and
  // the 16 rows of a 16-lane group hit distinct 4-bank groups
  __shared__ __align__(16) float As[2][TM][DLG_TK + 4];   // [m][k]
  __shared__ __align__(16) float Bs[2][TN][DLG_TK + 4];   // [n][k]
  const int nwg = gridDim.x;
  const int bid0 = xcd_remap(blockIdx.x, nwg);
  const int ks = bid0 / ntiles, bid = bid0 - ks * ntiles;   // split-K slice, output tile
  const int tm = bid / ntn, tn = bid - (bid / ntn) * ntn;
  const int kbeg = ks * kchunk, kend = min(K, kbeg + kchunk);
  const int m0 = tm * TM, n0 = tn * TN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = (wv >> 1) * (16 * BM), wn = (wv & 1) * (16 * BN);
  const bool a_kfast = sak == 1, b_nfast = sbn == 1;
  float ra[LA], rb[LB];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < LA; ++u) {
      const int e = tid + u * 256;
      int m, k;
      if (a_kfast) { m = e >> 5; k = e & 31; } else { k = e / TM; m = e - (e / TM) * TM; }
      const int gm = m0 + m, gk = k0 + k;
      ra[u] = (gm < M && gk < kend) ? A[(long long)gm * sam + (long long)gk * sak] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int e = tid + u * 256;
      int kb, n;
      if (b_nfast) { kb = e / TN; n = e - (e / TN) * TN; } else { n = e >> 5; kb = e & 31; }
      const int gk2 = k0 + kb, gn = n0 + n;
      rb[u] = (gk2 < kend && gn < N) ? B[(long long)gk2 * sbk + (long long)gn * sbn] : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < LA; ++u) {
      const int e = tid + u * 256;
      if (a_kfast) As[buf][e >> 5][e & 31] = ra[u];
      else As[buf][e - (e / TM) * TM][e / TM] = ra[u];
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int e = tid + u * 256;
      if (b_nfast) Bs[buf][e - (e / TN) * TN][e / TN] = rb[u];
      else Bs[buf][e >> 5][e & 31] = rb[u];
    }
  };
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 acc[BM][BN];
#pragma unroll
  for (int i = 0; i < BM; ++i)
#pragma unroll
    for (int j = 0; j < BN; ++j) acc[i][j] = (f4){0.f, 0.f, 0.f, 0.f};
  const int nslab = kend > kbeg ? (kend - kbeg + DLG_TK - 1) / DLG_TK : 0;
  if (nslab > 0) {
    load(kbeg);
    store(0);
  }
  __syncthreads();
  const int li = lane & 15, lg = lane >> 4;
  for (int s = 0; s < nslab; ++s) {
    const int cur = s & 1;
    if (s + 1 < nslab) load(kbeg + (s + 1) * DLG_TK);
    // MFMA j of a 16-deep chunk covers k = c + 4 * lg + j across the lane
    // groups (same permutation on both operands: the sum over k is unchanged)
#pragma unroll
    for (int c = 0; c < DLG_TK; c += 16) {
      f4 av[BM], bv[BN];
#pragma unroll
      for (int i = 0; i < BM; ++i) av[i] = *(const f4*)&As[cur][wm + 16 * i + li][c + 4 * lg];
#pragma unroll
      for (int j = 0; j < BN; ++j) bv[j] = *(const f4*)&Bs[cur][wn + 16 * j + li][c + 4 * lg];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < BM; ++i)
#pragma unroll
          for (int j = 0; j < BN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][q], bv[j][q], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nslab) store(cur ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < BM; ++i)
#pragma unroll
    for (int j = 0; j < BN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + 16 * i + 4 * lg + r, gn = n0 + wn + 16 * j + li;
        if (gm < M && gn < N) {
          if (Cw != nullptr) Cw[((long long)ks * M + gm) * N + gn] = acc[i][j][r];
          else C[(long long)gm * N + gn] = acc[i][j][r];
        }
      }
}

// Split-K partials [ks][M*N] summed in slice order (deterministic).
__global__ __launch_bounds__(256) void dl_gemm_reduce_kernel(const float* __restrict__ Cw, int ksplit, long long mn,
                                                             float* __restrict__ C) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < mn; i += (long long)gridDim.x * 256) {
    float v = 0.f;
    for (int k = 0; k < ksplit; ++k) v += Cw[(long long)k * mn + i];
    C[i] = v;
  }
}

static int dl_gemm_tile() {   // 0: 64 x 64, 1: 64 x 128, 2: 128 x 128 workgroup tiles (H2O3_DL_GEMM_TILE)
  static int t = -1;
  if (t < 0) {
    const char* e = getenv("H2O3_DL_GEMM_TILE");
    t = e == nullptr ? 0 : (strcmp(e, "64x128") == 0 ? 1 : (strcmp(e, "128x128") == 0 ? 2 : 0));
  }
  return t;
}

// Split-K plan: slices of K (multiples of the 32-deep slab) until the grid has
// ~4 workgroups per CU -- the thin products of a step (the 2-unit output
// layer, the input layer's dW) have few output tiles but K = batch or width.
static void dl_gemm_plan(int M, int N, int K, int TM, int TN, int& ksplit, int& kchunk) {
  const int tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  const int nslab = (K + DLG_TK - 1) / DLG_TK;
  if (tiles <= 0 || nslab <= 0) {
    ksplit = 1;
    kchunk = max(K, 1);
    return;
  }
  int want = (1024 + tiles - 1) / tiles;
  want = min(want, max(1, nslab / 4));        // at least 4 slabs (128 deep) per slice
  want = min(want, 32);
  const int spk = (nslab + want - 1) / max(want, 1);
  kchunk = spk * DLG_TK;
  ksplit = K > 0 ? (K + kchunk - 1) / kchunk : 1;
}

static void dl_gemm_dims(int& TM, int& TN) {
  const int t = dl_gemm_tile();
  TM = t == 2 ? 128 : 64;
  TN = t == 0 ? 64 : 128;
}

extern "C" long long h2o_dl_gemm_ws(int M, int N, int K) {
  int ks, kc, TM, TN;
  dl_gemm_dims(TM, TN);
  dl_gemm_plan(M, N, K, TM, TN, ks, kc);
  return ks > 1 ? (long long)ks * M * N : 0;
}

extern "C" int h2o_dl_gemm(int M, int N, int K, const float* A, long long sam, long long sak, const float* B,
                           long long sbk, long long sbn, float* C, float* ws, long long ws_elems, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (K < 0 || !A || !B || !C) return (int)hipErrorInvalidValue;
  int TM, TN;
  dl_gemm_dims(TM, TN);
  const int ntm = (M + TM - 1) / TM, ntn = (N + TN - 1) / TN;
  int ksplit, kchunk;
  dl_gemm_plan(M, N, K, TM, TN, ksplit, kchunk);
  if (ksplit > 1 && (ws == nullptr || ws_elems < (long long)ksplit * M * N)) {
    ksplit = 1;                               // no workspace: one slice
    kchunk = max(K, 1);
  }
  const int ntiles = ntm * ntn;
  float* cw = ksplit > 1 ? ws : (float*)nullptr;
  const dim3 grid(ntiles * ksplit);
  const int t = dl_gemm_tile();
  if (t == 2)
    hipLaunchKernelGGL((dl_gemm_kernel<4, 4>), grid, dim3(256), 0, s, M, N, K, A, sam, sak, B, sbk, sbn, C, ntn,
                       ntiles, kchunk, cw);
  else if (t == 1)
    hipLaunchKernelGGL((dl_gemm_kernel<2, 4>), grid, dim3(256), 0, s, M, N, K, A, sam, sak, B, sbk, sbn, C, ntn,
                       ntiles, kchunk, cw);
  else
    hipLaunchKernelGGL((dl_gemm_kernel<2, 2>), grid, dim3(256), 0, s, M, N, K, A, sam, sak, B, sbk, sbn, C, ntn,
                       ntiles, kchunk, cw);
  if (ksplit > 1) {
    const long long mn = (long long)M * N;
    const int g = (int)min((mn + 255) / 256, 4096LL);
    hipLaunchKernelGGL(dl_gemm_reduce_kernel, dim3(g), dim3(256), 0, s, ws, ksplit, mn, C);
  }
  H2O_CHECK_LAUNCH();
}
