// Deep Learning (MLP) kernels: the fused element-wise / per-neuron parts of
// a training step; the dense products run on the library GEMM (hipBLASLt).
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
    const float wv = w[c];
    const float grad = gw[c] + (wv > 0.f ? p.l1 : (wv < 0.f ? -p.l1 : 0.f)) + wv * p.l2;
    float nw;
    if (p.ada) {
      float* a2 = ada + 2 * ((long long)row * I + c);
      const float g2 = grad * grad;
      g2sum += g2;
      const float eg2 = p.rho * a2[1] + (1.f - p.rho) * g2;
      const float rate = sqrtf((a2[0] + p.eps) / (eg2 + p.eps));
      a2[1] = eg2;
      a2[0] = p.rho * a2[0] + (1.f - p.rho) * rate * rate * g2;
      nw = wv - rate * grad;
    } else if (!p.nesterov) {
      const float delta = -p.rate * grad;
      nw = wv + delta;
      if (p.has_momenta) {
        float* m = mom + (long long)row * I + c;
        nw += p.momentum * m[0];
        m[0] = delta;
      }
    } else {
      float tmp = -grad;
      if (p.has_momenta) {
        float* m = mom + (long long)row * I + c;
        m[0] = m[0] * p.momentum + tmp;
        tmp = m[0];
      }
      nw = wv + p.rate * tmp;
    }
    w[c] = nw;
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
  if (threadIdx.x == 0) {
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

}  // extern "C"
