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
