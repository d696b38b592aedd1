// Forest scoring: traverse every tree for every row and accumulate per-class
// leaf values.  Reference: hex/tree/CompressedTree.java:score0 (byte-coded
// tree walk per row) and SharedTreeModel.score0.
//
// The forest is flattened into struct-of-arrays node tables shared by all
// trees (feat / thr / left / right / na_left / cat bitset / value).  One
// thread scores one row against a block of trees; the raw data is column-
// major float32 (the Frame's own column tensors stacked), NaN = NA,
// categorical columns hold their level code as a float.
#include "common.h"

__global__ __launch_bounds__(256) void forest_predict_kernel(
    const float* __restrict__ X, long long N, const int* __restrict__ feat, const float* __restrict__ thr,
    const int* __restrict__ left, const int* __restrict__ right, const uint8_t* __restrict__ na_left,
    const int* __restrict__ cat_off, const int* __restrict__ cat_len, const uint8_t* __restrict__ cat_bits,
    const float* __restrict__ value, const int* __restrict__ roots, const int* __restrict__ tclass, int T,
    int K, float* __restrict__ out, int* __restrict__ leaf_out) {
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  for (int t = 0; t < T; ++t) {
    int nd = roots[t];
    int l = left[nd];
    while (l >= 0) {
      const float x = X[(size_t)feat[nd] * N + r];
      bool go_left;
      const int co = cat_off[nd];
      if (co >= 0) {
        if (x != x) go_left = na_left[nd];
        else {
          const int c = (int)x;
          go_left = (c < 0 || c >= cat_len[nd]) ? (na_left[nd] != 0) : (cat_bits[co + c] != 0);
        }
      } else {
        go_left = (x != x) ? (na_left[nd] != 0) : (x < thr[nd]);
      }
      nd = go_left ? l : right[nd];
      l = left[nd];
    }
    if (out) out[r * K + tclass[t]] += value[nd];
    if (leaf_out) leaf_out[r * T + t] = nd - roots[t];
  }
}

extern "C" int h2o_forest_predict(const float* X, long long N, const int* feat, const float* thr, const int* left,
                                  const int* right, const uint8_t* na_left, const int* cat_off, const int* cat_len,
                                  const uint8_t* cat_bits, const float* value, const int* roots, const int* tclass,
                                  int T, int K, float* out, int* leaf_out, hipStream_t s) {
  if (N <= 0 || T <= 0) return 0;
  const int threads = 256;
  const long long blocks = (N + threads - 1) / threads;
  hipLaunchKernelGGL(forest_predict_kernel, dim3((unsigned)blocks), dim3(threads), 0, s, X, N, feat, thr, left, right,
                     na_left, cat_off, cat_len, cat_bits, value, roots, tclass, T, K, out, leaf_out);
  return (int)hipGetLastError();
}
