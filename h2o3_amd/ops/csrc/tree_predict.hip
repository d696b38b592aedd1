// Forest scoring: traverse every tree for every row and accumulate per-class
// leaf values.  Reference: hex/tree/CompressedTree.java:score0 (byte-coded
// tree walk per row) and SharedTreeModel.score0.
//
// The forest is flattened into one packed 16-byte node table shared by all
// trees (plus leaf values and categorical bitsets).  One thread scores one
// row against every tree; the raw data is column-
// major float32 (the Frame's own column tensors stacked), NaN = NA,
// categorical columns hold their level code as a float.
#include "common.h"
#include <cstdlib>

// Packed node (16 B, one load per visit): x = feature | NA-left << 30 |
// categorical << 31, the threshold's bits, left, right (-1 at a leaf).  The
// per-row sum stays in a register for single-output forests (K == 1) and is
// stored once per row; multi-class forests add into out[r, class].
// TW trees walked together per thread: TW independent node -> feature ->
// node load chains in flight instead of one (the walk is latency-bound).
template <bool K1, int TW>
__global__ __launch_bounds__(256) void forest_predict_kernel(
    const float* __restrict__ X, long long N, const int4* __restrict__ nodes, const int* __restrict__ cat_off,
    const int* __restrict__ cat_len, const uint8_t* __restrict__ cat_bits, const float* __restrict__ value,
    const int* __restrict__ roots, const int* __restrict__ tclass, int T, int K, float* __restrict__ out,
    int* __restrict__ leaf_out) {
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  float acc = 0.f;
  auto go = [&](const int4& n, int nd) -> int {
    const int f = n.x & 0x3FFFFFFF;
    const float x = X[(size_t)f * N + r];
    const bool nal = (n.x >> 30) & 1;
    bool go_left;
    if (n.x < 0) {   // categorical: left-level bitset
      if (x != x) go_left = nal;
      else {
        const int c = (int)x;
        go_left = (c < 0 || c >= cat_len[nd]) ? nal : (cat_bits[cat_off[nd] + c] != 0);
      }
    } else {
      go_left = (x != x) ? nal : (x < __int_as_float(n.y));
    }
    return go_left ? n.z : n.w;
  };
  for (int t0 = 0; t0 < T; t0 += TW) {
    int nd[TW];
    int4 n[TW];
#pragma unroll
    for (int k = 0; k < TW; ++k) {
      nd[k] = t0 + k < T ? roots[t0 + k] : -1;
      n[k] = nd[k] >= 0 ? nodes[nd[k]] : int4{0, 0, -1, -1};
    }
    bool live = true;
    while (live) {
      live = false;
#pragma unroll
      for (int k = 0; k < TW; ++k) {
        if (n[k].z >= 0) {
          nd[k] = go(n[k], nd[k]);
          n[k] = nodes[nd[k]];
          live |= n[k].z >= 0;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < TW; ++k) {
      if (nd[k] < 0) continue;
      const int t = t0 + k;
      if (leaf_out) leaf_out[r * T + t] = nd[k] - roots[t];
      if constexpr (K1) acc += value[nd[k]];
      else if (out) out[r * K + tclass[t]] += value[nd[k]];
    }
  }
  if constexpr (K1) {
    if (out) out[r] += acc;
  }
}

extern "C" int h2o_forest_predict(const float* X, long long N, const int* nodes, const int* cat_off,
                                  const int* cat_len, const uint8_t* cat_bits, const float* value, const int* roots,
                                  const int* tclass, int T, int K, float* out, int* leaf_out, hipStream_t s) {
  if (N <= 0 || T <= 0) return 0;
  const int threads = 256;
  const long long blocks = (N + threads - 1) / threads;
  // trees per thread walked together (H2O3_PREDICT_TW = 1 / 2 / 4, default 2)
  static const int tw = getenv("H2O3_PREDICT_TW") ? atoi(getenv("H2O3_PREDICT_TW")) : 2;
#define FP_LAUNCH(K1_, TW_)                                                                                   \
  hipLaunchKernelGGL((forest_predict_kernel<K1_, TW_>), dim3((unsigned)blocks), dim3(threads), 0, s, X, N,      \
                     (const int4*)nodes, cat_off, cat_len, cat_bits, value, roots, tclass, T, K, out, leaf_out)
  if (K == 1) {
    if (tw >= 4) FP_LAUNCH(true, 4);
    else if (tw == 1) FP_LAUNCH(true, 1);
    else FP_LAUNCH(true, 2);
  } else {
    if (tw >= 4) FP_LAUNCH(false, 4);
    else if (tw == 1) FP_LAUNCH(false, 1);
    else FP_LAUNCH(false, 2);
  }
#undef FP_LAUNCH
  return (int)hipGetLastError();
}
