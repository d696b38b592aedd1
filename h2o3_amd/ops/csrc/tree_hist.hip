// GPU tree engine kernels: per-node feature histograms (LDS-staged), stable
// row partition, and per-row leaf assignment.
//
// Re-design of the reference's ScoreBuildHistogram2 MRTask
// (h2o-algos/src/main/java/hex/tree/ScoreBuildHistogram2.java) and the
// DHistogram accumulation (hex/tree/DHistogram.java:updateHisto): instead of
// one Java histogram object per (node, column) filled chunk-by-chunk, rows are
// kept grouped by tree node (ridx permutation + per-node segments), the
// binned feature matrix is row-major uint8/uint16, and one workgroup
// accumulates a [feature-group x bins x channels] histogram of one node's row
// range in LDS before flushing the non-zero bins to HBM with float atomics.
//
// Channels (MODE):
//   0 : H2O squared-error criterion  (w, w*y, w*y*y)   C = 3
//   1 : second-order (XGBoost)       (g, h)            C = 2
//   2 : weighted count               (w)               C = 1
//
// Histogram layout in HBM: hist[F][n_slots][Bs][C] (feature-major so a
// multi-GPU reduce-scatter can shard by feature).
#include "common.h"

template <int MODE> struct Chan { static constexpr int C = MODE == 0 ? 3 : (MODE == 1 ? 2 : 1); };

template <typename CodeT> struct Code4;
template <> struct Code4<uint8_t> {
  typedef uint32_t vec;
  __device__ static inline void unpack(vec v, int* c) {
    c[0] = v & 0xff; c[1] = (v >> 8) & 0xff; c[2] = (v >> 16) & 0xff; c[3] = v >> 24;
  }
};
template <> struct Code4<uint16_t> {
  typedef uint2 vec;
  __device__ static inline void unpack(vec v, int* c) {
    c[0] = v.x & 0xffff; c[1] = v.x >> 16; c[2] = v.y & 0xffff; c[3] = v.y >> 16;
  }
};

// work[i] = (slot, pos_start, pos_count, unused)
template <typename CodeT, int MODE>
__global__ __launch_bounds__(1024) void hist_build_kernel(
    const CodeT* __restrict__ codes, int Fp, const int* __restrict__ ridx,
    const float* __restrict__ va, const float* __restrict__ vb,
    const int4* __restrict__ work, int F, int FG, int Bs,
    double* __restrict__ hist, int n_slots) {
  constexpr int C = Chan<MODE>::C;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int4 wk = work[blockIdx.x];
  const int fg0 = blockIdx.y * FG;
  const int nf = min(FG, F - fg0);          // real features in this group
  const int nf4 = min(FG, Fp - fg0);        // loadable (padded) features
  const int stride_f = Bs * C;
  const int total = FG * stride_f;
  for (int i = threadIdx.x; i < total; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();

  const int pend = wk.y + wk.z;
  for (int p = wk.y + threadIdx.x; p < pend; p += blockDim.x) {
    const int r = ridx[p];
    float c0, c1 = 0.f, c2 = 0.f;
    if (MODE == 0) {
      const float y = va[r];
      const float w = vb ? vb[r] : 1.f;
      if (w == 0.f) continue;
      c0 = w; c1 = w * y; c2 = c1 * y;
    } else if (MODE == 1) {
      c0 = va[r]; c1 = vb[r];
      if (c0 == 0.f && c1 == 0.f) continue;
    } else {
      c0 = vb ? vb[r] : 1.f;
      if (c0 == 0.f) continue;
    }
    const CodeT* row = codes + (size_t)r * Fp + fg0;
    for (int j = 0; j < nf4; j += 4) {
      typename Code4<CodeT>::vec v = *reinterpret_cast<const typename Code4<CodeT>::vec*>(row + j);
      int c[4];
      Code4<CodeT>::unpack(v, c);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (j + k < nf) {
          float* h = lds + (j + k) * stride_f + c[k] * C;
          lds_add(h, c0);
          if (C > 1) lds_add(h + 1, c1);
          if (C > 2) lds_add(h + 2, c2);
        }
      }
    }
  }
  __syncthreads();
  const int tot_real = nf * stride_f;
  for (int i = threadIdx.x; i < tot_real; i += blockDim.x) {
    const float v = lds[i];
    if (v != 0.f) {
      const int j = i / stride_f;
      const int rem = i - j * stride_f;
      gbl_add(hist + ((size_t)(fg0 + j) * n_slots + wk.x) * stride_f + rem, (double)v);
    }
  }
}

template <typename CodeT>
static int launch_hist(const void* codes, int Fp, const int* ridx, const float* va, const float* vb,
                       const int4* work, int n_work, int F, int FG, int Bs, double* hist, int n_slots,
                       int mode, int threads, hipStream_t s) {
  const int n_fg = (F + FG - 1) / FG;
  dim3 grid(n_work, n_fg);
  const int C = mode == 0 ? 3 : (mode == 1 ? 2 : 1);
  size_t lds = (size_t)FG * Bs * C * sizeof(float);
  const CodeT* cc = (const CodeT*)codes;
  switch (mode) {
    case 0: hipLaunchKernelGGL((hist_build_kernel<CodeT, 0>), grid, dim3(threads), lds, s, cc, Fp, ridx, va, vb, work, F, FG, Bs, hist, n_slots); break;
    case 1: hipLaunchKernelGGL((hist_build_kernel<CodeT, 1>), grid, dim3(threads), lds, s, cc, Fp, ridx, va, vb, work, F, FG, Bs, hist, n_slots); break;
    default: hipLaunchKernelGGL((hist_build_kernel<CodeT, 2>), grid, dim3(threads), lds, s, cc, Fp, ridx, va, vb, work, F, FG, Bs, hist, n_slots); break;
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
__global__ __launch_bounds__(256) void part_count_kernel(
    const CodeT* __restrict__ codes, long long rs, long long fs, const int* __restrict__ ridx,
    const int4* __restrict__ work, const int* __restrict__ feat, const uint8_t* __restrict__ masks,
    int Bs, int* __restrict__ cnt) {
  const int4 wk = work[blockIdx.x];
  const int f = feat[wk.x];
  const uint8_t* m = masks + (size_t)wk.x * Bs;
  int local = 0;
  for (int p = wk.y + threadIdx.x; p < wk.y + wk.z; p += blockDim.x) {
    const int r = ridx[p];
    const int c = codes[(size_t)r * rs + (size_t)f * fs];
    local += m[c] ? 1 : 0;
  }
  // block reduce
  __shared__ int red[4];
  for (int o = 32; o > 0; o >>= 1) local += __shfl_xor(local, o, 64);
  if (lane_id() == 0) red[wave_id()] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < (int)(blockDim.x / 64); ++w) t += red[w];
    cnt[blockIdx.x] = t;
  }
}

// loff[i], roff[i]: destination start of chunk i's left / right rows.
template <typename CodeT>
__global__ __launch_bounds__(256) void part_scatter_kernel(
    const CodeT* __restrict__ codes, long long rs, long long fs, const int* __restrict__ ridx,
    const int4* __restrict__ work, const int* __restrict__ feat, const uint8_t* __restrict__ masks,
    int Bs, const int* __restrict__ loff, const int* __restrict__ roff, int* __restrict__ out) {
  const int4 wk = work[blockIdx.x];
  const int f = feat[wk.x];
  const uint8_t* m = masks + (size_t)wk.x * Bs;
  __shared__ int wl[4];
  int lbase = loff[blockIdx.x], rbase = roff[blockIdx.x];
  const int nw = blockDim.x / 64;
  for (int t0 = wk.y; t0 < wk.y + wk.z; t0 += blockDim.x) {
    const int p = t0 + threadIdx.x;
    const bool valid = p < wk.y + wk.z;
    int r = 0;
    bool left = false;
    if (valid) {
      r = ridx[p];
      left = m[codes[(size_t)r * rs + (size_t)f * fs]] != 0;
    }
    const unsigned long long bl = __ballot(valid && left);
    const unsigned long long lt = (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
    const int wpre = __popcll(bl & lt);
    if (lane_id() == 0) wl[wave_id()] = __popcll(bl);
    __syncthreads();
    int lpre = 0, ltot = 0;
    for (int w = 0; w < nw; ++w) {
      const int c = wl[w];
      if (w < wave_id()) lpre += c;
      ltot += c;
    }
    const int tile_n = min((int)blockDim.x, wk.y + wk.z - t0);
    if (valid) {
      const int li = lpre + wpre;              // lefts before me in tile
      const int my_idx = threadIdx.x;          // position within tile
      if (left) out[lbase + li] = r;
      else out[rbase + (my_idx - li)] = r;
    }
    lbase += ltot;
    rbase += tile_n - ltot;
    __syncthreads();
  }
}

// nid[ridx[p]] = leaf for p in segment.  work[i] = (leaf_id, start, count, -)
__global__ __launch_bounds__(256) void fill_nid_kernel(const int* __restrict__ ridx, const int4* __restrict__ work,
                                                       int* __restrict__ nid) {
  const int4 wk = work[blockIdx.x];
  for (int p = wk.y + threadIdx.x; p < wk.y + wk.z; p += blockDim.x) nid[ridx[p]] = wk.x;
}

extern "C" {

int h2o_hist_build(const void* codes, int code_bytes, int Fp, const int* ridx, const float* va,
                   const float* vb, const int* work, int n_work, int F, int FG, int Bs, double* hist,
                   int n_slots, int mode, int threads, hipStream_t s) {
  if (n_work <= 0) return 0;
  if (code_bytes == 1)
    return launch_hist<uint8_t>(codes, Fp, ridx, va, vb, (const int4*)work, n_work, F, FG, Bs, hist, n_slots, mode, threads, s);
  return launch_hist<uint16_t>(codes, Fp, ridx, va, vb, (const int4*)work, n_work, F, FG, Bs, hist, n_slots, mode, threads, s);
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
                     const int* loff, const int* roff, int* out, hipStream_t s) {
  if (n_work <= 0) return 0;
  if (code_bytes == 1)
    hipLaunchKernelGGL(part_scatter_kernel<uint8_t>, dim3(n_work), dim3(256), 0, s, (const uint8_t*)codes, rs, fs, ridx, (const int4*)work, feat, masks, Bs, loff, roff, out);
  else
    hipLaunchKernelGGL(part_scatter_kernel<uint16_t>, dim3(n_work), dim3(256), 0, s, (const uint16_t*)codes, rs, fs, ridx, (const int4*)work, feat, masks, Bs, loff, roff, out);
  return (int)hipGetLastError();
}

int h2o_fill_nid(const int* ridx, const int* work, int n_work, int* nid, hipStream_t s) {
  if (n_work <= 0) return 0;
  hipLaunchKernelGGL(fill_nid_kernel, dim3(n_work), dim3(256), 0, s, ridx, (const int4*)work, nid);
  return (int)hipGetLastError();
}

}  // extern "C"
