// Partition-free GBM level histograms: microbenchmark (round-5 A/B).
//
// The production tree engine partitions row indices by node every level
// (part_flags / part_compact) and builds each node's histogram from its own
// contiguous row range.  The alternative measured here streams ALL rows every
// level with a per-row node id: a workgroup owns (row block, node group,
// feature group), keeps that group's g/h histograms in LDS, skips rows whose
// node is outside its group, and flushes with global atomics.  With the
// subtraction trick only the smaller child of each split is built
// (2^(d-1) nodes at depth d); after the level a kernel applies the splits to
// the node ids (the partition-free replacement of the row partition).
//
// Synthetic data of the bench's GBM shape: N rows x F = 100 uint8 codes
// (255 bins + NA), random node ids, g/h per row.  Prints ms per level
// (histograms + flush + node-id update) and the depth-8 tree total.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/pf_hist_mb scripts/pf_hist_mb.hip
//   scripts/pf_hist_mb 12500000
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

constexpr int F = 100;
constexpr int NBIN = 256;

// grid: (row blocks, node groups x feature groups); LDS [NG][FG][NBIN][2] f32
__global__ __launch_bounds__(256) void pf_hist_kernel(const unsigned char* __restrict__ codes,
                                                      const int* __restrict__ nid, const float* __restrict__ g,
                                                      const float* __restrict__ h, long long N, int NG, int FG,
                                                      int nfg, long long rows_per_block, float* __restrict__ hist) {
  extern __shared__ float sh[];
  const int grp = blockIdx.y;
  const int ng = grp / nfg, fgi = grp - ng * nfg;
  const int n0 = ng * NG, f0 = fgi * FG;
  const int fcnt = min(FG, F - f0);
  const int cells = NG * FG * NBIN * 2;
  for (int i = threadIdx.x; i < cells; i += 256) sh[i] = 0.f;
  __syncthreads();
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(N, r0 + rows_per_block);
  // a wave takes 64 consecutive rows; each lane one row, looping over the
  // group's features (LDS atomics, as the production kernels)
  for (long long r = r0 + threadIdx.x; r < r1; r += 256) {
    const int n = nid[r] - n0;
    if (n < 0 || n >= NG) continue;
    const float gv = g[r], hv = h[r];
    const unsigned char* c = codes + r * F + f0;
    float* base = sh + (size_t)n * FG * NBIN * 2;
    for (int f = 0; f < fcnt; ++f) {
      float* cell = base + ((size_t)f * NBIN + c[f]) * 2;
      __hip_atomic_fetch_add(cell, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(cell + 1, hv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < cells; i += 256) {
    const float v = sh[i];
    if (v == 0.f) continue;
    const int nn = i / (FG * NBIN * 2), rem = i - nn * FG * NBIN * 2;
    const int f = rem / (NBIN * 2), cb = rem - f * NBIN * 2;
    if (f >= fcnt) continue;
    float* dst = hist + (((size_t)(n0 + nn) * F + f0 + f) * NBIN * 2) + cb;
    __hip_atomic_fetch_add(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// split application: nid[r] -> child id from the node's split (feature, bin)
__global__ void pf_apply_kernel(const unsigned char* __restrict__ codes, int* __restrict__ nid,
                                const int* __restrict__ sf, const int* __restrict__ sb, long long N, int nodes) {
  for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < N; r += (long long)gridDim.x * 256) {
    const int n = nid[r];
    if (n < 0 || n >= nodes) continue;
    const int c = codes[r * F + sf[n]];
    nid[r] = 2 * n + (c > sb[n] ? 1 : 0);
  }
}

__global__ void pf_fill_nid(int* nid, long long N, int nodes, int built, unsigned seed) {
  for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < N; r += (long long)gridDim.x * 256) {
    unsigned x = (unsigned)r * 2654435761u ^ seed;
    x ^= x >> 15;
    x *= 2246822519u;
    x ^= x >> 13;
    const int node = (int)(x % (unsigned)nodes);
    // rows of non-built siblings get -1 (the subtraction trick skips them)
    nid[r] = node < built ? node : -1;
  }
}

int main(int argc, char** argv) {
  const long long N = argc > 1 ? atoll(argv[1]) : 12500000LL;
  const int depth = 8;
  unsigned char* codes;
  int* nid;
  float *g, *h, *hist;
  int *sf, *sb;
  CHECK(hipMalloc(&codes, N * F));
  CHECK(hipMalloc(&nid, N * 4));
  CHECK(hipMalloc(&g, N * 4));
  CHECK(hipMalloc(&h, N * 4));
  const size_t hist_bytes = (size_t)(1 << (depth - 1)) * F * NBIN * 2 * 4;
  CHECK(hipMalloc(&hist, hist_bytes));
  CHECK(hipMalloc(&sf, 4096 * 4));
  CHECK(hipMalloc(&sb, 4096 * 4));
  {
    std::vector<unsigned char> hc(N * F);
    unsigned s = 12345u;
    for (auto& v : hc) {
      s = s * 1664525u + 1013904223u;
      v = (unsigned char)(s >> 24);
    }
    CHECK(hipMemcpy(codes, hc.data(), N * F, hipMemcpyHostToDevice));
    std::vector<float> hv(N, 0.25f);
    CHECK(hipMemcpy(h, hv.data(), N * 4, hipMemcpyHostToDevice));
    for (long long i = 0; i < N; ++i) hv[i] = (i % 7) * 0.1f - 0.3f;
    CHECK(hipMemcpy(g, hv.data(), N * 4, hipMemcpyHostToDevice));
    std::vector<int> hs(4096), hb(4096);
    for (int i = 0; i < 4096; ++i) {
      hs[i] = (i * 37) % F;
      hb[i] = (i * 91) % 250;
    }
    CHECK(hipMemcpy(sf, hs.data(), 4096 * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(sb, hb.data(), 4096 * 4, hipMemcpyHostToDevice));
  }
  CHECK(hipFuncSetAttribute((const void*)pf_hist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  double total = 0.0;
  printf("{\"rows\": %lld, \"features\": %d, \"bins\": %d, \"levels\": [\n", N, F, NBIN);
  for (int d = 0; d < depth; ++d) {
    const int nodes = 1 << d;
    const int built = d == 0 ? 1 : nodes / 2;
    hipLaunchKernelGGL(pf_fill_nid, dim3(4096), dim3(256), 0, 0, nid, N, nodes, built, 777u + d);
    CHECK(hipGetLastError());
    // LDS budget 128 KB: NG nodes x FG features x 256 bins x (g, h) f32
    const int NG = built >= 4 ? 4 : built;
    const int FG = 64 / NG > F ? F : 64 / NG;
    const int nfg = (F + FG - 1) / FG;
    const int groups = ((built + NG - 1) / NG) * nfg;
    int rb = (2048 + groups - 1) / groups;
    if (rb < 1) rb = 1;
    const long long rpb = (N + rb - 1) / rb;
    const size_t lds = (size_t)NG * FG * NBIN * 2 * 4;
    float best = 1e30f;
    for (int it = 0; it < 4; ++it) {
      CHECK(hipMemsetAsync(hist, 0, (size_t)built * F * NBIN * 2 * 4, 0));
      CHECK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(pf_hist_kernel, dim3(rb, groups), dim3(256), lds, 0, codes, nid, g, h, N, NG, FG, nfg, rpb,
                         hist);
      CHECK(hipGetLastError());
      hipLaunchKernelGGL(pf_apply_kernel, dim3(4096), dim3(256), 0, 0, codes, nid, sf, sb, N, built);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
      // the apply kernel rewrote nid: restore this level's ids
      hipLaunchKernelGGL(pf_fill_nid, dim3(4096), dim3(256), 0, 0, nid, N, nodes, built, 777u + d);
    }
    total += best;
    printf("  {\"depth\": %d, \"nodes_built\": %d, \"node_group\": %d, \"feature_group\": %d, \"workgroups\": %d, "
           "\"ms\": %.3f}%s\n",
           d, built, NG, FG, rb * groups, best, d + 1 < depth ? "," : "");
    fflush(stdout);
  }
  printf("], \"tree_ms_depth8\": %.3f}\n", total);
  return 0;
}
