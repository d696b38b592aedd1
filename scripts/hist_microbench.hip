// Microbenchmark for the tree histogram kernel variants (one process,
// interleaved rounds, hipEvent timing).  Build: hipcc --offload-arch=gfx950 -O3
//   -o hist_mb scripts/hist_microbench.hip ; run: ./hist_mb
// Variants (all FGL features x RPW rows per wave instruction):
//   0 baseline f32 ds_add, stride Bs*C
//   1 padded stride (Bs*C + 1) to spread LDS banks across features
//   2 integer ds_add_u32 on fixed-point values
//   3 no flush (LDS only)          (timing only)
//   4 plain ds_write, no atomics   (timing only: upper bound)
//   5 lane=row mapping (old)       (timing reference)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int VAR>
__global__ __launch_bounds__(512) void hk(const unsigned char* __restrict__ codes, int Fp, const int* __restrict__ ridx,
                                          const float* __restrict__ va, const float* __restrict__ vb, int rows_per_block,
                                          int N, int F, int Bs, int FGL, double* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int C = 2;
  const int stride_f = (VAR == 1) ? Bs * C + 1 : (VAR == 6 ? Bs * C * 2 : Bs * C);
  const int fg0 = blockIdx.y * FGL;
  const int nf = min(FGL, F - fg0);
  for (int i = threadIdx.x; i < FGL * stride_f; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  const int p_begin = blockIdx.x * rows_per_block;
  const int pend = min(N, p_begin + rows_per_block);
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (VAR == 5) {
    for (int p = p_begin + threadIdx.x; p < pend; p += blockDim.x) {
      const int r = ridx[p];
      const float w = vb[r], y = va[r];
      const unsigned char* row = codes + (size_t)r * Fp + fg0;
      for (int j = 0; j < nf; ++j) {
        float* h = lds + j * stride_f + row[j] * C;
        __hip_atomic_fetch_add(h, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(h + 1, w * y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  } else {
    const int RPW = 64 / FGL;
    const int fl = lane % FGL, rs = lane / FGL;
    const bool lane_ok = rs < RPW;
    const bool fok = fl < nf && lane_ok;
    const int fcl = min(fl, nf - 1);
    const unsigned char* cbase = codes + fg0 + fcl;
    float* hbase = lds + fl * stride_f;
    const int step = nw * RPW;
    constexpr int U = 8;
    for (int p0 = p_begin + wv * RPW + (lane_ok ? rs : 0); p0 < pend; p0 += U * step) {
      int rr[U]; float c0[U], c1[U]; int code[U];
#pragma unroll
      for (int u = 0; u < U; ++u) rr[u] = ridx[min(p0 + u * step, pend - 1)];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = rr[u];
        const float y = va[r], w = vb[r];
        c0[u] = w; c1[u] = w * y;
        code[u] = cbase[(size_t)r * Fp];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = fok && (p0 + u * step < pend);
        if (ok) {
          float* h = hbase + code[u] * C * (VAR == 6 ? 2 : 1);
          if (VAR == 6) {
            unsigned long long* hi = (unsigned long long*)h;
            __hip_atomic_fetch_add(hi, (unsigned long long)(long long)(c0[u] * 1099511627776.f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(hi + 1, (unsigned long long)(long long)(c1[u] * 1099511627776.f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else if (VAR == 2) {
            unsigned* hi = (unsigned*)h;
            __hip_atomic_fetch_add(hi, (unsigned)(int)(c0[u] * 1024.f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(hi + 1, (unsigned)(int)(c1[u] * 1024.f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else if (VAR == 4) {
            h[0] = c0[u]; h[1] = c1[u];
          } else {
            __hip_atomic_fetch_add(h, c0[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(h + 1, c1[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
    }
  }
  __syncthreads();
  if (VAR == 3) { if (threadIdx.x == 0 && lds[0] == 12345.f) hist[0] = 1; return; }
  for (int i = threadIdx.x; i < nf * Bs * C; i += blockDim.x) {
    const int j = i / (Bs * C), rem = i - j * Bs * C;
    const float v = lds[j * stride_f + rem];
    if (v != 0.f) __hip_atomic_fetch_add(hist + (size_t)(fg0 + j) * Bs * C + rem, (double)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int VAR>
float run(const unsigned char* codes, int Fp, const int* ridx, const float* va, const float* vb, int N, int F, int Bs,
          int FGL, double* hist, int nblk_rows, int threads) {
  int rpb = (N + nblk_rows - 1) / nblk_rows;
  dim3 grid(nblk_rows, (F + FGL - 1) / FGL);
  int stride = (VAR == 1) ? Bs * 2 + 1 : (VAR == 6 ? Bs * 4 : Bs * 2);
  size_t lds = (size_t)FGL * stride * 4;
  if (VAR == 5) lds = (size_t)FGL * Bs * 2 * 4;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(hk<VAR>, grid, dim3(threads), lds, 0, codes, Fp, ridx, va, vb, rpb, N, F, Bs, FGL, hist);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  return ms;
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 10000000;
  const int F = 100, Fp = 112, Bs = 256;
  std::vector<unsigned char> hc((size_t)N * Fp);
  srand(1);
  for (size_t i = 0; i < hc.size(); ++i) hc[i] = rand() % 255;
  std::vector<int> hr(N);
  for (int i = 0; i < N; ++i) hr[i] = i;
  std::vector<float> hv(N, 0.5f), hw(N, 1.0f);
  unsigned char* dc; int* dr; float *dv, *dw; double* dh;
  CK(hipMalloc(&dc, hc.size())); CK(hipMalloc(&dr, N * 4)); CK(hipMalloc(&dv, N * 4)); CK(hipMalloc(&dw, N * 4));
  CK(hipMalloc(&dh, (size_t)F * Bs * 2 * 8));
  CK(hipMemcpy(dc, hc.data(), hc.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dr, hr.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dv, hv.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, hw.data(), N * 4, hipMemcpyHostToDevice));
  const int fgls[] = {20, 32, 64};
  const int nblks[] = {256, 1024};
  printf("N=%d F=%d Bs=%d  (ms; min over 5 interleaved rounds)\n", N, F, Bs);
  for (int fgl : fgls) for (int nb : nblks) {
    float best[7] = {1e9, 1e9, 1e9, 1e9, 1e9, 1e9, 1e9};
    for (int round = 0; round < 5; ++round) {
      best[0] = std::min(best[0], run<0>(dc, Fp, dr, dv, dw, N, F, Bs, fgl, dh, nb, 512));
      best[1] = std::min(best[1], run<1>(dc, Fp, dr, dv, dw, N, F, Bs, fgl, dh, nb, 512));
      best[2] = std::min(best[2], run<2>(dc, Fp, dr, dv, dw, N, F, Bs, fgl, dh, nb, 512));
      best[3] = std::min(best[3], run<3>(dc, Fp, dr, dv, dw, N, F, Bs, fgl, dh, nb, 512));
      best[4] = std::min(best[4], run<4>(dc, Fp, dr, dv, dw, N, F, Bs, fgl, dh, nb, 512));
      if (fgl <= 32) best[6] = std::min(best[6], run<6>(dc, Fp, dr, dv, dw, N, F, Bs, fgl, dh, nb, 512));
      if (fgl == 20) best[5] = std::min(best[5], run<5>(dc, Fp, dr, dv, dw, N, F, Bs, fgl, dh, nb, 512));
    }
    printf("FGL=%2d blocks_rows=%4d  base %.3f  padded %.3f  int %.3f  noflush %.3f  nowrite %.3f  lane=row %.3f  u64 %.3f\n", fgl, nb,
           best[0], best[1], best[2], best[3], best[4], fgl == 20 ? best[5] : -1.f, best[6]);
  }
  return 0;
}
