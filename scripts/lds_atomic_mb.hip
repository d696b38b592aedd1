// LDS atomic throughput microbenchmark (no global loads in the loop): what is
// the per-CU ceiling of returnless ds_add for the histogram formulations?
//   ADDR 0: random bin in a 256-bin region per feature lane group ([f][bin] layout)
//   ADDR 1: conflict-free (lane-private address)
//   ADDR 2: all 64 lanes same address
// TYPE 0: u64 add, 1: u32 add, 2: f32 add, 3: two u32 adds to one 64-bit entry
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_mb scripts/lds_atomic_mb.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int TYPE, int ADDR>
__global__ __launch_bounds__(512) void k(int iters, unsigned seed, unsigned long long* out) {
  __shared__ __attribute__((aligned(16))) unsigned long long lds[16 * 257];
  for (int i = threadIdx.x; i < 16 * 257; i += blockDim.x) lds[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  unsigned x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
  const int f = lane & 15;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      x = x * 1664525u + 1013904223u;
      int a;
      if (ADDR == 0) a = f * 257 + ((x >> 13) & 255);
      else if (ADDR == 1) a = (threadIdx.x & 511) * 8 + (u & 7);   // distinct per lane
      else a = 5;
      a = a % (16 * 257);
      if (TYPE == 0) {
        __hip_atomic_fetch_add(&lds[a], (unsigned long long)(x | 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (TYPE == 1) {
        unsigned* l32 = reinterpret_cast<unsigned*>(lds);
        __hip_atomic_fetch_add(&l32[a], (x | 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (TYPE == 2) {
        float* lf = reinterpret_cast<float*>(lds);
        __hip_atomic_fetch_add(&lf[a], (float)(x & 7), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        unsigned* l32 = reinterpret_cast<unsigned*>(lds);
        __hip_atomic_fetch_add(&l32[2 * (a / 2)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&l32[2 * (a / 2) + 1], (x | 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  __syncthreads();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < 16 * 257; i += blockDim.x) s += lds[i];
  if (s == 0x123456789ull) out[0] = s;   // keep the work alive
}

template <int TYPE, int ADDR>
static void run(const char* name, int blocks, int iters, unsigned long long* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipLaunchKernelGGL((k<TYPE, ADDR>), dim3(blocks), dim3(512), 0, 0, iters, 7u, out);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<TYPE, ADDR>), dim3(blocks), dim3(512), 0, 0, iters, 7u + r, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  ms /= 5;
  const double ops = (double)blocks * 512 * iters * 8 * (TYPE == 3 ? 2 : 1);
  const double per_cu_clk = ops / (ms * 1e-3) / 256 / 2.4e9;
  printf("%-28s %8.3f ms  %7.1f G lane-atomics/s  %5.2f per CU-clock(2.4GHz)\n", name, ms, ops / ms / 1e6, per_cu_clk);
}

int main() {
  unsigned long long* out;
  CK(hipMalloc(&out, 8));
  const int blocks = 256 * 4, iters = 2000;
  run<0, 0>("u64 random-bin", blocks, iters, out);
  run<0, 1>("u64 conflict-free", blocks, iters, out);
  run<0, 2>("u64 same-address", blocks, iters, out);
  run<1, 0>("u32 random-bin", blocks, iters, out);
  run<1, 1>("u32 conflict-free", blocks, iters, out);
  run<2, 0>("f32 random-bin", blocks, iters, out);
  run<2, 1>("f32 conflict-free", blocks, iters, out);
  run<3, 0>("2x u32 random-bin", blocks, iters, out);
  return 0;
}
