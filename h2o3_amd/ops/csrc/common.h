// Shared helpers for the h2o3_amd HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define H2O_WAVE 64

#define H2O_CHECK_LAUNCH() return (int)hipGetLastError()

__device__ __forceinline__ int lane_id() { return threadIdx.x & (H2O_WAVE - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x / H2O_WAVE; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, H2O_WAVE);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, H2O_WAVE);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, H2O_WAVE));
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, H2O_WAVE));
  return v;
}

// LDS float atomic add, no return -> ds_add_f32
__device__ __forceinline__ void lds_add(float* p, float v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Global float atomic add, no return -> global_atomic_add_f32 (agent scope)
__device__ __forceinline__ void gbl_add(float* p, float v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gbl_add(double* p, double v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// XCD-aware bijective remap of a 1-D block id (blocks sharing an XCD get a
// contiguous range of logical ids).  cdna_hip_programming.md §5 "XCD swizzle".
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nx = 8;
  if (nwg <= nx) return orig;
  int q = nwg / nx, r = nwg % nx;
  int xcd = orig % nx;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / nx;
}
