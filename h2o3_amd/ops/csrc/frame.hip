// Frame-level column kernels: batched rollups and the numeric model-matrix
// expansion.
//
// Reference: water/fvec/RollupStats.java (one MRTask per Vec computing min /
// max / mean / sigma / NA / zero / inf counts and the integer flag, run for
// every column of a frame before a model build) and hex/DataInfo.java (the
// standardized, NA-imputed numeric block of the model matrix).
//
// MI355X design.  A frame is a set of column tensors in HBM.  Rollups: ONE
// launch per pass covers every column (grid y = column, x = row slices);
// each thread keeps counts, sums, min / max and the integer flag in
// registers, a block reduces them and writes 10 doubles per (column, slice);
// torch sums the slices (and the ranks) on the device, the squared-deviation
// pass takes the exact means from there, and the host reads all columns in
// one copy.
// Expansion: the row-major [n, P] design matrix is written by 64 x 64 tiles
// transposed through LDS (coalesced column reads, coalesced 256-B row
// writes), NA imputation and standardization fused -- a per-column strided
// write of a 4000-B-pitch matrix touches one cache line per element.
#include "common.h"

struct FrCol {
  const void* p;
  int dtype;   // 0 f32, 1 f64
  int pad;
};

__device__ __forceinline__ double fr_load(const FrCol& c, long long i) {
  return c.dtype ? reinterpret_cast<const double*>(c.p)[i] : (double)reinterpret_cast<const float*>(c.p)[i];
}

// Two passes, like Vec.rollups (plain f64 sums, then the squared deviations
// from the exact mean -- large offsets keep their precision):
// pass 0: part[(col * gridDim.x + slice) * 10 + k] =
//   0 n finite, 1 sum, 2 -, 3 NaN, 4 zeros, 5 +inf, 6 -inf, 7 non-integer, 8 min, 9 max
// pass 1 (mean[col] given on the device): field 0 = sum of (x - mean)^2 over finite x
__global__ __launch_bounds__(256) void rollup_multi_kernel(const FrCol* __restrict__ cols, long long n,
                                                           const double* __restrict__ mean, int pass,
                                                           double* __restrict__ part) {
  const FrCol c = cols[blockIdx.y];
  double cnt = 0.0, s1 = 0.0;
  double nan = 0.0, zer = 0.0, pin = 0.0, nin = 0.0, nint = 0.0;
  double mn = 1.7976931348623157e308, mx = -1.7976931348623157e308;
  const double mu = pass ? mean[blockIdx.y] : 0.0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  auto acc = [&](double x) {
    if (x != x) { nan += 1.0; return; }
    if (isinf(x)) { if (x > 0) pin += 1.0; else nin += 1.0; return; }
    if (pass) {
      const double d = x - mu;
      s1 += d * d;
      return;
    }
    cnt += 1.0; s1 += x;
    zer += x == 0.0 ? 1.0 : 0.0;
    nint += x != rint(x) ? 1.0 : 0.0;
    mn = fmin(mn, x); mx = fmax(mx, x);
  };
  // 4 independent loads in flight per thread
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const double x0 = fr_load(c, i), x1 = fr_load(c, i + stride), x2 = fr_load(c, i + 2 * stride),
                 x3 = fr_load(c, i + 3 * stride);
    acc(x0); acc(x1); acc(x2); acc(x3);
  }
  for (; i < n; i += stride) acc(fr_load(c, i));
  __shared__ double red[256][10];
  double* r = red[threadIdx.x];
  r[0] = pass ? s1 : cnt; r[1] = s1; r[2] = 0.0; r[3] = nan; r[4] = zer; r[5] = pin; r[6] = nin; r[7] = nint;
  r[8] = mn; r[9] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      double* a = red[threadIdx.x];
      const double* b = red[threadIdx.x + o];
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += b[k];
      a[8] = fmin(a[8], b[8]);
      a[9] = fmax(a[9], b[9]);
    }
    __syncthreads();
  }
  if (threadIdx.x < 10) part[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 10 + threadIdx.x] = red[0][threadIdx.x];
}

// X[r, base + j] = ((isnan(x) ? plug[j] : x) - mean[j]) / sd[j] for the
// ncols numeric columns (j < ncols), in f64 then rounded to X's type (the
// same arithmetic as DataInfo.expand's torch path); 64 x 64 tiles via LDS.
template <typename OT>
__global__ __launch_bounds__(256) void expand_numeric_kernel(const FrCol* __restrict__ cols, int ncols, long long n,
                                                             const double* __restrict__ plug,
                                                             const double* __restrict__ mean,
                                                             const double* __restrict__ sd, OT* __restrict__ X,
                                                             int ldx, int base) {
  __shared__ OT tile[64][65];
  __shared__ FrCol ct[64];
  __shared__ double cp[3][64];
  const long long r0 = (long long)blockIdx.x * 64;
  const int j0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
  // the tile's column table and constants once per block (no dependent
  // table -> pointer -> data chain per element)
  if (threadIdx.x < 64) {
    const int j = j0 + threadIdx.x;
    ct[threadIdx.x] = j < ncols ? cols[j] : FrCol{nullptr, 0, 0};
    cp[0][threadIdx.x] = j < ncols ? plug[j] : 0.0;
    cp[1][threadIdx.x] = j < ncols ? mean[j] : 0.0;
    cp[2][threadIdx.x] = j < ncols ? sd[j] : 1.0;
  }
  __syncthreads();
  // read: thread (tx = row, ty + 4k = column), all 16 loads issued first
  const long long rr = r0 + tx;
  double xv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = ty + 4 * i;
    xv[i] = (j0 + k < ncols && rr < n) ? fr_load(ct[k], rr) : 0.0;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = ty + 4 * i;
    double x = xv[i];
    if (x != x) x = cp[0][k];
    tile[k][tx] = (OT)((x - cp[1][k]) / cp[2][k]);
  }
  __syncthreads();
  // write: thread (tx = column, ty + 4k = row)
  for (int k = ty; k < 64; k += 4) {
    const long long r = r0 + k;
    const int j = j0 + tx;
    if (j < ncols && r < n) X[(size_t)r * ldx + base + j] = tile[tx][k];
  }
}

extern "C" {

int h2o_rollup_multi(const void* cols, int ncols, long long n, int slices, const double* mean, int pass,
                     double* part, hipStream_t s) {
  if (ncols <= 0) return 0;
  if (slices <= 0 || ncols > 65535 || (pass && !mean)) return -1;
  hipLaunchKernelGGL(rollup_multi_kernel, dim3(slices, ncols), dim3(256), 0, s, (const FrCol*)cols, n, mean, pass,
                     part);
  return (int)hipGetLastError();
}

// out_dtype 0: float32 X, 1: float64 X
int h2o_expand_numeric(const void* cols, int ncols, long long n, const double* plug, const double* mean,
                       const double* sd, void* X, int ldx, int base, int out_dtype, hipStream_t s) {
  if (ncols <= 0 || n <= 0) return 0;
  if (base < 0 || base + ncols > ldx) return -1;
  const dim3 grid((unsigned)((n + 63) / 64), (unsigned)((ncols + 63) / 64));
  if (grid.y > 65535) return -2;
  if (out_dtype == 0)
    hipLaunchKernelGGL(expand_numeric_kernel<float>, grid, dim3(256), 0, s, (const FrCol*)cols, ncols, n, plug, mean,
                       sd, (float*)X, ldx, base);
  else
    hipLaunchKernelGGL(expand_numeric_kernel<double>, grid, dim3(256), 0, s, (const FrCol*)cols, ncols, n, plug,
                       mean, sd, (double*)X, ldx, base);
  return (int)hipGetLastError();
}

}  // extern "C"
