// Aggregation kernels for metrics and group-bys.
//
// Binomial metric sketch: the merged logit histogram behind AUC / PR-AUC /
// the threshold table / gains-lift, plus the weighted sums behind logloss,
// MSE and the response mean, in ONE pass over the scored rows.
//
// Reference: hex/AUC2.java (AUCBuilder: per-chunk score bins merged in
// MRTask.reduce) and hex/ModelMetricsBinomial.java (MetricBuilderBinomial:
// per-row logloss / squared error accumulation).
//
// MI355X design.  The sketch has 2 x 2^18 f64 bins in HBM (4 MB, far past
// LDS), so rows go straight to global f64 atomics.  Early in a boosting run
// (and for any model with few leaves) the scores take a handful of distinct
// values, so millions of rows hit the SAME few bins and plain per-row
// atomics serialise on those addresses.  Each wave therefore aggregates
// before it issues an atomic: the lowest pending lane's bin is broadcast,
// every lane holding that bin joins one wave sum, one lane adds it, and the
// loop repeats over the distinct bins of the wave (at most 64 rounds, one
// when the scores are constant).  The row filter (NaN score or response) is
// fused, so the caller never compacts the arrays.
#include "common.h"

#define MH_LIM 40.0

__device__ __forceinline__ int mh_bin(double p, int nb) {
  double x = log(fmax(p, 1e-300)) - log1p(-fmin(p, 1.0 - 1e-16));
  x = fmin(fmax(x, -MH_LIM), MH_LIM);
  long long b = (long long)((x + MH_LIM) * ((double)nb / (2.0 * MH_LIM)));
  return (int)(b < 0 ? 0 : (b > nb - 1 ? nb - 1 : b));
}

// H[2 * nb]: positives' weights in [0, nb), negatives' in [nb, 2 nb).
// sums[5]: sum w, sum w * logloss, sum w * (y - p)^2, sum w * y, row count.
__global__ __launch_bounds__(256) void logit_hist_kernel(const double* __restrict__ p, const double* __restrict__ y,
                                                         const double* __restrict__ w, long long n, int nb,
                                                         double* __restrict__ H, double* __restrict__ sums) {
  const int lane = lane_id();
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  // the loop bound is uniform over the block, so every lane takes part in
  // the ballots below
  for (long long base = (long long)blockIdx.x * blockDim.x; base < n; base += stride) {
    const long long i = base + threadIdx.x;
    bool v = false;
    int key = 0;
    double wi = 0.0;
    if (i < n) {
      const double pi = p[i], yi = y[i];
      if (!isnan(pi) && !isnan(yi)) {
        v = true;
        wi = w ? w[i] : 1.0;
        const double pc = fmin(fmax(pi, 1e-15), 1.0 - 1e-15);
        s0 += wi;
        s1 -= wi * (yi * log(pc) + (1.0 - yi) * log(1.0 - pc));
        s2 += wi * (yi - pi) * (yi - pi);
        s3 += wi * yi;
        s4 += 1.0;
        key = mh_bin(pi, nb) + nb * (int)(1.0 - yi);
      }
    }
    unsigned long long act = __ballot(v);
    while (act) {
      const int leader = __ffsll((long long)act) - 1;
      const int lk = __shfl(key, leader, H2O_WAVE);
      const bool m = v && key == lk;
      const unsigned long long mm = __ballot(m);
      const double c = wave_sum(m ? wi : 0.0);
      if (lane == leader) gbl_add(&H[lk], c);
      if (m) v = false;
      act &= ~mm;
    }
  }
  __shared__ double red[5][4];
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  s3 = wave_sum(s3);
  s4 = wave_sum(s4);
  const int wv = wave_id();
  if (lane == 0) {
    red[0][wv] = s0;
    red[1][wv] = s1;
    red[2][wv] = s2;
    red[3][wv] = s3;
    red[4][wv] = s4;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    const double t = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
    gbl_add(&sums[threadIdx.x], t);
  }
}

// Grouped sums / minima / maxima out[g, c] (+)= v[i, c] over rows i with
// idx[i] == g (rows with idx outside [0, nbins) are skipped): the group-by / class-count / leaf-sum
// primitive (water/rapids/ast/prims/mungers/AstGroup.java's per-group
// accumulators, hex/ModelMetrics* class tallies).  The same contention
// problem as the sketch above: few groups, millions of rows.  Each wave
// first merges lanes that share a group (up to PEEL rounds, which covers the
// few-group case completely), then lanes still pending add directly.  With
// nbins * C <= LDS_MAX the block accumulates in LDS (ds_add_f64) and flushes
// once; otherwise the atomics go to global memory (global_atomic_add_f64,
// global_atomic_min_f64 / max_f64).
#define GS_LDS_MAX 8192
#define GS_PEEL 8

// OP 0: sum, 1: min, 2: max (the caller fills out with 0 / +inf / -inf).
template <int OP>
__device__ __forceinline__ double gs_ident() {
  return OP == 0 ? 0.0 : (OP == 1 ? __builtin_inf() : -__builtin_inf());
}
template <int OP>
__device__ __forceinline__ double gs_comb(double a, double b) {
  return OP == 0 ? a + b : (OP == 1 ? fmin(a, b) : fmax(a, b));
}
template <int OP>
__device__ __forceinline__ double gs_wave(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = gs_comb<OP>(v, __shfl_xor(v, o, H2O_WAVE));
  return v;
}
template <int OP, bool LDS>
__device__ __forceinline__ void gs_atomic(double* p, double v) {
  constexpr int scope = LDS ? __HIP_MEMORY_SCOPE_WORKGROUP : __HIP_MEMORY_SCOPE_AGENT;
  if (OP == 0)
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, scope);
  else if (OP == 1)
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, scope);
  else
    __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, scope);
}

template <int OP, bool LDS>
__global__ __launch_bounds__(256) void group_reduce_kernel(const long long* __restrict__ idx,
                                                           const double* __restrict__ v, long long n, int C,
                                                           int nbins, double* __restrict__ out) {
  __shared__ double acc[LDS ? GS_LDS_MAX : 1];
  const int lane = lane_id();
  const int tot = nbins * C;
  if (LDS) {
    for (int j = threadIdx.x; j < tot; j += blockDim.x) acc[j] = gs_ident<OP>();
    __syncthreads();
  }
  double* dst = LDS ? acc : out;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long base = (long long)blockIdx.x * blockDim.x; base < n; base += stride) {
    const long long i = base + threadIdx.x;
    long long g = i < n ? idx[i] : -1;
    bool pend = g >= 0 && g < nbins;
    const int key = pend ? (int)g : -1;
    unsigned long long act = __ballot(pend);
    for (int r = 0; r < GS_PEEL && act; ++r) {
      const int leader = __ffsll((long long)act) - 1;
      const int lk = __shfl(key, leader, H2O_WAVE);
      const bool m = pend && key == lk;
      const unsigned long long mm = __ballot(m);
      if (__popcll(mm) == 1) {
        // a singleton group: no merge to gain, the lane adds on its own
        if (m)
          for (int c = 0; c < C; ++c) gs_atomic<OP, LDS>(&dst[(size_t)lk * C + c], v[(size_t)i * C + c]);
      } else {
        for (int c = 0; c < C; ++c) {
          const double t = gs_wave<OP>(m ? v[(size_t)i * C + c] : gs_ident<OP>());
          if (lane == leader) gs_atomic<OP, LDS>(&dst[(size_t)lk * C + c], t);
        }
      }
      if (m) pend = false;
      act &= ~mm;
    }
    if (pend)
      for (int c = 0; c < C; ++c) gs_atomic<OP, LDS>(&dst[(size_t)key * C + c], v[(size_t)i * C + c]);
  }
  if (LDS) {
    __syncthreads();
    for (int j = threadIdx.x; j < tot; j += blockDim.x)
      if (acc[j] != gs_ident<OP>()) gs_atomic<OP, false>(&out[j], acc[j]);
  }
}

template <int OP>
static int gs_launch(const long long* idx, const double* v, long long n, int C, int nbins, double* out,
                     hipStream_t s) {
  const bool lds = (long long)nbins * C <= GS_LDS_MAX;
  long long blocks = (n + 255) / 256;
  // LDS mode flushes nbins * C atomics per block: fewer, fuller blocks
  const long long cap = lds ? 1024 : 4096;
  if (blocks > cap) blocks = cap;
  if (lds)
    hipLaunchKernelGGL((group_reduce_kernel<OP, true>), dim3((unsigned)blocks), dim3(256), 0, s, idx, v, n, C, nbins,
                       out);
  else
    hipLaunchKernelGGL((group_reduce_kernel<OP, false>), dim3((unsigned)blocks), dim3(256), 0, s, idx, v, n, C,
                       nbins, out);
  return (int)hipGetLastError();
}

extern "C" {

// p, y: f64 [n]; w: f64 [n] or null (unit weights); H: f64 [2 nb] and
// sums: f64 [5], both zeroed by the caller (they accumulate).
int h2o_logit_hist(const double* p, const double* y, const double* w, long long n, int nb, double* H, double* sums,
                   hipStream_t s) {
  if (n <= 0) return 0;
  if (nb <= 0) return -1;
  long long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;   // 16 waves per CU on 256 CUs, grid-stride past that
  hipLaunchKernelGGL(logit_hist_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, y, w, n, nb, H, sums);
  return (int)hipGetLastError();
}

// idx: i64 [n]; v: f64 [n, C] row-major; out: f64 [nbins, C], filled by the
// caller with the op's identity (0 / +inf / -inf): it accumulates.
// op 0 sum, 1 min, 2 max.
int h2o_group_reduce(const long long* idx, const double* v, long long n, int C, int nbins, int op, double* out,
                     hipStream_t s) {
  if (n <= 0 || C <= 0 || nbins <= 0) return 0;
  if ((long long)nbins * C > 0x7fffffffLL) return -1;
  if (op == 0) return gs_launch<0>(idx, v, n, C, nbins, out, s);
  if (op == 1) return gs_launch<1>(idx, v, n, C, nbins, out, s);
  if (op == 2) return gs_launch<2>(idx, v, n, C, nbins, out, s);
  return -2;
}

}  // extern "C"
