// Fused best-split search over node histograms.
//
// Reference: hex/tree/DTree.java:findBestSplitPoint (DTree.java:984) — for
// every (node, column) it builds cumulative w/wY/wYY arrays from the low and
// high ends, tries every bin boundary with NAs sent left, right, or split off
// alone (NAvsREST), and keeps the best squared-error reduction subject to
// min_rows / min_split_improvement / monotone constraints.
//
// MI355X design: one wave64 per (node, feature).  The histogram row
// [Bs bins][2 channels] f64 streams through the wave in 64-bin chunks; an
// in-register shuffle scan gives each lane its cumulative left statistics,
// every lane scores its own threshold for the three NA placements, and a
// wave arg-max produces one candidate record per (node, feature).  This
// replaces ~20 PyTorch kernels over an [n, F, Bs, C] f64 tensor with one
// launch that reads the histogram exactly once.
//
// Criteria: CRIT 0 = H2O squared error on (w, wy) channels + node wYY total;
//           CRIT 1 = second-order gain on (g, h) (XGBoost).
#include "common.h"

struct SplitRec {
  double gain;
  double lw;   // left channel 0
  double ly;   // left channel 1
  int t;       // threshold bin (left = bins <= t)
  int opt;     // 0: NA right, 1: NA left, 2: NA vs rest
};

__device__ __forceinline__ double shfl_up_d(double v, int d) {
  return __shfl_up(v, d, 64);
}

template <int CRIT>
__device__ __forceinline__ double score(double a, double b, double lam, double alpha) {
  if (CRIT == 1) {
    double g = a;
    if (alpha > 0) g = copysign(fmax(fabs(g) - alpha, 0.0), g);
    return g * g / (b + lam);
  }
  return a > 0 ? b * b / a : 0.0;
}

template <int CRIT>
__device__ __forceinline__ bool valid_split(double lw, double ly, double rw, double ry, double min_rows, double lam,
                                            double mono) {
  double pl, pr;
  if (CRIT == 1) {
    const double mcw = fmax(min_rows, 1e-12);
    if (!(ly >= mcw && ry >= mcw)) return false;
    pl = -lw / (ly + lam);
    pr = -rw / (ry + lam);
  } else {
    if (!(lw >= min_rows && rw >= min_rows && lw > 0 && rw > 0)) return false;
    pl = ly / lw;
    pr = ry / rw;
    if ((float)pl == (float)pr) return false;
  }
  if (mono > 0 && pl > pr) return false;
  if (mono < 0 && pl < pr) return false;
  return true;
}

// H: [Fl][n][Bs][2] f64 (local feature slice).  grid: ceil(n*Fl/4) blocks of 256.
template <int CRIT>
__global__ __launch_bounds__(256) void split_kernel(const double* __restrict__ H, int Fl, int n, int Bs,
                                                    const double* __restrict__ node_wyy,
                                                    const unsigned char* __restrict__ feat_ok,  // [n][Fl]
                                                    const float* __restrict__ mono,            // [Fl]
                                                    double min_rows, double msi, double lam, double alpha,
                                                    double gamma, SplitRec* __restrict__ out,
                                                    const double* __restrict__ bnd, int use_bounds) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gw >= n * Fl) return;
  const int node = gw / Fl;
  const int f = gw - node * Fl;
  const int lane = threadIdx.x & 63;
  SplitRec best;
  best.gain = -INFINITY; best.t = 0; best.opt = 0; best.lw = 0; best.ly = 0;
  if (!feat_ok[(size_t)node * Fl + f]) {
    if (lane == 0) out[(size_t)node * Fl + f] = best;
    return;
  }
  const double* h = H + ((size_t)f * n + node) * (size_t)Bs * 2;
  const int B = Bs - 1;  // non-NA bins; NA bin = B
  // pass 1: non-NA totals
  double tw = 0, ty = 0;
  for (int b = lane; b < B; b += 64) { tw += h[2 * b]; ty += h[2 * b + 1]; }
  tw = wave_sum(tw);
  ty = wave_sum(ty);
  const double nw = h[2 * B], ny = h[2 * B + 1];
  const double Tw = tw + nw, Ty = ty + ny;
  const double sT = score<CRIT>(Tw, Ty, lam, alpha);
  const bool has_na = CRIT == 1 ? (ny > 0 || nw != 0) : (nw > 0);
  double se_before = 0;
  if (CRIT == 0) {
    se_before = fmax(node_wyy[node] - sT, 0.0);
    if (!(se_before > 0)) {
      if (lane == 0) out[(size_t)node * Fl + f] = best;
      return;
    }
  }
  const double mo = mono ? (double)mono[f] : 0.0;
  double carry_w = 0, carry_y = 0;
  for (int c0 = 0; c0 < B; c0 += 64) {
    const int b = c0 + lane;
    double vw = b < B ? h[2 * b] : 0.0, vy = b < B ? h[2 * b + 1] : 0.0;
    // inclusive wave scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const double uw = shfl_up_d(vw, d), uy = shfl_up_d(vy, d);
      if (lane >= d) { vw += uw; vy += uy; }
    }
    const double lw = carry_w + vw, ly = carry_y + vy;
    carry_w += __shfl(vw, 63, 64);
    carry_y += __shfl(vy, 63, 64);
    if (b <= B - 2) {
      const double rw = tw - lw, ry = ty - ly;
      // opt 0: NA right
      {
        const double RW = rw + nw, RY = ry + ny;
        if (valid_split<CRIT>(lw, ly, RW, RY, min_rows, lam, mo)) {
          double g = score<CRIT>(lw, ly, lam, alpha) + score<CRIT>(RW, RY, lam, alpha) - sT;
          if (CRIT == 1) g = 0.5 * g - gamma;
          if (g > best.gain) { best.gain = g; best.t = b; best.opt = 0; best.lw = lw; best.ly = ly; }
        }
      }
      if (has_na) {  // opt 1: NA left
        const double LW = lw + nw, LY = ly + ny;
        if (valid_split<CRIT>(LW, LY, rw, ry, min_rows, lam, mo)) {
          double g = score<CRIT>(LW, LY, lam, alpha) + score<CRIT>(rw, ry, lam, alpha) - sT;
          if (CRIT == 1) g = 0.5 * g - gamma;
          if (g > best.gain) { best.gain = g; best.t = b; best.opt = 1; best.lw = LW; best.ly = LY; }
        }
      }
    }
  }
  // opt 2: NA vs rest (lane 0 only; ties resolved in favour of lower bins)
  if (lane == 0 && has_na && valid_split<CRIT>(tw, ty, nw, ny, min_rows, lam, mo)) {
    double g = score<CRIT>(tw, ty, lam, alpha) + score<CRIT>(nw, ny, lam, alpha) - sT;
    if (CRIT == 1) g = 0.5 * g - gamma;
    if (g > best.gain) { best.gain = g; best.t = 0; best.opt = 2; best.lw = tw; best.ly = ty; }
  }
  // threshold: minimum improvement
  if (CRIT == 0) {
    if (!(best.gain > se_before * msi)) best.gain = -INFINITY;
  } else {
    if (!(best.gain > 0)) best.gain = -INFINITY;
  }
  // wave arg-max (prefer larger gain, then lower opt-major order like the reference scan)
  for (int o = 32; o > 0; o >>= 1) {
    const double og = __shfl_xor(best.gain, o, 64);
    const int ot = __shfl_xor(best.t, o, 64);
    const int oo = __shfl_xor(best.opt, o, 64);
    const double ow = __shfl_xor(best.lw, o, 64);
    const double oy = __shfl_xor(best.ly, o, 64);
    const int mykey = best.opt * 65536 + best.t, okey = oo * 65536 + ot;
    if (og > best.gain || (og == best.gain && okey < mykey)) {
      best.gain = og; best.t = ot; best.opt = oo; best.lw = ow; best.ly = oy;
    }
  }
  // node prediction bounds of monotone constraints (Constraints.java; applied
  // to this column's best split as DTree.java:1386-1445 does): a child
  // prediction outside [lo, hi] either vetoes the split (use_bounds == 0) or
  // is clamped, and the gain loses what the clamped constant costs
  // (w (c - mean)^2 for squared error, (h + lambda) (c - c*)^2 / 2 second order)
  if (bnd && lane == 0 && best.gain > -INFINITY) {
    const double lo = bnd[2 * node], hi = bnd[2 * node + 1];
    if (lo > -INFINITY || hi < INFINITY) {
      const double lw = best.lw, ly = best.ly, rw = Tw - lw, ry = Ty - ly;
      double pl, pr, al, ar;
      if (CRIT == 1) { al = ly + lam; ar = ry + lam; pl = -lw / al; pr = -rw / ar; al *= 0.5; ar *= 0.5; }
      else { al = lw; ar = rw; pl = ly / lw; pr = ry / rw; }
      const double cl = fmin(fmax(pl, lo), hi), cr = fmin(fmax(pr, lo), hi);
      if (cl != pl || cr != pr) {
        if (!use_bounds) best.gain = -INFINITY;
        else best.gain -= al * (cl - pl) * (cl - pl) + ar * (cr - pr) * (cr - pr);
      }
    }
  }
  if (lane == 0) out[(size_t)node * Fl + f] = best;
}

extern "C" int h2o_split_find_b(const double* H, int Fl, int n, int Bs, const double* node_wyy,
                                const unsigned char* feat_ok, const float* mono, double min_rows, double msi,
                                double lam, double alpha, double gamma, int crit, void* out, const double* bnd,
                                int use_bounds, hipStream_t s);

extern "C" int h2o_split_find(const double* H, int Fl, int n, int Bs, const double* node_wyy,
                              const unsigned char* feat_ok, const float* mono, double min_rows, double msi,
                              double lam, double alpha, double gamma, int crit, void* out, hipStream_t s) {
  return h2o_split_find_b(H, Fl, n, Bs, node_wyy, feat_ok, mono, min_rows, msi, lam, alpha, gamma, crit, out,
                          nullptr, 0, s);
}

// bnd: [n][2] node prediction bounds (lo, hi; +-inf = none) or nullptr
extern "C" int h2o_split_find_b(const double* H, int Fl, int n, int Bs, const double* node_wyy,
                                const unsigned char* feat_ok, const float* mono, double min_rows, double msi,
                                double lam, double alpha, double gamma, int crit, void* out, const double* bnd,
                                int use_bounds, hipStream_t s) {
  if (n <= 0 || Fl <= 0) return 0;
  const int waves = n * Fl;
  dim3 grid((waves + 3) / 4);
  if (crit == 1)
    hipLaunchKernelGGL(split_kernel<1>, grid, dim3(256), 0, s, H, Fl, n, Bs, node_wyy, feat_ok, mono, min_rows, msi,
                       lam, alpha, gamma, (SplitRec*)out, bnd, use_bounds);
  else
    hipLaunchKernelGGL(split_kernel<0>, grid, dim3(256), 0, s, H, Fl, n, Bs, node_wyy, feat_ok, mono, min_rows, msi,
                       lam, alpha, gamma, (SplitRec*)out, bnd, use_bounds);
  return (int)hipGetLastError();
}

// Per-node winner selection over the feature records of split_kernel and
// the go-left code mask, so the host reads ONE packed [n, 10] record per level:
//   pk[node] = {gain, feat(global), t, opt, L0, L1, R0, R1, T0, T1}
// T = node totals from feature 0's histogram (H[0][node][:][c]); ties keep
// the lowest feature (deterministic, matches torch max()).
__global__ __launch_bounds__(64) void split_select_kernel(const SplitRec* __restrict__ rec, const double* __restrict__ H,
                                                          int Fl, int n, int Bs, int f0, double* __restrict__ pk,
                                                          uint8_t* __restrict__ mask) {
  const int node = blockIdx.x;
  const int lane = threadIdx.x;
  double best = -INFINITY;
  int bf = 0;
  for (int f = lane; f < Fl; f += 64) {
    const double g = rec[(size_t)node * Fl + f].gain;
    if (g > best) { best = g; bf = f; }
  }
  // wave arg-max (lowest feature on ties)
  for (int o = 32; o > 0; o >>= 1) {
    const double og = __shfl_xor(best, o, 64);
    const int of = __shfl_xor(bf, o, 64);
    if (og > best || (og == best && of < bf)) { best = og; bf = of; }
  }
  double t0 = 0.0, t1 = 0.0;
  for (int b = lane; b < Bs; b += 64) {
    const double* h = H + ((size_t)node * Bs + b) * 2;   // feature 0
    t0 += h[0];
    t1 += h[1];
  }
  t0 = wave_sum(t0);
  t1 = wave_sum(t1);
  const SplitRec r = rec[(size_t)node * Fl + bf];
  if (lane == 0) {
    double* o = pk + (size_t)node * 10;
    o[0] = best; o[1] = (double)(bf + f0); o[2] = (double)r.t; o[3] = (double)r.opt;
    o[4] = r.lw; o[5] = r.ly; o[6] = t0 - r.lw; o[7] = t1 - r.ly; o[8] = t0; o[9] = t1;
  }
  const int B = Bs - 1;
  for (int c = lane; c < Bs; c += 64) {
    bool left;
    if (c == Bs - 1) left = r.opt == 1;
    else if (r.opt == 2) left = c < B;
    else left = c <= r.t;
    mask[(size_t)node * Bs + c] = left ? 1 : 0;
  }
}

extern "C" int h2o_split_select(const void* rec, const double* H, int Fl, int n, int Bs, int f0, double* pk,
                                uint8_t* mask, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(split_select_kernel, dim3(n), dim3(64), 0, s, (const SplitRec*)rec, H, Fl, n, Bs, f0, pk, mask);
  return (int)hipGetLastError();
}

// split_select_kernel + the split decision of the level, so the host never has
// to look at the record before the partition runs: ok = finite gain and (SE
// criterion) node weight >= min_w2 = 2*min_rows (min_w2 < 0 disables the test).
// Nodes that do not split get feature 0 and an all-ones mask (every row stays
// left = in place).  pk rows are `stride` doubles: the 10 fields of
// split_select_kernel, then ok; the partition fills field 11 (left count).
__global__ __launch_bounds__(64) void split_select2_kernel(const SplitRec* __restrict__ rec,
                                                           const double* __restrict__ H, int Fl, int n, int Bs,
                                                           int f0, double min_w2, int stride,
                                                           double* __restrict__ pk, uint8_t* __restrict__ mask,
                                                           int* __restrict__ feat_out) {
  const int node = blockIdx.x;
  const int lane = threadIdx.x;
  double best = -INFINITY;
  int bf = 0;
  for (int f = lane; f < Fl; f += 64) {
    const double g = rec[(size_t)node * Fl + f].gain;
    if (g > best) { best = g; bf = f; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const double og = __shfl_xor(best, o, 64);
    const int of = __shfl_xor(bf, o, 64);
    if (og > best || (og == best && of < bf)) { best = og; bf = of; }
  }
  double t0 = 0.0, t1 = 0.0;
  for (int b = lane; b < Bs; b += 64) {
    const double* h = H + ((size_t)node * Bs + b) * 2;   // feature 0
    t0 += h[0];
    t1 += h[1];
  }
  t0 = wave_sum(t0);
  t1 = wave_sum(t1);
  const SplitRec r = rec[(size_t)node * Fl + bf];
  const bool ok = isfinite(best) && (min_w2 < 0.0 || t0 >= min_w2);
  if (lane == 0) {
    double* o = pk + (size_t)node * stride;
    o[0] = best; o[1] = (double)(bf + f0); o[2] = (double)r.t; o[3] = (double)r.opt;
    o[4] = r.lw; o[5] = r.ly; o[6] = t0 - r.lw; o[7] = t1 - r.ly; o[8] = t0; o[9] = t1;
    o[10] = ok ? 1.0 : 0.0;
    // field 12 (stride > 12): the node's NA weight on the chosen feature; 0 =
    // no NA reached this node, so NAs of later data follow the heavier child
    // (DTree.java:1475-1478 decides this per node)
    if (stride > 12) o[12] = H[(((size_t)bf * n + node) * Bs + (Bs - 1)) * 2];
    feat_out[node] = ok ? bf + f0 : 0;
  }
  const int B = Bs - 1;
  for (int c = lane; c < Bs; c += 64) {
    bool left;
    if (!ok) left = true;
    else if (c == Bs - 1) left = r.opt == 1;
    else if (r.opt == 2) left = c < B;
    else left = c <= r.t;
    mask[(size_t)node * Bs + c] = left ? 1 : 0;
  }
}

extern "C" int h2o_split_select2(const void* rec, const double* H, int Fl, int n, int Bs, int f0, double min_w2,
                                 int stride, double* pk, uint8_t* mask, int* feat_out, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(split_select2_kernel, dim3(n), dim3(64), 0, s, (const SplitRec*)rec, H, Fl, n, Bs, f0, min_w2,
                     stride, pk, mask, feat_out);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Pair-based categorical split search (DTree.findBestSplitPoint for enum
// columns: levels ordered by mean response, then the ordered prefix splits).
// One workgroup per eligible (node, feature) pair -- with mtries / column
// sampling only a few features per node are eligible, so pairs, not the full
// [node x feature] grid, are the unit of work.  The pair's bins are read
// straight out of the level histogram H [Fl][n][Bs][C] (no gathered copy),
// (key, bin) is bitonic-sorted in LDS (ties by bin index == a stable sort),
// the sorted channels are prefix-summed in f64, every thread scores its
// thresholds for the three NA placements and a block arg-max (lowest
// concatenated index on ties, like torch's max over [A | B | C]) writes
// (gain, k) per pair.  Numeric pairs keep bin order (no sort).
// out[2p] = gain (-inf if none), out[2p+1] = k in [0, 2(B-1)].
// ---------------------------------------------------------------------------
template <int CRIT, int BP>
__global__ __launch_bounds__(256) void cat_pair_kernel(const double* __restrict__ H, int n, int Bs, int C,
                                                       const int* __restrict__ pf, const int* __restrict__ pn,
                                                       const unsigned char* __restrict__ pcat,
                                                       const float* __restrict__ pmono,
                                                       const double* __restrict__ node_wyy, double min_rows,
                                                       double msi, double lam, double alpha, double gamma,
                                                       double* __restrict__ out, const int* __restrict__ plist,
                                                       const int* __restrict__ pcount, int Bscan,
                                                       const int* __restrict__ pbins) {
  __shared__ double sk[BP];   // sort key, then channel-0 prefix sums
  __shared__ double s1[BP];   // channel-1 prefix sums
  __shared__ int si[BP];      // bin index (sort payload)
  __shared__ double red_g[4];
  __shared__ int red_k[4];
  __shared__ int nfin[256];   // per-thread count of occupied levels, then its exclusive scan
  constexpr int PER = BP / 256;
  // plist: this launch scores the pcount[0] pairs listed (narrow / wide
  // split of a level's pairs); the grid is an upper bound, the rest exit
  int p = blockIdx.x;
  if (plist != nullptr) {
    if (p >= pcount[0]) return;
    p = plist[p];
  }
  const int tid = threadIdx.x;
  const int B = Bs - 1;       // NA bin index; k = i | nt + i | 2 nt over the full width
  // bins scanned: a feature with at most Bscan bins leaves [Bscan, B) empty;
  // thresholds there repeat the all-left partition and lose the lowest-k tie
  const int Bsc = pbins != nullptr ? min(min(B, Bscan), pbins[p]) : min(B, Bscan);
  const double* h = H + ((size_t)pf[p] * n + pn[p]) * (size_t)Bs * C;
  const bool cat = pcat[p] != 0;
  int M = BP;                 // sorted prefix length
  if (!cat) {
    for (int b = tid; b < BP; b += 256) {
      sk[b] = b < Bsc ? (double)b : INFINITY;
      si[b] = b;
    }
  } else {
    // Occupied levels (finite key) first, in bin order, then the empty ones
    // in bin order: the empty levels' INF keys already sit in their final
    // (bin-index) order, so only the occupied prefix -- a few dozen levels
    // of a 1000-level column in a deep node -- goes through the bitonic
    // network.  Same order, hence the same k, as sorting all BP keys.
    double key[PER];
    int cnt = 0;
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int b = tid * PER + e;
      double kk = INFINITY;
      if (b < Bsc) {
        if (CRIT == 1) {
          const double g = h[(size_t)b * C], hh = h[(size_t)b * C + 1];
          kk = hh > 0 ? g / hh : INFINITY;
        } else {
          const double w = h[(size_t)b * C], wy = h[(size_t)b * C + 1];
          kk = w > 0 ? wy / w : INFINITY;
        }
      }
      key[e] = kk;
      cnt += kk < INFINITY ? 1 : 0;
    }
    nfin[tid] = cnt;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {            // inclusive Hillis-Steele scan
      const int u = tid >= d ? nfin[tid - d] : 0;
      __syncthreads();
      nfin[tid] += u;
      __syncthreads();
    }
    const int m = nfin[255];
    int before = nfin[tid] - cnt;                  // occupied levels ahead of this thread's run
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int b = tid * PER + e;
      const bool occ = key[e] < INFINITY;
      const int pos = occ ? before : m + b - before;
      sk[pos] = key[e];
      si[pos] = b;
      before += occ ? 1 : 0;
    }
    M = 2;
    while (M < m) M <<= 1;
  }
  __syncthreads();
  if (cat) {
    for (int k = 2; k <= M; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < M; i += 256) {
          const int l = i ^ j;
          if (l > i) {
            const double a = sk[i], c = sk[l];
            const int ia = si[i], ic = si[l];
            const bool gt = a > c || (a == c && ia > ic);
            const bool up = (i & k) == 0;
            if (gt == up) { sk[i] = c; sk[l] = a; si[i] = ic; si[l] = ia; }
          }
        }
        __syncthreads();
      }
    }
  }
  // gather the sorted channels; per-thread serial prefix over a contiguous run
  double c0[PER], c1[PER];
  double a0 = 0, a1 = 0;
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int b = tid * PER + e;
    double v0 = 0, v1 = 0;
    if (b < Bsc) {
      const int j = si[b];
      v0 = h[(size_t)j * C];
      v1 = h[(size_t)j * C + 1];
    }
    a0 += v0; a1 += v1;
    c0[e] = a0; c1[e] = a1;
  }
  __syncthreads();
  // exclusive scan of the per-thread totals (Hillis-Steele over 256 in LDS)
  sk[tid] = a0; s1[tid] = a1;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {
    const double u0 = tid >= d ? sk[tid - d] : 0.0, u1 = tid >= d ? s1[tid - d] : 0.0;
    __syncthreads();
    sk[tid] += u0; s1[tid] += u1;
    __syncthreads();
  }
  const double off0 = tid > 0 ? sk[tid - 1] : 0.0, off1 = tid > 0 ? s1[tid - 1] : 0.0;
  const double tw = sk[255], ty = s1[255];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    sk[tid * PER + e] = off0 + c0[e];
    s1[tid * PER + e] = off1 + c1[e];
  }
  __syncthreads();
  const double nw = h[(size_t)B * C], ny = h[(size_t)B * C + 1];
  const double Tw = tw + nw, Ty = ty + ny;
  const double sT = score<CRIT>(Tw, Ty, lam, alpha);
  const bool has_na = CRIT == 1 ? (ny > 0 || nw != 0) : (nw > 0);
  const double mo = pmono ? (double)pmono[p] : 0.0;
  double se_before = 0;
  bool dead = false;
  if (CRIT == 0) {
    se_before = fmax((node_wyy ? node_wyy[pn[p]] : 0.0) - sT, 0.0);
    dead = !(se_before > 0);
  }
  const int nt = B - 1;
  double bg = -INFINITY;
  int bk = 0x7fffffff;
  const int nts = min(nt, Bsc);
  if (!dead) {
    for (int i = tid; i < nts; i += 256) {
      const double lw = sk[i], ly = s1[i];
      const double rw = tw - lw, ry = ty - ly;
      {
        const double RW = rw + nw, RY = ry + ny;
        if (valid_split<CRIT>(lw, ly, RW, RY, min_rows, lam, mo)) {
          double g = score<CRIT>(lw, ly, lam, alpha) + score<CRIT>(RW, RY, lam, alpha) - sT;
          if (CRIT == 1) g = 0.5 * g - gamma;
          if (g > bg || (g == bg && i < bk)) { bg = g; bk = i; }
        }
      }
      if (has_na) {
        const double LW = lw + nw, LY = ly + ny;
        if (valid_split<CRIT>(LW, LY, rw, ry, min_rows, lam, mo)) {
          double g = score<CRIT>(LW, LY, lam, alpha) + score<CRIT>(rw, ry, lam, alpha) - sT;
          if (CRIT == 1) g = 0.5 * g - gamma;
          if (g > bg || (g == bg && nt + i < bk)) { bg = g; bk = nt + i; }
        }
      }
    }
    if (tid == 0 && has_na && valid_split<CRIT>(tw, ty, nw, ny, min_rows, lam, mo)) {
      double g = score<CRIT>(tw, ty, lam, alpha) + score<CRIT>(nw, ny, lam, alpha) - sT;
      if (CRIT == 1) g = 0.5 * g - gamma;
      if (g > bg || (g == bg && 2 * nt < bk)) { bg = g; bk = 2 * nt; }
    }
  }
  // block arg-max: larger gain, then lower k
  const int lane = tid & 63, wv = tid >> 6;
  for (int o = 32; o > 0; o >>= 1) {
    const double og = __shfl_xor(bg, o, 64);
    const int ok = __shfl_xor(bk, o, 64);
    if (og > bg || (og == bg && ok < bk)) { bg = og; bk = ok; }
  }
  if (lane == 0) { red_g[wv] = bg; red_k[wv] = bk; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w)
      if (red_g[w] > bg || (red_g[w] == bg && red_k[w] < bk)) { bg = red_g[w]; bk = red_k[w]; }
    bool keep = bg > -INFINITY;
    if (CRIT == 0) keep = keep && bg > se_before * msi;
    else keep = keep && bg > 0;
    out[2 * (size_t)p] = keep ? bg : -INFINITY;
    out[2 * (size_t)p + 1] = keep ? (double)bk : 0.0;
  }
}

template <int CRIT>
static int cat_pair_launch(int BP, dim3 g, hipStream_t s, const double* H, int n, int Bs, int C, const int* pf,
                           const int* pn, const unsigned char* pcat, const float* pmono, const double* wyy,
                           double min_rows, double msi, double lam, double alpha, double gamma, double* out,
                           const int* plist = nullptr, const int* pcount = nullptr, int Bscan = 1 << 30,
                           const int* pbins = nullptr) {
#define CPK(bp)                                                                                                \
  case bp:                                                                                                     \
    hipLaunchKernelGGL((cat_pair_kernel<CRIT, bp>), g, dim3(256), 0, s, H, n, Bs, C, pf, pn, pcat, pmono, wyy, \
                       min_rows, msi, lam, alpha, gamma, out, plist, pcount, Bscan, pbins);                    \
    return 0;
  switch (BP) {
    CPK(256) CPK(512) CPK(1024) CPK(2048) CPK(4096)
    default: return -2;
  }
#undef CPK
}

// P pairs (pf: local feature slot, pn: node) of the level histogram H
// [Fl][n][Bs][C] f64; Bs - 1 <= 4096.
extern "C" int h2o_cat_pairs(const double* H, int n, int Bs, int C, int P, const int* pf, const int* pn,
                             const unsigned char* pcat, const float* pmono, const double* node_wyy, double min_rows,
                             double msi, double lam, double alpha, double gamma, int crit, double* out,
                             hipStream_t s) {
  if (P <= 0) return 0;
  if (C < 2 || Bs < 2) return -1;
  int BP = 256;
  while (BP < Bs - 1) BP <<= 1;
  if (BP > 4096) return -2;
  const dim3 g(P);
  const int rc = crit == 1 ? cat_pair_launch<1>(BP, g, s, H, n, Bs, C, pf, pn, pcat, pmono, node_wyy, min_rows,
                                                  msi, lam, alpha, gamma, out)
                           : cat_pair_launch<0>(BP, g, s, H, n, Bs, C, pf, pn, pcat, pmono, node_wyy, min_rows,
                                                msi, lam, alpha, gamma, out);
  if (rc) return rc;
  return (int)hipGetLastError();
}

// Narrow / wide pair lists for h2o_cat_pairs2: pairs whose feature has at
// most narrow_max bins go to lists[0..cnt0), the others to lists[P..P+cnt1)
// (wave-aggregated atomics; order inside a list is irrelevant -- every pair
// writes its own out[2p]).
__global__ __launch_bounds__(256) void pair_lists_kernel(const int* __restrict__ pbins, int P, int narrow_max,
                                                         int* __restrict__ lists, int* __restrict__ cnt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = p < P;
  const bool nar = live && pbins[p] <= narrow_max;
  const int lane = threadIdx.x & 63;
  const unsigned long long act = __ballot(live);
  if (act == 0ull) return;
  const unsigned long long bn = __ballot(nar);
  const unsigned long long bw = act & ~bn;
  const int leader = __ffsll((long long)act) - 1;
  int baseN = 0, baseW = 0;
  if (lane == leader) {
    baseN = atomicAdd(cnt, (int)__popcll(bn));
    baseW = atomicAdd(cnt + 1, (int)__popcll(bw));
  }
  baseN = __shfl(baseN, leader, 64);
  baseW = __shfl(baseW, leader, 64);
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  if (!live) return;
  if (nar) lists[baseN + __popcll(bn & below)] = p;
  else lists[P + baseW + __popcll(bw & below)] = p;
}

// h2o_cat_pairs with the level's pairs split by width: pairs of features with
// <= narrow_max (< 256) bins run the BP = 256 instance (a quarter of the LDS
// scans and scoring of the 1024-wide one), the rest the full-width instance.
// pbins[P]: bins of each pair's feature; lists: int[2P + 2] scratch.
extern "C" int h2o_cat_pairs2(const double* H, int n, int Bs, int C, int P, const int* pf, const int* pn,
                              const unsigned char* pcat, const float* pmono, const double* node_wyy,
                              double min_rows, double msi, double lam, double alpha, double gamma, int crit,
                              double* out, const int* pbins, int narrow_max, int* lists, hipStream_t s) {
  if (P <= 0) return 0;
  if (C < 2 || Bs < 2 || narrow_max < 1 || narrow_max > 255) return -1;
  int BP = 256;
  while (BP < Bs - 1) BP <<= 1;
  if (BP > 4096) return -2;
  int* cnt = lists + 2 * (size_t)P;
  hipMemsetAsync(cnt, 0, 2 * sizeof(int), s);
  hipLaunchKernelGGL(pair_lists_kernel, dim3((P + 255) / 256), dim3(256), 0, s, pbins, P, narrow_max, lists, cnt);
  const dim3 g(P);
  int rc = crit == 1 ? cat_pair_launch<1>(256, g, s, H, n, Bs, C, pf, pn, pcat, pmono, node_wyy, min_rows, msi,
                                          lam, alpha, gamma, out, lists, cnt, narrow_max, pbins)
                     : cat_pair_launch<0>(256, g, s, H, n, Bs, C, pf, pn, pcat, pmono, node_wyy, min_rows, msi,
                                          lam, alpha, gamma, out, lists, cnt, narrow_max, pbins);
  if (rc) return rc;
  rc = crit == 1 ? cat_pair_launch<1>(BP, g, s, H, n, Bs, C, pf, pn, pcat, pmono, node_wyy, min_rows, msi, lam,
                                      alpha, gamma, out, lists + P, cnt + 1, Bs - 1, pbins)
                 : cat_pair_launch<0>(BP, g, s, H, n, Bs, C, pf, pn, pcat, pmono, node_wyy, min_rows, msi, lam,
                                      alpha, gamma, out, lists + P, cnt + 1, Bs - 1, pbins);
  if (rc) return rc;
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per-node winner + split record of the row-direct pair path.  The frontier's
// pairs are node-major with kp pairs per node (the node's sampled features in
// ascending order); res[2p] = gain, res[2p + 1] = k from cat_pair_kernel.
// One workgroup per node: winner = largest gain, lowest feature on ties (the
// reference scans columns in order and keeps the first best); the record and
// go-left mask are rebuilt from the winner's own histogram Hp[pair] (for a
// categorical winner the (mean response, bin) order is re-sorted in LDS, the
// same key and tie rule as the scoring kernel), so the level needs no host
// round trip: the output is split_select2_kernel's packed record
//   pk[node] = {gain, feat, t, opt, L0, L1, R0, R1, T0, T1, ok}
// plus mask[node][Bs] (all ones when the node does not split) and feat_out.
// T = node totals from the winner's (or the first pair's) histogram.
// ---------------------------------------------------------------------------
template <int CRIT, int BP>
__global__ __launch_bounds__(256) void pair_select_kernel(const double* __restrict__ Hp, int Bs, int kp,
                                                          const double* __restrict__ res,
                                                          const int* __restrict__ pfeat,
                                                          const unsigned char* __restrict__ fcat, double min_w2,
                                                          int stride, double* __restrict__ pk,
                                                          uint8_t* __restrict__ mask, int* __restrict__ feat_out,
                                                          const int* __restrict__ fbins) {
  __shared__ double sk[BP];
  __shared__ int si[BP];
  __shared__ double rg[4];
  __shared__ int rj[4];
  __shared__ double rs[4][4];
  const int node = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int B = Bs - 1;
  // winner over the node's kp pairs
  double bg = -INFINITY;
  int bj = 0x7fffffff;
  for (int j = tid; j < kp; j += 256) {
    const double g = res[2 * ((size_t)node * kp + j)];
    if (g > bg || (g == bg && j < bj)) { bg = g; bj = j; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const double og = __shfl_xor(bg, o, 64);
    const int oj = __shfl_xor(bj, o, 64);
    if (og > bg || (og == bg && oj < bj)) { bg = og; bj = oj; }
  }
  if (lane == 0) { rg[wv] = bg; rj[wv] = bj; }
  __syncthreads();
  bg = rg[0]; bj = rj[0];
  for (int w = 1; w < 4; ++w)
    if (rg[w] > bg || (rg[w] == bg && rj[w] < bj)) { bg = rg[w]; bj = rj[w]; }
  const bool win = bg > -INFINITY && bj < kp;
  const size_t pw = (size_t)node * kp + (win ? bj : 0);
  const double* h = Hp + pw * (size_t)Bs * 2;
  const int f = pfeat[pw];
  const bool cat = win && fcat[f] != 0;
  const int kk = win ? (int)res[2 * pw + 1] : 0;
  const int nt = B - 1;
  const int opt = kk < nt ? 0 : (kk < 2 * nt ? 1 : 2);
  const int t = opt == 0 ? kk : (opt == 1 ? kk - nt : 0);
  const bool na_left = opt == 1;
  // bins of the winner's feature: [Bw, B) hold no rows (and may be unwritten)
  const int Bw = fbins != nullptr ? min(B, fbins[f]) : B;
  // rank of every non-NA bin in the split order
  for (int b = tid; b < BP; b += 256) {
    double key = INFINITY;
    if (b < Bw) {
      if (!cat) {
        key = (double)b;
      } else {
        const double a0 = h[2 * (size_t)b], a1 = h[2 * (size_t)b + 1];
        key = CRIT == 1 ? (a1 > 0 ? a0 / a1 : INFINITY) : (a0 > 0 ? a1 / a0 : INFINITY);
      }
    }
    sk[b] = key;
    si[b] = b;
  }
  __syncthreads();
  if (cat) {
    for (int k = 2; k <= BP; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < BP; i += 256) {
          const int l = i ^ j;
          if (l > i) {
            const double a = sk[i], c = sk[l];
            const int ia = si[i], ic = si[l];
            const bool gt = a > c || (a == c && ia > ic);
            const bool up = (i & k) == 0;
            if (gt == up) { sk[i] = c; sk[l] = a; si[i] = ic; si[l] = ia; }
          }
        }
        __syncthreads();
      }
    }
  }
  // sk[] is free now: reuse it as rank-by-bin
  int* rank = reinterpret_cast<int*>(sk);   // BP ints fit in BP doubles
  for (int r = tid; r < BP; r += 256) rank[si[r]] = r;
  __syncthreads();
  // left / total sums and the mask
  double l0 = 0, l1 = 0, t0 = 0, t1 = 0, n0 = 0, n1 = 0;
  for (int b = tid; b < Bs; b += 256) {
    const bool live = b < Bw || b >= B;
    const double a0 = live ? h[2 * (size_t)b] : 0.0, a1 = live ? h[2 * (size_t)b + 1] : 0.0;
    t0 += a0; t1 += a1;
    bool left;
    if (b >= B) {
      left = na_left;
    } else {
      n0 += a0; n1 += a1;
      const bool in_left = rank[b] <= t;
      const double bw = CRIT == 1 ? a1 : a0;
      const bool empty = cat && bw <= 0;
      if (opt == 2) left = !empty || na_left;
      else left = empty ? na_left : in_left;
      if (opt != 2 && in_left) { l0 += a0; l1 += a1; }
    }
    mask[(size_t)node * Bs + b] = left ? 1 : 0;   // overwritten below when the node does not split
  }
  double v[6] = {l0, l1, t0, t1, n0, n1};
#pragma unroll
  for (int q = 0; q < 6; ++q) v[q] = wave_sum(v[q]);
  __syncthreads();
  __shared__ double red6[6][4];
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < 6; ++q) red6[q][wv] = v[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 6; ++q) v[q] = red6[q][0] + red6[q][1] + red6[q][2] + red6[q][3];
  const double na0 = v[2] - v[4], na1 = v[3] - v[5];
  double L0, L1;
  if (opt == 2) { L0 = v[4]; L1 = v[5]; }
  else { L0 = v[0] + (na_left ? na0 : 0.0); L1 = v[1] + (na_left ? na1 : 0.0); }
  const bool ok = win && isfinite(bg) && (min_w2 < 0.0 || v[2] >= min_w2);
  if (tid == 0) {
    double* o = pk + (size_t)node * stride;
    o[0] = bg; o[1] = (double)f; o[2] = (double)t; o[3] = (double)opt;
    o[4] = L0; o[5] = L1; o[6] = v[2] - L0; o[7] = v[3] - L1; o[8] = v[2]; o[9] = v[3];
    o[10] = ok ? 1.0 : 0.0;
    if (stride > 12) o[12] = na0;   // the node's NA weight on the winner (per-node NA direction)
    feat_out[node] = ok ? f : 0;
  }
  if (!ok) {
    __syncthreads();
    for (int b = tid; b < Bs; b += 256) mask[(size_t)node * Bs + b] = 1;
  }
}

template <int CRIT>
static int pair_select_launch(int BP, int n, hipStream_t s, const double* Hp, int Bs, int kp, const double* res,
                              const int* pfeat, const unsigned char* fcat, double min_w2, int stride, double* pk,
                              uint8_t* mask, int* feat_out, const int* fbins = nullptr) {
#define PSK(bp)                                                                                                   \
  case bp:                                                                                                        \
    hipLaunchKernelGGL((pair_select_kernel<CRIT, bp>), dim3(n), dim3(256), 0, s, Hp, Bs, kp, res, pfeat, fcat, \
                       min_w2, stride, pk, mask, feat_out, fbins);                                                \
    return 0;
  switch (BP) {
    PSK(256) PSK(512) PSK(1024) PSK(2048) PSK(4096)
    default: return -2;
  }
#undef PSK
}

// n nodes x kp pairs (node-major); Hp [n*kp][Bs][2] f64; res [n*kp][2]
// (cat_pair_kernel output); pfeat [n*kp] global feature ids; fcat [F] u8.
extern "C" int h2o_pair_select(const double* Hp, int n, int Bs, int kp, const double* res, const int* pfeat,
                               const unsigned char* fcat, int crit, double min_w2, int stride, double* pk,
                               uint8_t* mask, int* feat_out, hipStream_t s) {
  if (n <= 0) return 0;
  if (kp <= 0 || Bs < 3 || stride < 11) return -1;
  int BP = 256;
  while (BP < Bs - 1) BP <<= 1;
  if (BP > 4096) return -2;
  const int rc = crit == 1 ? pair_select_launch<1>(BP, n, s, Hp, Bs, kp, res, pfeat, fcat, min_w2, stride, pk, mask,
                                                   feat_out)
                           : pair_select_launch<0>(BP, n, s, Hp, Bs, kp, res, pfeat, fcat, min_w2, stride, pk, mask,
                                                   feat_out);
  if (rc) return rc;
  return (int)hipGetLastError();
}

// h2o_pair_select for pair histograms written up to each feature's bins
// (fbins [F]: codes below the NA bin; h2o_pair_hist4b).
extern "C" int h2o_pair_select2(const double* Hp, int n, int Bs, int kp, const double* res, const int* pfeat,
                                const unsigned char* fcat, int crit, double min_w2, int stride, double* pk,
                                uint8_t* mask, int* feat_out, const int* fbins, hipStream_t s) {
  if (n <= 0) return 0;
  if (kp <= 0 || Bs < 3 || stride < 11) return -1;
  int BP = 256;
  while (BP < Bs - 1) BP <<= 1;
  if (BP > 4096) return -2;
  const int rc = crit == 1 ? pair_select_launch<1>(BP, n, s, Hp, Bs, kp, res, pfeat, fcat, min_w2, stride, pk, mask,
                                                   feat_out, fbins)
                           : pair_select_launch<0>(BP, n, s, Hp, Bs, kp, res, pfeat, fcat, min_w2, stride, pk, mask,
                                                   feat_out, fbins);
  if (rc) return rc;
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// UniformAdaptive per-node re-binning on the device (reference
// DHistogram.java:366-386 / DTree.java:337: each (node, column) histogram is
// re-binned into nb uniform bins over the column's range in that node).  The
// level histogram H [Fl][n][Bs][C] (f64, Bs = B fine cells + the NA bin) is on
// the fixed grid of nbins_top_level cells; a node's coarse bin is a run of
// fine cells, and folding each run into its LAST cell keeps every cumulative
// sum at an allowed boundary (any split search then only sees coarse
// boundaries).  Two kernels, one 64-lane wave per (feature, node) row:
//   ua_range: first / last occupied fine cell (any channel != 0), or (B, -1);
//   ua_fold:  out[b] = sum of H over (previous end, b] at every run end b,
//             0 elsewhere; categorical rows and the NA bin copied unchanged.
// Lane l owns cells [l*cpl, (l+1)*cpl); the carry into a lane (the sum since
// the last end before its first cell) is a segmented wave scan of the lanes'
// tails.  Replaces the torch chain (occupancy, amin/amax, cumsum, cummax,
// gather, where) on [Fl, n, B, C] f64 tensors of models/tree/engine.py.
constexpr int UA_MAXC = 4;

__global__ __launch_bounds__(256) void ua_range_kernel(const double* __restrict__ H, int rows, int Bs, int C,
                                                       int* __restrict__ first, int* __restrict__ last) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int B = Bs - 1;
  const double* h = H + (long long)row * Bs * C;
  int lo = B, hi = -1;
  for (int b = lane; b < B; b += 64) {
    bool occ = false;
    for (int c = 0; c < C; ++c) occ |= h[(long long)b * C + c] != 0.0;
    if (occ) { lo = min(lo, b); hi = max(hi, b); }
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o, 64));
    hi = max(hi, __shfl_xor(hi, o, 64));
  }
  if (lane == 0) { first[row] = lo; last[row] = hi; }
}

__global__ __launch_bounds__(256) void ua_fold_kernel(const double* __restrict__ H, int Fl, int n, int Bs, int C,
                                                      const int* __restrict__ first, const int* __restrict__ last,
                                                      int nb, const unsigned char* __restrict__ isnum,
                                                      double* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= Fl * n) return;
  const int f = row / n;
  const int B = Bs - 1;
  const double* h = H + (long long)row * Bs * C;
  double* o = out + (long long)row * Bs * C;
  if (!isnum[f]) {
    for (int e = lane; e < Bs * C; e += 64) o[e] = h[e];
    return;
  }
  for (int c = lane; c < C; c += 64) o[(long long)B * C + c] = h[(long long)B * C + c];   // NA bin
  const long long fi = first[row], la = last[row];
  const long long L = max(la - fi + 1, 1LL);
  const bool narrow = L <= nb;
  const int cpl = (B + 63) / 64;
  const int b0 = lane * cpl, b1 = min(B, b0 + cpl);
  auto is_end = [&](long long b) -> bool {
    if (b < fi || b > la) return false;
    if (narrow || b == la) return true;
    const long long cur = ((b - fi) * nb) / L;
    const long long nxt = ((b + 1 - fi) * nb) / L;
    return cur != nxt;
  };
  // pass 1: this lane's tail (sum after its last end) and whether it has an end
  double tail[UA_MAXC];
  for (int c = 0; c < UA_MAXC; ++c) tail[c] = 0.0;
  int has_end = 0;
  for (int b = b0; b < b1; ++b) {
    for (int c = 0; c < UA_MAXC; ++c)
      if (c < C) tail[c] += h[(long long)b * C + c];
    if (is_end(b)) {
      has_end = 1;
      for (int c = 0; c < UA_MAXC; ++c) tail[c] = 0.0;
    }
  }
  // segmented inclusive scan over lanes: (f1, v1) + (f2, v2) = (f1 | f2, f2 ? v2 : v1 + v2)
  int fl = has_end;
  double v[UA_MAXC];
  for (int c = 0; c < UA_MAXC; ++c) v[c] = tail[c];
  for (int o = 1; o < 64; o <<= 1) {
    const int pf = __shfl_up(fl, o, 64);
    double pv[UA_MAXC];
    for (int c = 0; c < UA_MAXC; ++c) pv[c] = __shfl_up(v[c], o, 64);
    if (lane >= o) {
      if (!fl)
        for (int c = 0; c < UA_MAXC; ++c) v[c] += pv[c];
      fl |= pf;
    }
  }
  // carry into this lane = the previous lane's inclusive value
  double run[UA_MAXC];
  for (int c = 0; c < UA_MAXC; ++c) {
    const double pv = __shfl_up(v[c], 1, 64);
    run[c] = lane > 0 ? pv : 0.0;
  }
  // pass 2: write the folded cells
  for (int b = b0; b < b1; ++b) {
    const bool e = is_end(b);
    for (int c = 0; c < UA_MAXC; ++c) {
      if (c < C) {
        run[c] += h[(long long)b * C + c];
        o[(long long)b * C + c] = e ? run[c] : 0.0;
        if (e) run[c] = 0.0;
      }
    }
  }
}

extern "C" int h2o_ua_range(const double* H, int rows, int Bs, int C, int* first, int* last, hipStream_t s) {
  if (rows <= 0) return 0;
  if (Bs < 2 || C < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ua_range_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, H, rows, Bs, C, first, last);
  return (int)hipGetLastError();
}

extern "C" int h2o_ua_fold(const double* H, int Fl, int n, int Bs, int C, const int* first, const int* last, int nb,
                           const unsigned char* isnum, double* out, hipStream_t s) {
  const int rows = Fl * n;
  if (rows <= 0) return 0;
  if (Bs < 2 || C < 1 || C > UA_MAXC || nb < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ua_fold_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, H, Fl, n, Bs, C, first, last, nb, isnum,
                     out);
  return (int)hipGetLastError();
}
