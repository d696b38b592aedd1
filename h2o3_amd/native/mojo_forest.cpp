// Host forest scorer for the standalone reference-layout MOJO reader
// (h2o3_amd/mojo/h2o_mojo.py _Tree arrays): every tree of a GBM / DRF / IF /
// uplift MOJO, decoded once into flat node arrays, walked per row in native
// code on a pool of threads (rows split across threads, so the per-row sums
// need no atomics).  The scoring rule is the reader's -- and the reference's
// SharedTreeMojoModel.scoreTree (h2o-genmodel .../algos/tree/
// SharedTreeMojoModel.java): numeric "d >= split goes right" on the float
// split value, bitset membership with the 1.1+ out-of-range-is-NA rule, the
// 1.2+ unseen-level-is-NA rule, NAs to the node's NA direction.  The numpy
// level-by-level walk in h2o_mojo.py stays as the fallback and the spec.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

namespace {

struct Forest {
  long long n;
  int ncols;
  const double* X;
  int ntrees;
  const long long* node_off;
  const long long* leaf_off;
  const long long* raw_off;
  const long long* raw_len;
  const int32_t* col;
  const int8_t* kind;
  const double* split;
  const uint8_t* na_left;
  const int64_t* bs_off;
  const int64_t* bs_n;
  const int64_t* bs_pos;
  const int64_t* left;
  const int64_t* right;
  const double* leaf;
  const uint8_t* raw;
  const double* root_leaf;
  const uint8_t* has_root_leaf;
  const int32_t* tree_out;
  int nout;
  double* out;
  double version;
  const int32_t* dom_len;
};

inline double tree_value(const Forest& F, int t, const double* row) {
  if (F.has_root_leaf[t]) return F.root_leaf[t];
  const long long no = F.node_off[t];
  const uint8_t* raw = F.raw + F.raw_off[t];
  const long long rlen = F.raw_len[t];
  long long j = 0;
  for (;;) {
    const long long g = no + j;
    const int c = F.col[g];
    const double d = row[c];
    bool nan = std::isnan(d);
    long long di = 0;
    if (!nan) di = d >= 9.0e18 ? (long long)9e18 : (d <= -9.0e18 ? (long long)-9e18 : (long long)d);
    bool right = false;
    const int k = F.kind[g];
    if (k == 0) {
      right = d >= F.split[g];
    } else if (k == 1) {
      const long long rel = di - F.bs_off[g];
      const bool inr = rel >= 0 && rel < F.bs_n[g];
      const long long relc = rel < 0 ? 0 : rel;
      long long bi = F.bs_pos[g] + (relc >> 3);
      if (bi > rlen - 1) bi = rlen - 1;
      right = inr && ((raw[bi] >> (relc & 7)) & 1);
      if (F.version >= 1.1) nan = nan || !inr;
    }
    if (F.version >= 1.2 && F.dom_len != nullptr) {
      const int dl = F.dom_len[c];
      nan = nan || (dl > 0 && di >= dl && !std::isnan(d));
    }
    const bool go_right = nan ? !F.na_left[g] : right;
    const long long nxt = go_right ? F.right[g] : F.left[g];
    if (nxt < 0) return F.leaf[F.leaf_off[t] + (-nxt - 1)];
    j = nxt;
  }
}

void score_rows(const Forest& F, long long r0, long long r1) {
  for (long long r = r0; r < r1; ++r) {
    const double* row = F.X + r * F.ncols;
    double* o = F.out + r * F.nout;
    for (int t = 0; t < F.ntrees; ++t) o[F.tree_out[t]] += tree_value(F, t, row);
  }
}

}  // namespace

extern "C" int h2o_mojo_forest_score(long long n, int ncols, const double* X, int ntrees, const long long* node_off,
                                     const long long* leaf_off, const long long* raw_off, const long long* raw_len,
                                     const int32_t* col, const int8_t* kind, const double* split,
                                     const uint8_t* na_left, const int64_t* bs_off, const int64_t* bs_n,
                                     const int64_t* bs_pos, const int64_t* left, const int64_t* right,
                                     const double* leaf, const uint8_t* raw, const double* root_leaf,
                                     const uint8_t* has_root_leaf, const int32_t* tree_out, int nout, double* out,
                                     double version, const int32_t* dom_len, int nthreads) {
  if (n <= 0 || ntrees <= 0) return 0;
  if (!X || !out || ncols <= 0 || nout <= 0) return 1;
  Forest F{n, ncols, X, ntrees, node_off, leaf_off, raw_off, raw_len, col, kind, split, na_left, bs_off, bs_n,
           bs_pos, left, right, leaf, raw, root_leaf, has_root_leaf, tree_out, nout, out, version, dom_len};
  int nt = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = (int)std::min<long long>(nt, std::max<long long>(1, n / 256));
  if (nt <= 1) {
    score_rows(F, 0, n);
    return 0;
  }
  std::vector<std::thread> th;
  const long long per = (n + nt - 1) / nt;
  for (int i = 0; i < nt; ++i) {
    const long long a = i * per, b = std::min(n, a + per);
    if (a >= b) break;
    th.emplace_back(score_rows, std::cref(F), a, b);
  }
  for (auto& t : th) t.join();
  return 0;
}

// XGBoost booster trees (mojo/xgb_booster.py, the legacy binary layout): per
// row, trees in booster order, f32 "v < cond goes left", missing to the
// node's default direction, leaf value (x the DART weight) added in f32 into
// the tree's output group -- the same f32 sums, in the same order, as the
// numpy walk (XGBoostJavaMojoModel / Predictor.predict semantics).
namespace {
struct XgbForest {
  long long n;
  int nfeat;
  const float* F;
  int ntrees;
  const long long* node_off;
  const int32_t* cleft;
  const int32_t* cright;
  const int32_t* feat;
  const uint8_t* dleft;
  const float* info;
  const int32_t* group;
  const float* wdrop;
  int ngroups;
  float* acc;
};

void xgb_rows(const XgbForest& X, long long r0, long long r1) {
  for (long long r = r0; r < r1; ++r) {
    const float* row = X.F + r * X.nfeat;
    float* a = X.acc + r * X.ngroups;
    for (int t = 0; t < X.ntrees; ++t) {
      const long long o = X.node_off[t];
      int c = 0;
      while (X.cleft[o + c] != -1) {
        const float v = row[X.feat[o + c]];
        const bool left = std::isnan(v) ? X.dleft[o + c] != 0 : v < X.info[o + c];
        c = left ? X.cleft[o + c] : X.cright[o + c];
      }
      float lv = X.info[o + c];
      if (X.wdrop != nullptr) lv = lv * X.wdrop[t];
      a[X.group[t]] += lv;
    }
  }
}
}  // namespace

extern "C" int h2o_xgb_forest_score(long long n, int nfeat, const float* F, int ntrees, const long long* node_off,
                                    const int32_t* cleft, const int32_t* cright, const int32_t* feat,
                                    const uint8_t* dleft, const float* info, const int32_t* group,
                                    const float* wdrop, int ngroups, float* acc, int nthreads) {
  if (n <= 0 || ntrees <= 0) return 0;
  if (!F || !acc || nfeat <= 0 || ngroups <= 0) return 1;
  XgbForest X{n, nfeat, F, ntrees, node_off, cleft, cright, feat, dleft, info, group, wdrop, ngroups, acc};
  int nt = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = (int)std::min<long long>(nt, std::max<long long>(1, n / 256));
  if (nt <= 1) {
    xgb_rows(X, 0, n);
    return 0;
  }
  std::vector<std::thread> th;
  const long long per = (n + nt - 1) / nt;
  for (int i = 0; i < nt; ++i) {
    const long long a = i * per, b = std::min(n, a + per);
    if (a >= b) break;
    th.emplace_back(xgb_rows, std::cref(X), a, b);
  }
  for (auto& t : th) t.join();
  return 0;
}
