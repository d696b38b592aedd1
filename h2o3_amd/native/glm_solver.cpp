// Host-side GLM penalized quadratic solver (the per-IRLS-iteration inner
// problem): minimise 1/2 b'Gb - r'b + l1 sum pen_j |b_j| + l2/2 sum pen_j b_j^2
// subject to lo <= b <= hi, by cyclic coordinate descent on the dense Gram.
//
// Reference: hex/glm/GLM.java (COD solver, fitCOD) and hex/optimization/ADMM.java
// (L1 solver over the Cholesky of the Gram).  Here the Gram is at most a few
// thousand wide and lives in host memory after the RCCL all-reduce; one sweep is
// P dense column updates (P^2 flops), with an active-set inner loop: after a
// full sweep only the non-zero coordinates are swept until they settle, then a
// full sweep re-checks the zeros (the usual KKT-checked active-set CD).
#include <cmath>
#include <cstring>
#include <vector>

extern "C" int h2o_glm_cd(int P, const double* G, const double* r, const double* pen, const double* lo,
                          const double* hi, double l1, double l2, double* beta, int max_iter, double tol) {
  std::vector<double> grad(P), diag(P);
  // grad = r - G beta ; G symmetric row-major
  for (int i = 0; i < P; ++i) {
    double s = r[i];
    const double* gi = G + (size_t)i * P;
    for (int j = 0; j < P; ++j) s -= gi[j] * beta[j];
    grad[i] = s;
    diag[i] = G[(size_t)i * P + i] + l2 * pen[i];
  }
  auto update = [&](int j) -> double {
    if (diag[j] <= 0) return 0.0;
    const double old = beta[j];
    const double v = grad[j] + G[(size_t)j * P + j] * old;
    const double t = l1 * pen[j];
    double nb = v > t ? v - t : (v < -t ? v + t : 0.0);
    nb /= diag[j];
    if (nb < lo[j]) nb = lo[j];
    if (nb > hi[j]) nb = hi[j];
    if (nb == old) return 0.0;
    const double d = nb - old;
    const double* gj = G + (size_t)j * P;  // column j == row j (symmetric)
    for (int i = 0; i < P; ++i) grad[i] -= gj[i] * d;
    beta[j] = nb;
    return std::fabs(d);
  };
  // Inner active-set sweeps keep only the active coordinates' gradients
  // current (|act|^2 per sweep instead of |act| P: the rule lasso of RuleFit
  // has a few dozen non-zeros among ~1000 rules); the full gradient is
  // rebuilt from the non-zeros before the next KKT-checking full sweep.
  std::vector<int> act;
  auto update_act = [&](int j) -> double {
    if (diag[j] <= 0) return 0.0;
    const double old = beta[j];
    const double v = grad[j] + G[(size_t)j * P + j] * old;
    const double t = l1 * pen[j];
    double nb = v > t ? v - t : (v < -t ? v + t : 0.0);
    nb /= diag[j];
    if (nb < lo[j]) nb = lo[j];
    if (nb > hi[j]) nb = hi[j];
    if (nb == old) return 0.0;
    const double d = nb - old;
    const double* gj = G + (size_t)j * P;
    for (int i : act) grad[i] -= gj[i] * d;
    beta[j] = nb;
    return std::fabs(d);
  };
  auto refresh = [&]() {
    std::vector<int> nz;
    for (int j = 0; j < P; ++j)
      if (beta[j] != 0.0) nz.push_back(j);
    for (int i = 0; i < P; ++i) {
      double s = r[i];
      const double* gi = G + (size_t)i * P;
      for (int j : nz) s -= gi[j] * beta[j];
      grad[i] = s;
    }
  };
  int it = 0;
  for (; it < max_iter; ++it) {
    double maxd = 0.0;
    for (int j = 0; j < P; ++j) maxd = std::fmax(maxd, update(j));
    if (maxd < tol) break;
    act.clear();
    for (int j = 0; j < P; ++j)
      if (beta[j] != 0.0) act.push_back(j);
    if ((int)act.size() < P) {
      for (int k = 0; k < max_iter; ++k) {
        double m = 0.0;
        for (int j : act) m = std::fmax(m, update_act(j));
        if (m < tol) break;
      }
      refresh();
    }
  }
  return it;
}
