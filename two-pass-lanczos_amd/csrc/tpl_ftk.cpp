// tpl_ftk.cpp — built-in f(T_k) e_1 solvers for the projected tridiagonal problem.
//
// They replace the harness closures of the reference:
//   inv: sparse LU of T_k (src/bin/tradeoff.rs:97-132,245-258; src/bin/stability.rs:161-170)
//        or dense partial-pivot LU (tests/correctness.rs:171-179) -> here: tridiagonal
//        Gaussian elimination with partial pivoting (the LAPACK dgtsv scheme), O(k).
//   exp: dense self-adjoint EVD, y' = Q exp(Lambda) Q^T e_1 (src/bin/stability.rs:175-193)
//        -> here: implicit-shift QL on the tridiagonal T_k; Q is applied through its
//        recorded rotations (O(k^2)) instead of being accumulated (O(k^3)).
//   sq : y' = T_k^2 e_1 (tests/correctness.rs:287-299).
// inv and sq are O(k), exp O(k^2) host work on at most 2k doubles: small next to
// the 2k-1 device SpMVs of a solve.
#include <cmath>
#if defined(__x86_64__)
#include <xmmintrin.h>
#endif
#include <cstring>
#include <string>
#include <vector>

#include "tpl_internal.h"

namespace {

// sqrt(a^2 + b^2) without over/underflow: the plain formula when both magnitudes are
// safely inside the double range (the usual case; glibc's hypot costs ~10x more and
// dominates the QL sweep), std::hypot otherwise.
inline double hyp(double a, double b) {
  const double fa = std::fabs(a), fb = std::fabs(b);
  const double big = fa > fb ? fa : fb, small = fa > fb ? fb : fa;
  if (big < 1e150 && (small > 1e-150 || small == 0.0)) return std::sqrt(a * a + b * b);
  return std::hypot(a, b);
}

void put_err(char* err, size_t cap, const std::string& m) {
  if (!err || cap == 0) return;
  const size_t n = m.size() < cap - 1 ? m.size() : cap - 1;
  std::memcpy(err, m.data(), n);
  err[n] = '\0';
}

} // namespace

extern "C" {

int tpl_ftk_inv(const double* alphas, size_t n_alphas, const double* betas, size_t n_betas,
                double* y_out, size_t y_cap, size_t* y_len, char* err_msg, size_t err_cap,
                void* /*user*/) {
  const size_t n = n_alphas;
  if (y_len) *y_len = n;
  if (n == 0) return 0;
  if (n_betas + 1 < n || y_cap < n) {
    put_err(err_msg, err_cap, "inconsistent tridiagonal sizes");
    return 1;
  }
  // dl (sub) = du (super) = betas, d = alphas, rhs = e_1. dgtsv, NRHS = 1.
  std::vector<double> dl(betas, betas + (n - 1)), d(alphas, alphas + n), du(betas, betas + (n - 1)),
      du2(n > 2 ? n - 2 : 0, 0.0), b(n, 0.0);
  b[0] = 1.0;
  for (size_t i = 0; i + 1 < n; ++i) {
    if (std::fabs(d[i]) >= std::fabs(dl[i])) {
      // no row interchange (a zero pivot here means both are zero: singular, keep going -> inf/nan)
      const double fact = dl[i] / d[i];
      d[i + 1] = d[i + 1] - fact * du[i];
      b[i + 1] = b[i + 1] - fact * b[i];
      if (i + 2 < n) du2[i] = 0.0;
    } else {
      // interchange rows i and i+1
      const double fact = d[i] / dl[i];
      d[i] = dl[i];
      const double temp = d[i + 1];
      d[i + 1] = du[i] - fact * temp;
      if (i + 2 < n) {
        du2[i] = du[i + 1];
        du[i + 1] = -fact * du2[i];
      }
      du[i] = temp;
      const double tb = b[i];
      b[i] = b[i + 1];
      b[i + 1] = tb - fact * b[i + 1];
    }
  }
  // back substitution with U = (d, du, du2)
  b[n - 1] = b[n - 1] / d[n - 1];
  if (n > 1) b[n - 2] = (b[n - 2] - du[n - 2] * b[n - 1]) / d[n - 2];
  for (size_t ii = n >= 3 ? n - 2 : 0; ii-- > 0;) {
    b[ii] = (b[ii] - du[ii] * b[ii + 1] - du2[ii] * b[ii + 2]) / d[ii];
  }
  std::memcpy(y_out, b.data(), n * sizeof(double));
  return 0;
}

int tpl_ftk_sq(const double* alphas, size_t n_alphas, const double* betas, size_t n_betas,
               double* y_out, size_t y_cap, size_t* y_len, char* err_msg, size_t err_cap,
               void* /*user*/) {
  const size_t n = n_alphas;
  if (y_len) *y_len = n;
  if (n == 0) return 0;
  if (n_betas + 1 < n || y_cap < n) {
    put_err(err_msg, err_cap, "inconsistent tridiagonal sizes");
    return 1;
  }
  // (T^2)[:, 0] = T (T e_1), T e_1 = (alpha_1, beta_1, 0, ...)
  for (size_t i = 0; i < n; ++i) y_out[i] = 0.0;
  const double a1 = alphas[0];
  const double b1 = n > 1 ? betas[0] : 0.0;
  y_out[0] = a1 * a1 + b1 * b1;
  if (n > 1) y_out[1] = b1 * a1 + alphas[1] * b1;
  if (n > 2) y_out[2] = betas[1] * b1;
  return 0;
}

int tpl_ftk_exp(const double* alphas, size_t n_alphas, const double* betas, size_t n_betas,
                double* y_out, size_t y_cap, size_t* y_len, char* err_msg, size_t err_cap,
                void* /*user*/) {
  const size_t n = n_alphas;
  if (y_len) *y_len = n;
  if (n == 0) return 0;
  if (n_betas + 1 < n || y_cap < n) {
    put_err(err_msg, err_cap, "inconsistent tridiagonal sizes");
    return 1;
  }
  // The converged off-diagonals and the first-row entries of converged eigenvectors
  // decay into the subnormal range, where every x86 operation costs ~100 cycles (73 ns
  // per rotation at k = 200); subnormals are flushed to zero for this solve only (their
  // contribution to y' is below 1e-300 relative) and the caller's mode is restored.
#if defined(__x86_64__)
  struct FtzGuard {
    unsigned int saved = _mm_getcsr();
    FtzGuard() { _mm_setcsr(saved | 0x8040); }  // FTZ | DAZ
    ~FtzGuard() { _mm_setcsr(saved); }
  } ftz;
#endif
  // Implicit QL with Wilkinson-type shifts (tql2 scheme), O(k^2): instead of
  // accumulating the eigenvector matrix Q = R_1 R_2 ... R_m (O(k) work per rotation), keep
  // only its first row q0 (u = Q^T e_1) and the rotations themselves; then
  // y' = Q exp(Lambda) Q^T e_1 = R_1 (R_2 (... (R_m w))), w_i = exp(lambda_i) q0_i.
  std::vector<double> d(alphas, alphas + n), e(n, 0.0), q0(n, 0.0);
  struct Rot {
    size_t i;
    double c, s;
  };
  // kept per thread across calls: a fresh multi-MB buffer per solve costs more in page
  // faults than the QL sweep itself
  static thread_local std::vector<Rot> rots;
  rots.clear();
  for (size_t i = 0; i + 1 < n; ++i) e[i] = betas[i];
  q0[0] = 1.0;
  const double eps = 2.220446049250313e-16;
  for (size_t l = 0; l < n; ++l) {
    int iter = 0;
    for (;;) {
      size_t m = l;
      for (; m + 1 < n; ++m) {
        const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
        if (std::fabs(e[m]) <= eps * dd) break;
      }
      if (m == l) break;
      if (++iter > 300) {
        put_err(err_msg, err_cap,
                tpl::msg_evd("NoConvergence").substr(0, std::string::npos));
        return 2;
      }
      double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
      double r = hyp(g, 1.0);
      g = d[m] - d[l] + e[l] / (g + (g >= 0.0 ? std::fabs(r) : -std::fabs(r)));
      double s = 1.0, c = 1.0, p = 0.0;
      size_t i = m;
      bool early = false;
      while (i-- > l) {
        double f = s * e[i];
        const double bb = c * e[i];
        r = hyp(f, g);
        e[i + 1] = r;
        if (r == 0.0) {
          d[i + 1] -= p;
          e[m] = 0.0;
          early = true;
          break;
        }
        s = f / r;
        c = g / r;
        g = d[i + 1] - p;
        r = (d[i] - g) * s + 2.0 * c * bb;
        p = s * r;
        d[i + 1] = g + p;
        g = c * r - bb;
        // Q <- Q R on columns (i, i+1): only row 0 is kept, the rotation is recorded
        f = q0[i + 1];
        q0[i + 1] = s * q0[i] + c * f;
        q0[i] = c * q0[i] - s * f;
        rots.push_back(Rot{i, c, s});
      }
      if (early) continue;
      d[l] -= p;
      e[l] = g;
      e[m] = 0.0;
    }
  }
  for (size_t i = 0; i < n; ++i) y_out[i] = std::exp(d[i]) * q0[i];
  for (size_t t = rots.size(); t-- > 0;) {  // y' = R_1 (... (R_m w))
    const Rot& R = rots[t];
    const double a = y_out[R.i], b = y_out[R.i + 1];
    y_out[R.i] = R.c * a + R.s * b;
    y_out[R.i + 1] = -R.s * a + R.c * b;
  }
  return 0;
}

} // extern "C"
