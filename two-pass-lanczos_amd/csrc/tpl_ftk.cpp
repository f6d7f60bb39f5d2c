// tpl_ftk.cpp — built-in f(T_k) e_1 solvers for the projected tridiagonal problem.
//
// They replace the harness closures of the reference:
//   inv: sparse LU of T_k (src/bin/tradeoff.rs:97-132,245-258; src/bin/stability.rs:161-170)
//        or dense partial-pivot LU (tests/correctness.rs:171-179) -> here: tridiagonal
//        Gaussian elimination with partial pivoting (the LAPACK dgtsv scheme), O(k).
//   exp: dense self-adjoint EVD, y' = Q exp(Lambda) Q^T e_1 (src/bin/stability.rs:175-193)
//        -> here: implicit-shift QL on the tridiagonal T_k with eigenvector accumulation.
//   sq : y' = T_k^2 e_1 (tests/correctness.rs:287-299).
// All three are O(k) or O(k^3) host work on at most 2k doubles: negligible next to
// the 2k-1 device SpMVs of a solve.
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "tpl_internal.h"

namespace {

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
  // Implicit QL with Wilkinson-type shifts (tql2 scheme). z is column-major n x n,
  // column i = eigenvector i.
  std::vector<double> d(alphas, alphas + n), e(n, 0.0), z(n * n, 0.0);
  for (size_t i = 0; i + 1 < n; ++i) e[i] = betas[i];
  for (size_t i = 0; i < n; ++i) z[i * n + i] = 1.0;
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
      double r = std::hypot(g, 1.0);
      g = d[m] - d[l] + e[l] / (g + (g >= 0.0 ? std::fabs(r) : -std::fabs(r)));
      double s = 1.0, c = 1.0, p = 0.0;
      size_t i = m;
      bool early = false;
      while (i-- > l) {
        double f = s * e[i];
        const double bb = c * e[i];
        r = std::hypot(f, g);
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
        double* zi = &z[i * n];
        double* zi1 = &z[(i + 1) * n];
        for (size_t kk = 0; kk < n; ++kk) {
          f = zi1[kk];
          zi1[kk] = s * zi[kk] + c * f;
          zi[kk] = c * zi[kk] - s * f;
        }
      }
      if (early) continue;
      d[l] -= p;
      e[l] = g;
      e[m] = 0.0;
    }
  }
  // y'_r = sum_i Q[r,i] exp(lambda_i) Q[0,i]
  for (size_t r = 0; r < n; ++r) y_out[r] = 0.0;
  for (size_t i = 0; i < n; ++i) {
    const double* q = &z[i * n];
    const double w = std::exp(d[i]) * q[0];
    for (size_t r = 0; r < n; ++r) y_out[r] += q[r] * w;
  }
  return 0;
}

} // extern "C"
