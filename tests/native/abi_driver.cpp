// abi_driver.cpp — C++ test driver of the C ABI (include/tpl.h), linked against the
// built libtpl_amd.so exactly as a C/C++/Rust caller would link it ("The
// C ABI is exercised by a C++ test driver and Python ctypes").
//
//   abi_driver <netgen-5000-3.dmx> <qfc> [--gpu]
//
// CPU part (no GPU needed): version string, device count, the .dmx/.qfc loader on the
// 5k fixture (sizes, symmetry, the qfc D = empty quirk) and its error texts, the
// built-in f(T_k) solvers against closed forms, the synthetic generator, the partition
// helper. --gpu: a two-pass solve through a host callback f and through the built-in
// inv (one device graph) — bitwise equal — and the one-pass solver within 1e-10.
// Exit status 0 = all checks passed; every failure prints one line.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "tpl.h"

static int g_fail = 0;
#define CHECK(cond, ...)                                  \
  do {                                                    \
    if (!(cond)) {                                        \
      std::printf("FAIL %s:%d: ", __FILE__, __LINE__);    \
      std::printf(__VA_ARGS__);                           \
      std::printf("\n");                                  \
      ++g_fail;                                           \
    }                                                     \
  } while (0)

static double entry(const tpl_csr_host& A, int64_t i, int64_t j) {
  for (int64_t q = A.row_ptr[i]; q < A.row_ptr[i + 1]; ++q)
    if (A.col_idx[q] == j) return A.vals[q];
  return 0.0;
}

// tpl_last_error_detail: status, message and the variant's fields (src/error.rs:20-58)
static tpl_error_detail detail() {
  tpl_error_detail d{};
  if (tpl_last_error_detail(&d) != TPL_OK) std::printf("FAIL: tpl_last_error_detail\n"), ++g_fail;
  return d;
}

// host f(T_k) returning one entry too few (-> ParameterMismatch y_k_prime), or an error
static int short_f(const double*, size_t na, const double*, size_t, double* y, size_t, size_t* len,
                   char*, size_t, void*) {
  for (size_t i = 0; i + 1 < na; ++i) y[i] = 0.0;
  *len = na - 1;
  return 0;
}
static int failing_f(const double*, size_t, const double*, size_t, double*, size_t, size_t*,
                     char* err, size_t ecap, void*) {
  std::snprintf(err, ecap, "custom solver failed");
  return 1;
}

// host f(T_k) callback that forwards to the built-in inv (so the solve takes the host path)
static int host_inv(const double* a, size_t na, const double* b, size_t nb, double* y, size_t cap,
                    size_t* len, char* err, size_t ecap, void* user) {
  ++*static_cast<int*>(user);
  return tpl_ftk_inv(a, na, b, nb, y, cap, len, err, ecap, nullptr);
}

static void cpu_checks(const char* dmx, const char* qfc, tpl_csr_host& A) {
  CHECK(std::strstr(tpl_version(), "gfx950") != nullptr, "version %s", tpl_version());
  CHECK(tpl_device_count() >= 0, "device count");
  // loader (src/utils/data_loader.rs:211-259)
  tpl_status st = tpl_load_kkt_system(dmx, qfc, &A);
  CHECK(st == TPL_OK, "load: %d %s", (int)st, tpl_last_error());
  if (st != TPL_OK) return;
  CHECK(A.n == 5115 && A.nnz == 20000, "n %lld nnz %lld", (long long)A.n, (long long)A.nnz);
  CHECK(A.num_nodes == 115 && A.num_arcs == 5000, "nodes/arcs");
  bool sym = true, sorted = true;
  for (int64_t i = 0; i < A.n; ++i)
    for (int64_t q = A.row_ptr[i]; q < A.row_ptr[i + 1]; ++q) {
      if (q > A.row_ptr[i] && A.col_idx[q] <= A.col_idx[q - 1]) sorted = false;
      if (entry(A, A.col_idx[q], i) != A.vals[q]) sym = false;
    }
  CHECK(sym && sorted, "symmetric %d sorted %d", (int)sym, (int)sorted);
  CHECK(entry(A, 0, 0) == 0.0, "D must be empty with a 3-line qfc");
  tpl_csr_host B{};
  st = tpl_load_kkt_system("/nonexistent.dmx", qfc, &B);
  CHECK(st == TPL_ERR_DATA_LOADER, "missing file status %d", (int)st);
  CHECK(std::string(tpl_last_error()) == "I/O error: No such file or directory (os error 2)",
        "message '%s'", tpl_last_error());
  tpl_error_detail d = detail();
  CHECK(d.status == TPL_ERR_DATA_LOADER && std::string(d.message) == tpl_last_error() &&
            std::string(d.param_name).empty(), "loader detail %d", (int)d.status);
  CHECK(tpl_last_error_detail(nullptr) == TPL_ERR_INVALID_ARGUMENT, "detail(NULL)");
  // malformed CSR on the host-only locality order (decreasing row_ptr, column out of
  // range, NULL columns): rejected before any indexing
  {
    const int64_t rp_bad[3] = {0, 2, 1};
    const int64_t rp_ok[3] = {0, 1, 2};
    const int32_t col_ok[2] = {1, 0}, col_oob[2] = {1, 7};
    int32_t perm[2], applied = -1;
    CHECK(tpl_locality_order(2, rp_bad, col_ok, 0, 0, perm, &applied) == TPL_ERR_INVALID_ARGUMENT,
          "locality_order: decreasing row_ptr");
    CHECK(tpl_locality_order(2, rp_ok, col_oob, 0, 0, perm, &applied) == TPL_ERR_INVALID_ARGUMENT,
          "locality_order: column out of range");
    CHECK(tpl_locality_order(2, rp_ok, nullptr, 0, 0, perm, &applied) == TPL_ERR_INVALID_ARGUMENT,
          "locality_order: NULL columns");
    CHECK(detail().status == TPL_ERR_INVALID_ARGUMENT, "invalid-argument detail");
    CHECK(tpl_locality_order(2, rp_ok, col_ok, 0, 0, perm, &applied) == TPL_OK, "locality_order ok");
    d = detail();
    CHECK(d.status == TPL_OK && std::string(d.message).empty(), "detail after success");
  }
  // built-in f(T_k) (include/tpl.h): T = [[2,1],[1,2]]
  const double al[2] = {2.0, 2.0}, be[1] = {1.0};
  double y[2];
  size_t len = 0;
  char err[128];
  CHECK(tpl_ftk_inv(al, 2, be, 1, y, 2, &len, err, sizeof err, nullptr) == 0 && len == 2, "inv");
  CHECK(std::fabs(y[0] - 2.0 / 3.0) < 1e-15 && std::fabs(y[1] + 1.0 / 3.0) < 1e-15, "inv y");
  CHECK(tpl_ftk_sq(al, 2, be, 1, y, 2, &len, err, sizeof err, nullptr) == 0, "sq");
  CHECK(y[0] == 5.0 && y[1] == 4.0, "sq y %g %g", y[0], y[1]);
  CHECK(tpl_ftk_exp(al, 2, be, 1, y, 2, &len, err, sizeof err, nullptr) == 0, "exp");
  // exp(T) e1 = (e^3 + e) / 2, (e^3 - e) / 2
  CHECK(std::fabs(y[0] - (std::exp(3.0) + std::exp(1.0)) / 2) < 1e-13 &&
            std::fabs(y[1] - (std::exp(3.0) - std::exp(1.0)) / 2) < 1e-13,
        "exp y %.17g %.17g", y[0], y[1]);
  CHECK(tpl_ftk_inv(al, 2, be, 0, y, 2, &len, err, sizeof err, nullptr) != 0, "size check");
  // synthetic generator (configs[4]'s family) and the partition helper
  tpl_csr_host G{};
  st = tpl_generate_kkt(20000, 231, 42, &G);
  CHECK(st == TPL_OK && G.num_arcs == 20000 && G.nnz == 80000, "generate %d", (int)st);
  int64_t starts[5];
  st = tpl_dist_partition(G.n, G.row_ptr, 4, starts);
  CHECK(st == TPL_OK && starts[0] == 0 && starts[4] == G.n, "partition");
  for (int r = 0; r < 4; ++r) CHECK(starts[r] < starts[r + 1], "partition order");
  tpl_csr_host_free(&G);
}

static void gpu_checks(tpl_csr_host& A) {
  if (tpl_device_count() < 1) {
    std::printf("FAIL: --gpu but no device\n");
    ++g_fail;
    return;
  }
  tpl_ctx_t ctx = nullptr;
  tpl_op_t op = nullptr;
  CHECK(tpl_ctx_create(0, &ctx) == TPL_OK, "ctx %s", tpl_last_error());
  CHECK(tpl_op_create_csr(ctx, A.n, A.nnz, A.row_ptr, A.col_idx, A.vals, &op) == TPL_OK,
        "op %s", tpl_last_error());
  if (!op) return;
  const int64_t n = A.n;
  std::vector<double> b(n, 0.0), x1(n), x2(n), x3(n);
  for (int64_t i = 0; i < n; ++i)  // b = A (1/sqrt(n)) 1  (src/bin/tradeoff.rs:235-236)
    for (int64_t q = A.row_ptr[i]; q < A.row_ptr[i + 1]; ++q) b[i] += A.vals[q] / std::sqrt((double)n);
  int calls = 0;
  CHECK(tpl_lanczos_two_pass(op, b.data(), n, 50, host_inv, &calls, x1.data(), TPL_MEM_HOST) == TPL_OK,
        "two-pass host f: %s", tpl_last_error());
  CHECK(calls == 1, "f called %d times", calls);
  CHECK(tpl_lanczos_two_pass(op, b.data(), n, 50, tpl_ftk_inv, nullptr, x2.data(), TPL_MEM_HOST) == TPL_OK,
        "two-pass device f: %s", tpl_last_error());
  CHECK(tpl_op_flags(op) & 32, "one-graph path not taken");
  CHECK(std::memcmp(x1.data(), x2.data(), n * sizeof(double)) == 0, "host f != device f");
  CHECK(tpl_lanczos(op, b.data(), n, 50, tpl_ftk_inv, nullptr, x3.data(), TPL_MEM_HOST) == TPL_OK,
        "one-pass: %s", tpl_last_error());
  double num = 0, den = 0;
  for (int64_t i = 0; i < n; ++i) {
    num += (x3[i] - x2[i]) * (x3[i] - x2[i]);
    den += x2[i] * x2[i];
  }
  CHECK(std::sqrt(num / den) < 1e-10, "one-pass vs two-pass %g", std::sqrt(num / den));
  uint64_t bytes = 0;
  CHECK(tpl_op_device_bytes(op, &bytes) == TPL_OK && bytes >= (uint64_t)(8 * n * 50), "device bytes %llu",
        (unsigned long long)bytes);
  // every LanczosErrorKind the engine raises, with its fields (tpl_last_error_detail)
  std::vector<double> z(n, 0.0);
  CHECK(tpl_lanczos_two_pass(op, z.data(), n, 5, tpl_ftk_inv, nullptr, x1.data(), TPL_MEM_HOST) ==
            TPL_ERR_INPUT, "zero b");
  tpl_error_detail d = detail();
  CHECK(d.status == TPL_ERR_INPUT &&
            std::string(d.inner) == "Input vector `b` must not be a zero vector." &&
            std::string(d.message) == "Invalid input parameter: " + std::string(d.inner),
        "InputError detail '%s'", d.inner);
  CHECK(tpl_lanczos_two_pass(op, b.data(), n - 1, 5, tpl_ftk_inv, nullptr, x1.data(), TPL_MEM_HOST) ==
            TPL_ERR_DIMENSION_MISMATCH, "dimension");
  d = detail();
  CHECK(d.status == TPL_ERR_DIMENSION_MISMATCH && d.operator_cols == (uint64_t)n &&
            d.vector_rows == (uint64_t)(n - 1), "DimensionMismatch detail %llu %llu",
        (unsigned long long)d.operator_cols, (unsigned long long)d.vector_rows);
  CHECK(tpl_lanczos_two_pass(op, b.data(), n, 20, short_f, nullptr, x1.data(), TPL_MEM_HOST) ==
            TPL_ERR_PARAMETER_MISMATCH, "y_k_prime mismatch");
  d = detail();
  CHECK(d.status == TPL_ERR_PARAMETER_MISMATCH && std::string(d.param_name) == "y_k_prime" &&
            d.expected == 20 && d.actual == 19 &&
            std::string(d.message) == "Parameter mismatch: `y_k_prime` expects size 20, but got 19.",
        "ParameterMismatch(y_k_prime) detail '%s' %llu %llu", d.param_name,
        (unsigned long long)d.expected, (unsigned long long)d.actual);
  CHECK(tpl_lanczos_two_pass(op, b.data(), n, 20, failing_f, nullptr, x1.data(), TPL_MEM_HOST) ==
            TPL_ERR_SOLVER, "solver error");
  d = detail();
  CHECK(d.status == TPL_ERR_SOLVER && std::string(d.inner) == "custom solver failed" &&
            std::string(d.message) == "The user-provided f(T_k) solver failed: custom solver failed",
        "SolverError detail '%s'", d.message);
  {
    double al[4] = {0, 0, 0, 0}, be[3] = {1, 1, 1}, yk[3] = {1, 0, 0};
    CHECK(tpl_lanczos_pass_two(op, b.data(), n, al, 4, be, 3, 4, 1.0, yk, 3, x1.data(), nullptr,
                               TPL_MEM_HOST) == TPL_ERR_PARAMETER_MISMATCH, "y_k mismatch");
    d = detail();
    CHECK(d.status == TPL_ERR_PARAMETER_MISMATCH && std::string(d.param_name) == "y_k" &&
              d.expected == 4 && d.actual == 3, "ParameterMismatch(y_k) detail");
  }
  tpl_op_destroy(op);
  tpl_ctx_destroy(ctx);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::printf("usage: abi_driver <dmx> <qfc> [--gpu]\n");
    return 2;
  }
  tpl_csr_host A{};
  cpu_checks(argv[1], argv[2], A);
  if (argc > 3 && std::strcmp(argv[3], "--gpu") == 0 && A.row_ptr) gpu_checks(A);
  tpl_csr_host_free(&A);
  std::printf("%s (%d failures)\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
