// The reference's own tests, restated against the C++ host API (include/tpl.hpp):
//   src/error.rs:70-127              error Display strings          (--cpu: no device needed)
//   src/algorithms/mod.rs:384-428    recurrence step, breakdown, zero b
//   src/algorithms/mod.rs:433-621    property tests on a KKT instance (k = 30, TOLERANCE 5e-9):
//                                    decomposition consistency, Lanczos relation,
//                                    orthonormality, reconstruction stability
//   tests/correctness.rs             f(A)b vs the analytic solution on diag(1..100),
//                                    b = StdRng::seed_from_u64(42), k = 30: inv / exp (1e-3),
//                                    z^2 (1e-12), one-pass and two-pass
// plus the solver-closure error paths of src/solvers.rs:75-85 (SolverError, ParameterMismatch).
// Usage: cpp_api_test --cpu | cpp_api_test --gpu KKT.dmx KKT.qfc
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "tpl.hpp"

static int g_fail = 0;
#define CHECK(cond, ...)                      \
  do {                                        \
    if (!(cond)) {                            \
      std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
      std::printf(__VA_ARGS__);               \
      std::printf("\n");                      \
      ++g_fail;                               \
    }                                         \
  } while (0)

using tpl::LanczosError;
using tpl::LanczosErrorKind;
using tpl::Mat;
using Vec = std::vector<double>;

// ---- rand 0.9 StdRng (ChaCha12), seed_from_u64, f64 = (u64 >> 11) * 2^-53 (the recipe of
// SURVEY.md §8(c); test infrastructure, checked below against the reference's values) ----
struct StdRng {
  uint32_t key[8];
  uint64_t counter = 0;
  uint32_t buf[64];
  int idx = 64;
  explicit StdRng(uint64_t s) {
    uint8_t bytes[32];
    for (int i = 0; i < 8; ++i) {
      s = s * 6364136223846793005ULL + 11634580027462260723ULL;
      const uint32_t xs = (uint32_t)(((s >> 18) ^ s) >> 27);
      const uint32_t rot = (uint32_t)(s >> 59);
      const uint32_t v = (xs >> rot) | (xs << ((32 - rot) & 31));
      std::memcpy(bytes + 4 * i, &v, 4);
    }
    std::memcpy(key, bytes, 32);
  }
  static uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
  void block(uint64_t ctr, uint32_t* out) {
    uint32_t st[16] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574, key[0], key[1], key[2], key[3],
                       key[4], key[5], key[6], key[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), 0, 0};
    uint32_t x[16];
    std::memcpy(x, st, sizeof x);
    auto qr = [&](int a, int b, int c, int d) {
      x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16);
      x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12);
      x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);
      x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
    };
    for (int r = 0; r < 6; ++r) {  // 12 rounds
      qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
      qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + st[i];
  }
  void refill() {
    for (int b = 0; b < 4; ++b) block(counter + b, buf + 16 * b);
    counter += 4;
    idx = 0;
  }
  uint64_t next_u64() {  // BlockRng::next_u64 with its boundary handling
    if (idx < 63) {
      const uint64_t v = ((uint64_t)buf[idx + 1] << 32) | buf[idx];
      idx += 2;
      return v;
    }
    if (idx == 63) {
      const uint64_t lo = buf[63];
      refill();
      const uint64_t v = ((uint64_t)buf[0] << 32) | lo;
      idx = 1;
      return v;
    }
    refill();
    const uint64_t v = ((uint64_t)buf[1] << 32) | buf[0];
    idx = 2;
    return v;
  }
  double random() { return (double)(next_u64() >> 11) * (1.0 / 9007199254740992.0); }
};
static Vec std_rng_vector(size_t n) {
  StdRng r(42);
  Vec b(n);
  for (auto& v : b) v = r.random();
  return b;
}

static double norm(const Vec& v) {
  double s = 0;
  for (double x : v) s += x * x;
  return std::sqrt(s);
}

// ---- src/error.rs:70-127 -------------------------------------------------------------------
static void error_message_tests() {
  CHECK(std::string(LanczosError::breakdown(42).what()) ==
            "Lanczos iteration breakdown at step 42: Beta coefficient is zero. The Krylov subspace is invariant.",
        "breakdown message");
  CHECK(std::string(LanczosError::dimension_mismatch(100, 99).what()) ==
            "Dimension mismatch: operator has 100 columns but vector has 99 rows.",
        "dimension mismatch message");
  CHECK(std::string(LanczosError::parameter_mismatch("y_k", 10, 9).what()) ==
            "Parameter mismatch: `y_k` expects size 10, but got 9.",
        "parameter mismatch message");
  CHECK(std::string(LanczosError::input_error("The initial vector `b` must not be a zero vector.").what()) ==
            "Invalid input parameter: The initial vector `b` must not be a zero vector.",
        "input error message");
  CHECK(std::string(LanczosError::evd_error("NoConvergence").what()) ==
            "A numerical error occurred during the eigendecomposition of T_k: NoConvergence",
        "evd error message");
  CHECK(std::string(LanczosError::solver_error("Custom solver failed").what()) ==
            "The user-provided f(T_k) solver failed: Custom solver failed",
        "solver error message");
  CHECK(LanczosError::parameter_mismatch("y_k", 10, 9) == LanczosError::parameter_mismatch("y_k", 10, 9) &&
            !(LanczosError::breakdown(1) == LanczosError::breakdown(2)),
        "PartialEq");
  // the StdRng restatement reproduces the reference's b
  const Vec b = std_rng_vector(4);
  const double want[4] = {0.52655741, 0.54272521, 0.6364651, 0.40590176};
  for (int i = 0; i < 4; ++i) CHECK(std::fabs(b[i] - want[i]) < 5e-9, "StdRng b[%d] = %.9f", i, b[i]);
}

// dense helpers for the small test matrices
static tpl::HipCsrOp dense_op(const tpl::Context& ctx, const std::vector<Vec>& a) {
  const int64_t n = (int64_t)a.size();
  std::vector<int64_t> rp(1, 0);
  std::vector<int32_t> ci;
  Vec v;
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t j = 0; j < n; ++j)
      if (a[i][j] != 0.0) {
        ci.push_back((int32_t)j);
        v.push_back(a[i][j]);
      }
    rp.push_back((int64_t)ci.size());
  }
  return tpl::HipCsrOp(ctx, n, rp, ci, v);
}

// ---- src/algorithms/mod.rs:384-428 ---------------------------------------------------------
static void unit_tests(const tpl::Context& ctx) {
  {  // test_recurrence_step_correctness: v_1 = e_1 on the 4x4 [2,-1] stencil: alpha 2, beta 1
    auto op = dense_op(ctx, {{2, -1, 0, 0}, {-1, 2, -1, 0}, {0, -1, 2, -1}, {0, 0, -1, 2}});
    const auto out = tpl::algorithms::lanczos_standard(op, {1, 0, 0, 0}, 2);
    CHECK(out.decomposition.steps_taken == 2, "steps %zu", out.decomposition.steps_taken);
    CHECK(std::fabs(out.decomposition.alphas[0] - 2.0) < 1e-15, "alpha %.17g", out.decomposition.alphas[0]);
    CHECK(std::fabs(out.decomposition.betas[0] - 1.0) < 1e-15, "beta %.17g", out.decomposition.betas[0]);
  }
  {  // test_breakdown_scenario: diag(2, 3), b = e_1, k = 2 -> steps_taken 1
    auto op = dense_op(ctx, {{2, 0}, {0, 3}});
    const auto out = tpl::algorithms::lanczos_standard(op, {1, 0}, 2);
    CHECK(out.decomposition.steps_taken == 1, "breakdown steps %zu", out.decomposition.steps_taken);
    CHECK(out.decomposition.betas.empty() && out.v_k.cols == 1, "breakdown shapes");
  }
  {  // test_zero_vector_input_returns_error (+ the exact kind and text)
    auto op = dense_op(ctx, {{1, 0}, {0, 1}});
    bool raised = false;
    try {
      tpl::algorithms::lanczos_standard(op, {0, 0}, 2);
    } catch (const LanczosError& e) {
      raised = e.kind() == LanczosErrorKind::InputError &&
               std::string(e.what()) == "Invalid input parameter: Input vector `b` must not be a zero vector.";
    }
    CHECK(raised, "zero b must be an InputError");
  }
}

// ---- src/algorithms/mod.rs:433-621, on a KKT instance ---------------------------------------
static void property_tests(const tpl::Context& ctx, const char* dmx, const char* qfc) {
  const double TOL = 5e-9;
  const size_t k = 30;
  const auto sys = tpl::load_kkt_system(dmx, qfc);
  const size_t n = (size_t)sys.n;
  tpl::HipCsrOp op(ctx, sys.n, sys.row_ptr, sys.col_idx, sys.vals);
  const Vec b = std_rng_vector(n);
  const auto std_out = tpl::algorithms::lanczos_standard(op, b, k);
  const auto po = tpl::algorithms::lanczos_pass_one(op, b, k);
  // decomposition consistency
  CHECK(std_out.decomposition.steps_taken == po.steps_taken, "steps_taken mismatch");
  for (size_t i = 0; i < po.alphas.size(); ++i)
    CHECK(std::fabs(std_out.decomposition.alphas[i] - po.alphas[i]) < TOL, "alpha %zu", i);
  for (size_t i = 0; i < po.betas.size(); ++i)
    CHECK(std::fabs(std_out.decomposition.betas[i] - po.betas[i]) < TOL, "beta %zu", i);
  const size_t s = std_out.decomposition.steps_taken;
  const Mat& V = std_out.v_k;
  // orthonormality: ||I - V^T V||_F
  double oe = 0.0;
  for (size_t i = 0; i < s; ++i)
    for (size_t j = 0; j < s; ++j) {
      double d = 0.0;
      for (size_t r = 0; r < n; ++r) d += V(r, i) * V(r, j);
      const double e = (i == j ? 1.0 : 0.0) - d;
      oe += e * e;
    }
  CHECK(std::sqrt(oe) < TOL, "orthonormality %.3e", std::sqrt(oe));
  // Lanczos relation: A V_k - V_k T_k = beta_k v_{k+1} e_k^T
  const auto out1 = tpl::algorithms::lanczos_standard(op, b, k + 1);
  CHECK(s == k && out1.decomposition.steps_taken == k + 1, "relation needs k + 1 steps");
  if (s == k && out1.decomposition.steps_taken == k + 1) {
    const double beta_k = out1.decomposition.betas[k - 1];
    double diff = 0.0;
    for (size_t c = 0; c < k; ++c) {
      Vec vc(n);
      for (size_t r = 0; r < n; ++r) vc[r] = V(r, c);
      const Vec av = op.apply(vc);
      for (size_t r = 0; r < n; ++r) {
        double vt = V(r, c) * std_out.decomposition.alphas[c];
        if (c > 0) vt += V(r, c - 1) * std_out.decomposition.betas[c - 1];
        if (c + 1 < k) vt += V(r, c + 1) * std_out.decomposition.betas[c];
        const double want = c + 1 == k ? beta_k * out1.v_k(r, k) : 0.0;
        const double e = av[r] - vt - want;
        diff += e * e;
      }
    }
    CHECK(std::sqrt(diff) < TOL, "Lanczos relation %.3e", std::sqrt(diff));
  }
  // reconstruction stability: V_k == V'_k (squared norm of the drift)
  Vec y(s);
  for (size_t i = 0; i < s; ++i) y[i] = 0.1 * (double)(i + 1);
  const auto p2 = tpl::algorithms::lanczos_pass_two_with_basis(op, b, po, y);
  double drift = 0.0;
  for (size_t i = 0; i < V.data.size(); ++i) drift += (V.data[i] - p2.v_k.data[i]) * (V.data[i] - p2.v_k.data[i]);
  CHECK(drift < TOL, "basis drift %.3e", drift);
  CHECK(drift == 0.0, "basis drift %.3e (the engine regenerates V_k bit for bit)", drift);
}

// ---- the partitioned operator through one RCCL rank (tpl.hpp Dist / HipCsrOp::partitioned):
// the solvers take it unchanged; its rows cover A once and x agrees with one GPU's
static void partition_tests(const char* dmx, const char* qfc) {
  const auto sys = tpl::load_kkt_system(dmx, qfc);
  const size_t n = (size_t)sys.n, k = 30;
  auto dist = std::make_shared<tpl::Dist>(0, 0, 1, tpl::Dist::unique_id());
  tpl::Context ctx(0);
  tpl::HipCsrOp single(ctx, sys.n, sys.row_ptr, sys.col_idx, sys.vals);
  const Vec b = std_rng_vector(n);
  const Vec x1 = tpl::solvers::lanczos_two_pass(single, b, k, tpl::ftk::inv());
  for (auto how : {tpl::Partition::Auto, tpl::Partition::Halo}) {
    auto op = tpl::HipCsrOp::partitioned(dist, sys.n, sys.row_ptr, sys.col_idx, sys.vals, how);
    const auto rows = op.local_rows();
    CHECK(rows.size() == n, "one rank holds every row (%zu of %zu)", rows.size(), n);
    std::vector<int> seen(n, 0);
    for (int64_t r : rows) seen[(size_t)r]++;
    CHECK(std::all_of(seen.begin(), seen.end(), [](int c) { return c == 1; }), "rows cover A once");
    Vec bl(rows.size());
    for (size_t i = 0; i < rows.size(); ++i) bl[i] = b[(size_t)rows[i]];
    const Vec xl = tpl::solvers::lanczos_two_pass(op, bl, k, tpl::ftk::inv());
    double d = 0.0, nx = 0.0;
    for (size_t i = 0; i < rows.size(); ++i) {
      const double e = xl[i] - x1[(size_t)rows[i]];
      d += e * e;
      nx += x1[(size_t)rows[i]] * x1[(size_t)rows[i]];
    }
    CHECK(std::sqrt(d) <= 1e-10 * std::sqrt(nx), "partitioned x vs one GPU %.3e",
          std::sqrt(d / nx));
  }
}

// ---- tests/correctness.rs -----------------------------------------------------------------
static void correctness_tests(const tpl::Context& ctx) {
  const size_t n = 100, k = 30;
  std::vector<int64_t> rp(n + 1);
  std::vector<int32_t> ci(n);
  Vec v(n), eig(n);
  for (size_t i = 0; i < n; ++i) {
    rp[i + 1] = (int64_t)i + 1;
    ci[i] = (int32_t)i;
    v[i] = eig[i] = (double)(i + 1);
  }
  tpl::HipCsrOp a(ctx, (int64_t)n, rp, ci, v);
  const Vec b = std_rng_vector(n);
  struct Case {
    const char* name;
    tpl::FtkSolver f;
    double (*g)(double);
    double tol;
  };
  const Case cases[] = {
      {"linear solve", tpl::ftk::inv(), [](double z) { return 1.0 / z; }, 1e-3},
      {"matrix exponential", tpl::ftk::exp(), [](double z) { return std::exp(z); }, 1e-3},
      {"matrix square", tpl::ftk::sq(), [](double z) { return z * z; }, 1e-12},
  };
  for (const Case& c : cases) {
    Vec xt(n);
    for (size_t i = 0; i < n; ++i) xt[i] = c.g(eig[i]) * b[i];
    for (int two = 0; two < 2; ++two) {
      const Vec x = two ? tpl::solvers::lanczos_two_pass(a, b, k, c.f) : tpl::solvers::lanczos(a, b, k, c.f);
      Vec d(n);
      for (size_t i = 0; i < n; ++i) d[i] = x[i] - xt[i];
      const double rel = norm(d) / norm(xt);
      CHECK(rel < c.tol, "%s %s error too high: %.3e", two ? "Two-pass" : "One-pass", c.name, rel);
    }
  }
  // LanczosCallback (src/algorithms/mod.rs:82-86): a stop at step 5 returns exactly the
  // 5-step result; the view carries T_5; an exception in the callback reaches the caller
  {
    const auto full = tpl::algorithms::lanczos_standard(a, b, k);
    size_t seen = 0;
    bool view_ok = true;
    const tpl::LanczosCallback stop5 = [&](size_t kk, const double* v, int64_t nn,
                                           const tpl::TridiagonalSystemView& t) {
      seen = kk;
      view_ok = view_ok && v != nullptr && nn == (int64_t)n && t.steps_taken == kk &&
                t.n_alphas == kk && t.n_betas == kk - 1 && t.alphas[kk - 1] == full.decomposition.alphas[kk - 1];
      return kk < 5;
    };
    const auto cut = tpl::algorithms::lanczos_standard(a, b, k, &stop5);
    CHECK(seen == 5 && view_ok && cut.decomposition.steps_taken == 5, "callback stop at 5 (seen %zu)", seen);
    bool same = cut.v_k.cols == 5;
    for (size_t i = 0; same && i < 5; ++i) same = cut.decomposition.alphas[i] == full.decomposition.alphas[i];
    for (size_t i = 0; same && i < n * 5; ++i) same = cut.v_k.data[i] == full.v_k.data[i];
    CHECK(same, "a stopped run is the truncated full run, bit for bit");
    const tpl::LanczosCallback boom = [](size_t kk, const double*, int64_t, const tpl::TridiagonalSystemView&) -> bool {
      if (kk == 3) throw std::runtime_error("callback failed");
      return true;
    };
    bool rethrown = false;
    try {
      tpl::algorithms::lanczos_standard(a, b, k, &boom);
    } catch (const std::runtime_error& e) {
      rethrown = std::string(e.what()) == "callback failed";
    }
    CHECK(rethrown, "an exception in the callback reaches the caller");
  }
  // a C++ closure (not a built-in: called on the host between the passes) gives the same x
  const tpl::FtkSolver user_sq = [](const Vec& al, const Vec& be) {
    const size_t s = al.size();
    Mat y(s, 1);  // T^2 e_1 = T (T e_1)
    Vec t1(s, 0.0);
    t1[0] = al[0];
    if (s > 1) t1[1] = be[0];
    for (size_t i = 0; i < s; ++i) {
      double acc = al[i] * t1[i];
      if (i > 0) acc += be[i - 1] * t1[i - 1];
      if (i + 1 < s) acc += be[i] * t1[i + 1];
      y(i, 0) = acc;
    }
    return y;
  };
  const Vec xs = tpl::solvers::lanczos_two_pass(a, b, k, user_sq);
  const Vec xb = tpl::solvers::lanczos_two_pass(a, b, k, tpl::ftk::sq());
  double dd = 0.0;
  for (size_t i = 0; i < n; ++i) dd = std::fmax(dd, std::fabs(xs[i] - xb[i]));
  CHECK(dd <= 1e-12 * norm(xb), "closure vs built-in sq: %.3e", dd);
  // src/solvers.rs:75 — Err(e) from the closure is SolverError(e.to_string())
  bool ok = false;
  try {
    tpl::solvers::lanczos_two_pass(a, b, k, [](const Vec&, const Vec&) -> Mat {
      throw std::runtime_error("Custom solver failed");
    });
  } catch (const LanczosError& e) {
    ok = e.kind() == LanczosErrorKind::SolverError &&
         std::string(e.what()) == "The user-provided f(T_k) solver failed: Custom solver failed";
  }
  CHECK(ok, "throwing closure -> SolverError");
  // src/solvers.rs:78-85 — a y' of the wrong length or width is ParameterMismatch
  for (int wide = 0; wide < 2; ++wide) {
    ok = false;
    try {
      tpl::solvers::lanczos(a, b, k, [wide](const Vec& al, const Vec&) {
        return wide ? Mat(al.size(), 2) : Mat(al.size() - 1, 1);
      });
    } catch (const LanczosError& e) {
      ok = e.kind() == LanczosErrorKind::ParameterMismatch && e.param_name() == "y_k_prime" &&
           e.expected() == k && e.actual() == (wide ? k : k - 1);
    }
    CHECK(ok, "y' of the wrong shape (%s) -> ParameterMismatch", wide ? "2 columns" : "k - 1 rows");
  }
  // DimensionMismatch before any device work
  ok = false;
  try {
    tpl::solvers::lanczos_two_pass(a, Vec(n - 1, 1.0), k, tpl::ftk::inv());
  } catch (const LanczosError& e) {
    ok = e.kind() == LanczosErrorKind::DimensionMismatch && e.operator_cols() == n && e.vector_rows() == n - 1;
  }
  CHECK(ok, "b of the wrong length -> DimensionMismatch");
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "--gpu") == 0;
  error_message_tests();
  if (gpu) {
    if (argc < 4) {
      std::printf("usage: cpp_api_test --gpu KKT.dmx KKT.qfc\n");
      return 2;
    }
    try {
      tpl::Context ctx(0);
      unit_tests(ctx);
      correctness_tests(ctx);
      property_tests(ctx, argv[2], argv[3]);
      partition_tests(argv[2], argv[3]);
    } catch (const std::exception& e) {
      std::printf("FAIL uncaught: %s\n", e.what());
      ++g_fail;
    }
  }
  std::printf("%s (%d failures)\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
