/*
 * tpl.hpp — header-only C++17 host API over the C ABI (tpl.h), mirroring the reference
 * crate's public surface for this path, so a compiled caller reads like the reference:
 *
 *   tpl::solvers::lanczos / lanczos_two_pass          src/solvers.rs:46-107, 133-175
 *   tpl::algorithms::lanczos_standard                 src/algorithms/lanczos.rs:55-156
 *   tpl::algorithms::lanczos_pass_one                 src/algorithms/lanczos_two_pass.rs:65-110
 *   tpl::algorithms::lanczos_pass_two[_with_basis]    src/algorithms/lanczos_two_pass.rs:128-166
 *   tpl::LanczosDecomposition / LanczosOutput /
 *     LanczosPassTwoOutput / TridiagonalSystemView    src/algorithms/mod.rs:57-135
 *   tpl::LanczosError (+ LanczosErrorKind)            src/error.rs:11-58
 *   tpl::HipCsrOp                                     faer LinOp<f64> on a sparse matrix
 *
 * Same argument meaning and error behaviour as the reference: a zero b is an InputError,
 * a failing f(T_k) closure a SolverError(its message), a y' of the wrong size a
 * ParameterMismatch { "y_k_prime", steps, rows }, breakdown truncates steps_taken. The
 * `stack` workspace argument has no counterpart (the operator owns its device workspace).
 * Vectors are host std::vector<double>; matrices are column-major (tpl::Mat), the layout
 * of faer's Mat<f64>. Errors of the engine that have no LanczosErrorKind (bad argument,
 * HIP failure, ...) are tpl::EngineError. Not thread-safe per operator (the reference is
 * single-threaded, Par::Seq).
 */
#ifndef TPL_HPP_
#define TPL_HPP_

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "tpl.h"

namespace tpl {

// ---- errors: src/error.rs:11-58 ------------------------------------------------------
enum class LanczosErrorKind { Breakdown, DimensionMismatch, InputError, ParameterMismatch, EvdError, SolverError };

class LanczosError : public std::exception {
 public:
  static LanczosError breakdown(size_t k) {
    LanczosError e(LanczosErrorKind::Breakdown);
    e.breakdown_step_ = k;
    e.msg_ = "Lanczos iteration breakdown at step " + std::to_string(k) +
             ": Beta coefficient is zero. The Krylov subspace is invariant.";
    return e;
  }
  static LanczosError dimension_mismatch(size_t operator_cols, size_t vector_rows) {
    LanczosError e(LanczosErrorKind::DimensionMismatch);
    e.operator_cols_ = operator_cols;
    e.vector_rows_ = vector_rows;
    e.msg_ = "Dimension mismatch: operator has " + std::to_string(operator_cols) +
             " columns but vector has " + std::to_string(vector_rows) + " rows.";
    return e;
  }
  static LanczosError input_error(const std::string& inner) {
    LanczosError e(LanczosErrorKind::InputError);
    e.inner_ = inner;
    e.msg_ = "Invalid input parameter: " + inner;
    return e;
  }
  static LanczosError parameter_mismatch(const std::string& name, size_t expected, size_t actual) {
    LanczosError e(LanczosErrorKind::ParameterMismatch);
    e.param_name_ = name;
    e.expected_ = expected;
    e.actual_ = actual;
    e.msg_ = "Parameter mismatch: `" + name + "` expects size " + std::to_string(expected) +
             ", but got " + std::to_string(actual) + ".";
    return e;
  }
  static LanczosError evd_error(const std::string& inner) {  // inner: faer's EvdError {:?}
    LanczosError e(LanczosErrorKind::EvdError);
    e.inner_ = inner;
    e.msg_ = "A numerical error occurred during the eigendecomposition of T_k: " + inner;
    return e;
  }
  static LanczosError solver_error(const std::string& inner) {
    LanczosError e(LanczosErrorKind::SolverError);
    e.inner_ = inner;
    e.msg_ = "The user-provided f(T_k) solver failed: " + inner;
    return e;
  }
  LanczosErrorKind kind() const { return kind_; }
  const char* what() const noexcept override { return msg_.c_str(); }  // the Display text
  const std::string& inner() const { return inner_; }
  const std::string& param_name() const { return param_name_; }
  size_t expected() const { return expected_; }
  size_t actual() const { return actual_; }
  size_t operator_cols() const { return operator_cols_; }
  size_t vector_rows() const { return vector_rows_; }
  size_t breakdown_step() const { return breakdown_step_; }
  bool operator==(const LanczosError& o) const { return kind_ == o.kind_ && msg_ == o.msg_; }

 private:
  explicit LanczosError(LanczosErrorKind k) : kind_(k) {}
  LanczosErrorKind kind_;
  std::string msg_, inner_, param_name_;
  size_t expected_ = 0, actual_ = 0, operator_cols_ = 0, vector_rows_ = 0, breakdown_step_ = 0;
};

// Engine failures with no LanczosErrorKind counterpart (tpl_status >= 100).
class EngineError : public std::runtime_error {
 public:
  EngineError(tpl_status s, const std::string& m) : std::runtime_error(m), status_(s) {}
  tpl_status status() const { return status_; }

 private:
  tpl_status status_;
};
class DataLoaderError : public std::runtime_error {  // src/utils/data_loader.rs:16-43
 public:
  using std::runtime_error::runtime_error;
};

namespace detail {
// Rebuild the variant from tpl_last_error_detail's fields (never by parsing text); the
// fields must reproduce the engine's message, else the binding and the engine disagree.
[[noreturn]] inline void throw_status(tpl_status st) {
  tpl_error_detail d{};
  tpl_last_error_detail(&d);
  const std::string msg = d.message ? d.message : "";
  auto s = [](const char* p) { return std::string(p ? p : ""); };
  switch (st) {
    case TPL_ERR_INPUT:
    case TPL_ERR_PARAMETER_MISMATCH:
    case TPL_ERR_DIMENSION_MISMATCH:
    case TPL_ERR_SOLVER:
    case TPL_ERR_EVD:
    case TPL_ERR_BREAKDOWN: {
      LanczosError e =
          st == TPL_ERR_INPUT ? LanczosError::input_error(s(d.inner))
          : st == TPL_ERR_PARAMETER_MISMATCH
              ? LanczosError::parameter_mismatch(s(d.param_name), (size_t)d.expected, (size_t)d.actual)
          : st == TPL_ERR_DIMENSION_MISMATCH
              ? LanczosError::dimension_mismatch((size_t)d.operator_cols, (size_t)d.vector_rows)
          : st == TPL_ERR_SOLVER ? LanczosError::solver_error(s(d.inner))
          : st == TPL_ERR_EVD    ? LanczosError::evd_error(s(d.inner))
                                 : LanczosError::breakdown((size_t)d.breakdown_step);
      if (msg != e.what())
        throw EngineError(TPL_ERR_INVALID_ARGUMENT, "error detail does not match the message: " + msg);
      throw e;
    }
    case TPL_ERR_DATA_LOADER: throw DataLoaderError(msg);
    default: throw EngineError(st, msg);
  }
}
inline void check(tpl_status st) {
  if (st != TPL_OK) throw_status(st);
}
}  // namespace detail

// ---- dense column-major matrix (faer Mat<f64>) ----------------------------------------
struct Mat {
  size_t rows = 0, cols = 0;
  std::vector<double> data;  // column-major, ld = rows
  Mat() = default;
  Mat(size_t r, size_t c) : rows(r), cols(c), data(r * c, 0.0) {}
  static Mat column(std::vector<double> v) {
    Mat m;
    m.rows = v.size();
    m.cols = 1;
    m.data = std::move(v);
    return m;
  }
  double& operator()(size_t i, size_t j) { return data[j * rows + i]; }
  double operator()(size_t i, size_t j) const { return data[j * rows + i]; }
};

// ---- scalar outputs: src/algorithms/mod.rs:57-135 ---------------------------------------
struct LanczosDecomposition {
  std::vector<double> alphas;  // steps_taken
  std::vector<double> betas;   // steps_taken - 1
  size_t steps_taken = 0;
  double b_norm = 0.0;
};
struct LanczosOutput {
  Mat v_k;  // n x steps_taken
  LanczosDecomposition decomposition;
};
struct LanczosPassTwoOutput {
  std::vector<double> x_k;
  Mat v_k;  // the regenerated basis V'_k
};
// View of T_k handed to the step callback (TridiagonalSystemView, src/algorithms/mod.rs:57-70).
struct TridiagonalSystemView {
  const double* alphas;
  size_t n_alphas;
  const double* betas;
  size_t n_betas;
  size_t steps_taken;
};
// LanczosCallback (src/algorithms/mod.rs:82-86): k (1-based), V_k as a DEVICE pointer
// (column-major, ld = n, k valid columns: the basis lives in HBM), the T_k view; return
// false to stop. Deviation: V_k is not copied to the host per step.
using LanczosCallback = std::function<bool(size_t k, const double* v_k_device, int64_t n,
                                           const TridiagonalSystemView& t_k)>;

// f(T_k) e_1 solver (the reference's f_tk_solver closure): (alphas, betas) -> y' (steps x 1).
// Throwing is the closure's Err(e): the solve fails with SolverError(e.what()).
using FtkSolver = std::function<Mat(const std::vector<double>& alphas, const std::vector<double>& betas)>;

// ---- device context and operator ---------------------------------------------------------
class Context {
 public:
  explicit Context(int device = 0) { detail::check(tpl_ctx_create(device, &ctx_)); }
  ~Context() {
    if (ctx_) tpl_ctx_destroy(ctx_);
  }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  tpl_ctx_t handle() const { return ctx_; }

 private:
  tpl_ctx_t ctx_ = nullptr;
};

// One rank's RCCL communicator over xGMI (tpl_dist_create), one process per GPU. Rank 0
// calls unique_id() and hands the bytes to the other ranks by the host program's own
// channel (MPI, a file, a socket). Shared by the partitioned operators built on it.
class Dist {
 public:
  using Id = std::array<uint8_t, TPL_DIST_ID_BYTES>;
  static Id unique_id() {
    Id id{};
    detail::check(tpl_dist_unique_id(id.data()));
    return id;
  }
  Dist(int device, int rank, int nranks, const Id& id) {
    detail::check(tpl_dist_create(device, rank, nranks, id.data(), &d_));
  }
  ~Dist() {
    if (d_) tpl_dist_destroy(d_);
  }
  Dist(const Dist&) = delete;
  Dist& operator=(const Dist&) = delete;
  tpl_dist_t handle() const { return d_; }

 private:
  tpl_dist_t d_ = nullptr;
};

// How HipCsrOp::partitioned splits a matrix over the ranks (include/tpl.h): replicated
// long rows (the KKT form), halo-exchange row blocks (any symmetric matrix), or Auto —
// tpl_dist_choose_partition's rule, shared with the Python and Rust bindings: replicated
// when it applies, else halo when the halo is at most half the widest block, else plain
// row blocks.
enum class Partition { Replicated, Halo, Auto };

// A symmetric sparse matrix resident in HBM (faer LinOp<f64> on SparseColMat<usize, f64>;
// symmetric, so its CSR arrays are the reference's CSC arrays). Columns ascending per row.
class HipCsrOp {
 public:
  HipCsrOp(const Context& ctx, int64_t n, const std::vector<int64_t>& row_ptr,
           const std::vector<int32_t>& col_idx, const std::vector<double>& vals) {
    if (n < 0 || (int64_t)row_ptr.size() != n + 1 || col_idx.size() != vals.size() ||
        (int64_t)col_idx.size() != row_ptr.back())  // row_ptr has n + 1 >= 1 entries here
      throw EngineError(TPL_ERR_INVALID_ARGUMENT, "CSR arrays do not match n / nnz");
    detail::check(tpl_op_create_csr(ctx.handle(), n, (int64_t)vals.size(), row_ptr.data(),
                                    col_idx.data(), vals.data(), &op_));
  }
  // This rank's part of the WHOLE matrix (every rank passes the same CSR; collective).
  // The solvers take it unchanged; b and x are then this rank's rows, local_rows().
  static HipCsrOp partitioned(std::shared_ptr<Dist> dist, int64_t n,
                              const std::vector<int64_t>& row_ptr,
                              const std::vector<int32_t>& col_idx,
                              const std::vector<double>& vals, Partition how = Partition::Auto) {
    if (!dist || n < 1 || (int64_t)row_ptr.size() != n + 1 || col_idx.size() != vals.size() ||
        (int64_t)col_idx.size() != row_ptr.back())
      throw EngineError(TPL_ERR_INVALID_ARGUMENT, "CSR arrays do not match n / nnz");
    HipCsrOp op;
    if (how == Partition::Replicated)
      detail::check(tpl_dist_op_create_replicated(dist->handle(), n, row_ptr.data(),
                                                  col_idx.data(), vals.data(), &op.op_));
    else if (how == Partition::Halo)
      detail::check(tpl_dist_op_create_halo(dist->handle(), n, nullptr, row_ptr.data(),
                                            col_idx.data(), vals.data(), &op.op_));
    else
      detail::check(tpl_dist_op_create_auto(dist->handle(), n, row_ptr.data(), col_idx.data(),
                                            vals.data(), &op.op_, nullptr));
    op.dist_ = std::move(dist);
    return op;
  }
  // The global row of each entry of this operator's vectors.
  std::vector<int64_t> local_rows() const {
    std::vector<int64_t> rows(std::max<size_t>(nrows(), 1));
    detail::check(tpl_op_local_rows(op_, rows.data()));
    rows.resize(nrows());
    return rows;
  }
  ~HipCsrOp() {
    if (op_) tpl_op_destroy(op_);  // before dist_ (the communicator) is released
  }
  HipCsrOp(HipCsrOp&& o) noexcept
      : op_(std::exchange(o.op_, nullptr)), dist_(std::move(o.dist_)) {}
  HipCsrOp& operator=(HipCsrOp&& o) noexcept {
    std::swap(op_, o.op_);
    std::swap(dist_, o.dist_);
    return *this;
  }
  HipCsrOp(const HipCsrOp&) = delete;
  HipCsrOp& operator=(const HipCsrOp&) = delete;
  size_t nrows() const { return (size_t)tpl_op_nrows(op_); }
  size_t ncols() const { return (size_t)tpl_op_nrows(op_); }
  // LinOp::apply: y = A x (compatibility path; the solvers never call it per step).
  std::vector<double> apply(const std::vector<double>& x) const {
    if (x.size() != nrows()) throw LanczosError::dimension_mismatch(ncols(), x.size());
    std::vector<double> y(nrows());
    detail::check(tpl_op_apply(op_, x.data(), y.data(), TPL_MEM_HOST));
    return y;
  }
  tpl_op_t handle() const { return op_; }

 private:
  HipCsrOp() = default;
  tpl_op_t op_ = nullptr;
  std::shared_ptr<Dist> dist_;  // partitioned operators: keeps the communicator alive
};

namespace detail {
// tpl_ftk_fn trampoline around an FtkSolver (user = the FtkSolver).
struct FtkCall {
  const FtkSolver* f;
  bool cols_mismatch = false;  // y' had ncols != 1 (src/solvers.rs:78: a ParameterMismatch)
  size_t rows = 0;
};
inline int ftk_trampoline(const double* a, size_t na, const double* b, size_t nb, double* y,
                          size_t ycap, size_t* ylen, char* err, size_t errcap, void* user) {
  auto* c = static_cast<FtkCall*>(user);
  try {
    const Mat m = (*c->f)(std::vector<double>(a, a + na), std::vector<double>(b, b + nb));
    c->rows = m.rows;
    if (m.cols != 1) {  // report a length the engine rejects; remapped after the call
      c->cols_mismatch = true;
      *ylen = m.rows != na ? m.rows : na + 1;
      return 0;
    }
    *ylen = m.rows;
    if (m.rows && ycap) std::memcpy(y, m.data.data(), (m.rows < ycap ? m.rows : ycap) * sizeof(double));
    return 0;
  } catch (const std::exception& e) {
    const size_t len = errcap ? std::min(std::strlen(e.what()), errcap - 1) : 0;
    if (errcap) {
      std::memcpy(err, e.what(), len);
      err[len] = '\0';
    }
    return 1;
  }
}
inline bool is_builtin(const FtkSolver& f, tpl_ftk_fn* out);
}  // namespace detail

// ---- built-in f(T_k) solvers (tpl_ftk_inv / _exp / _sq): as FtkSolvers and as markers the
// solvers recognise, so a built-in can run on the device inside the solve (tpl.h) ----------
namespace ftk {
struct Builtin {
  tpl_ftk_fn fn;
  Mat operator()(const std::vector<double>& a, const std::vector<double>& b) const {
    std::vector<double> y(a.size());
    size_t len = 0;
    char err[512] = {0};
    if (fn(a.data(), a.size(), b.data(), b.size(), y.data(), y.size(), &len, err, sizeof err, nullptr))
      throw std::runtime_error(err);
    y.resize(len);
    return Mat::column(std::move(y));
  }
};
inline FtkSolver inv() { return Builtin{tpl_ftk_inv}; }  // T_k^{-1} e_1 (tridiagonal LU, partial pivoting)
// exp(T_k) e_1: on the host a symmetric tridiagonal QL; as a solver's built-in it may run on
// the device instead (a Chebyshev expansion within an EVD-class tolerance of the QL result,
// include/tpl.h tpl_op_set_device_ftk) — tpl_op_set_device_ftk(op, 0) forces the host QL
inline FtkSolver exp() { return Builtin{tpl_ftk_exp}; }
inline FtkSolver sq() { return Builtin{tpl_ftk_sq}; }    // T_k^2 e_1
}  // namespace ftk

namespace detail {
inline bool is_builtin(const FtkSolver& f, tpl_ftk_fn* out) {
  if (const auto* b = f.target<ftk::Builtin>()) {
    *out = b->fn;
    return true;
  }
  return false;
}
inline void check_b(const HipCsrOp& op, const std::vector<double>& b) {
  if (b.size() != op.ncols()) throw LanczosError::dimension_mismatch(op.ncols(), b.size());
}
template <class Call>
std::vector<double> solve(const HipCsrOp& op, const std::vector<double>& b, size_t k,
                          const FtkSolver& f, Call call) {
  check_b(op, b);
  std::vector<double> x(op.nrows());
  tpl_ftk_fn fn = nullptr;
  if (is_builtin(f, &fn)) {  // the engine may evaluate it on the device
    detail::check(call(op.handle(), b.data(), (int64_t)b.size(), k, fn, nullptr, x.data()));
    return x;
  }
  FtkCall c{&f};
  const tpl_status st = call(op.handle(), b.data(), (int64_t)b.size(), k, &ftk_trampoline, &c, x.data());
  if (st == TPL_ERR_PARAMETER_MISMATCH && c.cols_mismatch) {
    tpl_error_detail d{};
    tpl_last_error_detail(&d);
    throw LanczosError::parameter_mismatch("y_k_prime", (size_t)d.expected, c.rows);
  }
  detail::check(st);
  return x;
}
}  // namespace detail

// ---- high-level API: src/solvers.rs -------------------------------------------------------
namespace solvers {
// solvers::lanczos (src/solvers.rs:46-107): x_k = ||b|| V_k f(T_k) e_1, V_k kept in HBM.
inline std::vector<double> lanczos(const HipCsrOp& op, const std::vector<double>& b, size_t k,
                                   const FtkSolver& f_tk_solver) {
  return detail::solve(op, b, k, f_tk_solver,
                       [](tpl_op_t o, const double* bp, int64_t n, size_t kk, tpl_ftk_fn fn, void* u,
                          double* x) { return tpl_lanczos(o, bp, n, kk, fn, u, x, TPL_MEM_HOST); });
}
// solvers::lanczos_two_pass (src/solvers.rs:133-175): O(n) memory, V_k regenerated in pass two.
inline std::vector<double> lanczos_two_pass(const HipCsrOp& op, const std::vector<double>& b,
                                            size_t k, const FtkSolver& f_tk_solver) {
  return detail::solve(op, b, k, f_tk_solver,
                       [](tpl_op_t o, const double* bp, int64_t n, size_t kk, tpl_ftk_fn fn, void* u,
                          double* x) { return tpl_lanczos_two_pass(o, bp, n, kk, fn, u, x, TPL_MEM_HOST); });
}
}  // namespace solvers

// ---- low-level API: src/algorithms/ -----------------------------------------------------
namespace algorithms {
namespace detail {
struct CbCall {
  const LanczosCallback* cb;
  std::exception_ptr err;
};
inline int step_trampoline(size_t k, const double* v, int64_t n, const double* a, size_t na,
                           const double* b, size_t nb, void* user) {
  auto* c = static_cast<CbCall*>(user);
  try {
    return (*c->cb)(k, v, n, TridiagonalSystemView{a, na, b, nb, k}) ? 1 : 0;
  } catch (...) {
    c->err = std::current_exception();  // rethrown after the solve; stops the iteration
    return 0;
  }
}
inline LanczosDecomposition decomp(std::vector<double> a, std::vector<double> b, size_t steps,
                                   double bn) {
  a.resize(steps);
  b.resize(steps ? steps - 1 : 0);
  return LanczosDecomposition{std::move(a), std::move(b), steps, bn};
}
}  // namespace detail

// lanczos_standard (src/algorithms/lanczos.rs:55-156), with an optional per-step callback.
inline LanczosOutput lanczos_standard(const HipCsrOp& op, const std::vector<double>& b, size_t k,
                                      const LanczosCallback* callback = nullptr) {
  ::tpl::detail::check_b(op, b);
  const size_t n = op.nrows();
  std::vector<double> al(k ? k : 1), be(k ? k : 1), v(n * (k ? k : 1));
  size_t steps = 0;
  double bn = 0.0;
  detail::CbCall c{callback, nullptr};
  const tpl_status st =
      tpl_lanczos_standard(op.handle(), b.data(), (int64_t)n, k, al.data(), be.data(), &steps, &bn,
                           v.data(), TPL_MEM_HOST, 0, callback ? &detail::step_trampoline : nullptr,
                           callback ? &c : nullptr);
  if (c.err) std::rethrow_exception(c.err);
  ::tpl::detail::check(st);
  LanczosOutput out;
  out.v_k.rows = n;
  out.v_k.cols = steps;
  v.resize(n * steps);
  out.v_k.data = std::move(v);
  out.decomposition = detail::decomp(std::move(al), std::move(be), steps, bn);
  return out;
}
// lanczos_pass_one (src/algorithms/lanczos_two_pass.rs:65-110): scalars only.
inline LanczosDecomposition lanczos_pass_one(const HipCsrOp& op, const std::vector<double>& b, size_t k) {
  ::tpl::detail::check_b(op, b);
  std::vector<double> al(k ? k : 1), be(k ? k : 1);
  size_t steps = 0;
  double bn = 0.0;
  ::tpl::detail::check(tpl_lanczos_pass_one(op.handle(), b.data(), (int64_t)b.size(), k, al.data(),
                                            be.data(), &steps, &bn, TPL_MEM_HOST));
  return detail::decomp(std::move(al), std::move(be), steps, bn);
}
// lanczos_pass_two_with_basis (src/algorithms/lanczos_two_pass.rs:149-166): x and V'_k.
inline LanczosPassTwoOutput lanczos_pass_two_with_basis(const HipCsrOp& op, const std::vector<double>& b,
                                                        const LanczosDecomposition& d,
                                                        const std::vector<double>& y_k) {
  ::tpl::detail::check_b(op, b);
  const size_t n = op.nrows();
  LanczosPassTwoOutput out;
  out.x_k.resize(n);
  out.v_k = Mat(n, d.steps_taken);
  ::tpl::detail::check(tpl_lanczos_pass_two(op.handle(), b.data(), (int64_t)n, d.alphas.data(),
                                            d.alphas.size(), d.betas.data(), d.betas.size(),
                                            d.steps_taken, d.b_norm, y_k.data(), y_k.size(),
                                            out.x_k.data(), out.v_k.data.data(), TPL_MEM_HOST));
  return out;
}
// lanczos_pass_two (src/algorithms/lanczos_two_pass.rs:128-140): x only (y_k = y' ||b||).
inline std::vector<double> lanczos_pass_two(const HipCsrOp& op, const std::vector<double>& b,
                                            const LanczosDecomposition& d, const std::vector<double>& y_k) {
  ::tpl::detail::check_b(op, b);
  std::vector<double> x(op.nrows());
  ::tpl::detail::check(tpl_lanczos_pass_two(op.handle(), b.data(), (int64_t)b.size(), d.alphas.data(),
                                            d.alphas.size(), d.betas.data(), d.betas.size(),
                                            d.steps_taken, d.b_norm, y_k.data(), y_k.size(),
                                            x.data(), nullptr, TPL_MEM_HOST));
  return x;
}
}  // namespace algorithms

// ---- data loader: src/utils/data_loader.rs:211-259 ------------------------------------------
struct KktSystem {
  int64_t n = 0, num_nodes = 0, num_arcs = 0;
  std::vector<int64_t> row_ptr;
  std::vector<int32_t> col_idx;
  std::vector<double> vals;
};
inline KktSystem load_kkt_system(const std::string& dmx, const std::string& qfc) {
  tpl_csr_host h{};
  ::tpl::detail::check(tpl_load_kkt_system(dmx.c_str(), qfc.c_str(), &h));
  KktSystem s;
  s.n = h.n;
  s.num_nodes = h.num_nodes;
  s.num_arcs = h.num_arcs;
  s.row_ptr.assign(h.row_ptr, h.row_ptr + h.n + 1);
  s.col_idx.assign(h.col_idx, h.col_idx + h.nnz);
  s.vals.assign(h.vals, h.vals + h.nnz);
  tpl_csr_host_free(&h);
  return s;
}

}  // namespace tpl

#endif  // TPL_HPP_
