// tpl_errors.cpp — error state and the reference's error texts (host only).
#include <string>

#include "tpl_internal.h"

namespace tpl {

namespace {
struct LastError {
  tpl_status code = TPL_OK;
  std::string msg;
  ErrDetail det;
};
thread_local LastError g_last;
}  // namespace

void set_last_error(const std::string& m) {
  g_last.code = m.empty() ? TPL_OK : TPL_ERR_INVALID_ARGUMENT;
  g_last.msg = m;
  g_last.det = ErrDetail{};
}
void set_last_error(tpl_status code, const std::string& m, const ErrDetail& d) {
  g_last.code = code;
  g_last.msg = m;
  g_last.det = d;
}

std::string msg_input(const std::string& what) { return "Invalid input parameter: " + what; }
std::string msg_param_mismatch(const std::string& name, size_t expected, size_t actual) {
  return "Parameter mismatch: `" + name + "` expects size " + std::to_string(expected) +
         ", but got " + std::to_string(actual) + ".";
}
std::string msg_solver(const std::string& e) {
  return "The user-provided f(T_k) solver failed: " + e;
}
std::string msg_dimension(int64_t operator_cols, int64_t vector_rows) {
  return "Dimension mismatch: operator has " + std::to_string(operator_cols) +
         " columns but vector has " + std::to_string(vector_rows) + " rows.";
}
std::string msg_evd(const std::string& e) {
  return "A numerical error occurred during the eigendecomposition of T_k: " + e;
}

void fail_input(const std::string& what) {
  ErrDetail d;
  d.inner = what;
  throw Error(TPL_ERR_INPUT, msg_input(what), d);
}
void fail_param_mismatch(const std::string& name, size_t expected, size_t actual) {
  ErrDetail d;
  d.param_name = name;
  d.expected = expected;
  d.actual = actual;
  throw Error(TPL_ERR_PARAMETER_MISMATCH, msg_param_mismatch(name, expected, actual), d);
}
void fail_dimension(int64_t operator_cols, int64_t vector_rows) {
  ErrDetail d;
  d.operator_cols = (uint64_t)operator_cols;
  d.vector_rows = (uint64_t)vector_rows;
  throw Error(TPL_ERR_DIMENSION_MISMATCH, msg_dimension(operator_cols, vector_rows), d);
}
void fail_solver(const std::string& e) {
  ErrDetail d;
  d.inner = e;
  throw Error(TPL_ERR_SOLVER, msg_solver(e), d);
}

const char* last_error() { return g_last.msg.c_str(); }

} // namespace tpl

extern "C" const char* tpl_last_error(void) { return tpl::last_error(); }

extern "C" tpl_status tpl_last_error_detail(tpl_error_detail* out) {
  if (!out) return TPL_ERR_INVALID_ARGUMENT;  // leaves the recorded error untouched
  const tpl::LastError& e = tpl::g_last;
  out->status = (int32_t)e.code;
  out->message = e.msg.c_str();
  out->inner = e.det.inner.c_str();
  out->param_name = e.det.param_name.c_str();
  out->expected = e.det.expected;
  out->actual = e.det.actual;
  out->operator_cols = e.det.operator_cols;
  out->vector_rows = e.det.vector_rows;
  out->breakdown_step = e.det.breakdown_step;
  return TPL_OK;
}
