// tpl_errors.cpp — error state and the reference's error texts (host only).
#include <string>

#include "tpl_internal.h"

namespace tpl {

static thread_local std::string g_last_error;
void set_last_error(const std::string& m) { g_last_error = m; }

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

const char* last_error() { return g_last_error.c_str(); }

} // namespace tpl

extern "C" const char* tpl_last_error(void) { return tpl::last_error(); }
