// tpl_internal.h — host-side internals shared by the runtime translation units.
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "../../include/tpl.h"

namespace tpl {

// The fields of a LanczosErrorKind variant (src/error.rs:20-58), carried beside the
// formatted message so a binding can rebuild the variant itself (tpl_last_error_detail).
struct ErrDetail {
  std::string inner;        // InputError / SolverError / EvdError: the {0} of the Display
  std::string param_name;   // ParameterMismatch
  uint64_t expected = 0, actual = 0;
  uint64_t operator_cols = 0, vector_rows = 0;  // DimensionMismatch
  uint64_t breakdown_step = 0;                  // Breakdown { k }
};

// An error carrying the C-ABI status and the reference-formatted message.
struct Error : std::exception {
  tpl_status code;
  std::string msg;
  ErrDetail det;
  Error(tpl_status c, std::string m, ErrDetail d = {}) : code(c), msg(std::move(m)), det(std::move(d)) {}
  const char* what() const noexcept override { return msg.c_str(); }
};
[[noreturn]] inline void fail(tpl_status c, const std::string& m) { throw Error(c, m); }

// Record the outcome of an ABI call on this thread (status TPL_OK and "" after success).
void set_last_error(const std::string& m);
void set_last_error(tpl_status code, const std::string& m, const ErrDetail& d);

// LanczosErrorKind Display strings (src/error.rs:20-58).
std::string msg_input(const std::string& what);                  // "Invalid input parameter: ..."
std::string msg_param_mismatch(const std::string& name, size_t expected, size_t actual);
std::string msg_solver(const std::string& e);
std::string msg_dimension(int64_t operator_cols, int64_t vector_rows);
std::string msg_evd(const std::string& e);

// Throw a LanczosErrorKind with its fields (message formatted as the reference does).
[[noreturn]] void fail_input(const std::string& what);
[[noreturn]] void fail_param_mismatch(const std::string& name, size_t expected, size_t actual);
[[noreturn]] void fail_dimension(int64_t operator_cols, int64_t vector_rows);
[[noreturn]] void fail_solver(const std::string& e);

} // namespace tpl
