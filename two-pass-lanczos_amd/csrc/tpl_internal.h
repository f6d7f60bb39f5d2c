// tpl_internal.h — host-side internals shared by the runtime translation units.
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "../../include/tpl.h"

namespace tpl {

// An error carrying the C-ABI status and the reference-formatted message.
struct Error : std::exception {
  tpl_status code;
  std::string msg;
  Error(tpl_status c, std::string m) : code(c), msg(std::move(m)) {}
  const char* what() const noexcept override { return msg.c_str(); }
};
[[noreturn]] inline void fail(tpl_status c, const std::string& m) { throw Error(c, m); }

void set_last_error(const std::string& m);

// LanczosErrorKind Display strings (src/error.rs:20-58).
std::string msg_input(const std::string& what);                  // "Invalid input parameter: ..."
std::string msg_param_mismatch(const std::string& name, size_t expected, size_t actual);
std::string msg_solver(const std::string& e);
std::string msg_dimension(int64_t operator_cols, int64_t vector_rows);
std::string msg_evd(const std::string& e);

} // namespace tpl
