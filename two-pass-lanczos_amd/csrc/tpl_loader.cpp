// tpl_loader.cpp — .dmx/.qfc reader with the reference's exact semantics,
// assembling the KKT operator A = [[D, E^T], [E, 0]] directly as CSR.
//
// Reference: src/utils/data_loader.rs
//   parse_dmx      (:68-156)  'c' comments, 'p min <nodes> <arcs>', 'a u v ...' arcs;
//                             arc j -> E[u-1, j] = +1, E[v-1, j] = -1; index 0 rejected.
//   parse_qfc      (:166-198) line 1 = m (must equal the dmx arc count); then
//                             `lines.skip(m).take(m)`, one f64 per line, no trimming.
//                             With qfcgen's 3-line files this reads NOTHING (D = empty).
//   load_kkt_system(:211-259) D on the diagonal of the arc block, E below, E^T right.
// The reference builds triplets and a CSC matrix; A is symmetric, so its CSR
// arrays are the same arrays. Duplicate triplets are summed (a self-loop arc
// u == v yields an explicit 0 entry), as faer's try_new_from_triplets does.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "tpl_internal.h"

namespace {

using tpl::fail;

// DataLoaderError Display strings (src/utils/data_loader.rs:16-43)
[[noreturn]] void err_io(int e) {
  fail(TPL_ERR_DATA_LOADER,
       std::string("I/O error: ") + std::strerror(e) + " (os error " + std::to_string(e) + ")");
}
[[noreturn]] void err_parse_int(const std::string& s) {
  fail(TPL_ERR_DATA_LOADER, "Parse error: Failed to parse integer from '" + s + "'");
}
[[noreturn]] void err_parse_float(const std::string& s) {
  fail(TPL_ERR_DATA_LOADER, "Parse error: Failed to parse float from '" + s + "'");
}
[[noreturn]] void err_problem_line() {
  fail(TPL_ERR_DATA_LOADER,
       "Format error: The 'p min' problem line was not found or was malformed.");
}
[[noreturn]] void err_eof() {
  fail(TPL_ERR_DATA_LOADER, "Format error: Unexpected end of file while reading data.");
}
[[noreturn]] void err_arc_mismatch(size_t qfc, size_t dmx) {
  fail(TPL_ERR_DATA_LOADER, "Dimension mismatch: qfc file specifies " + std::to_string(qfc) +
                                " arcs, but dmx file has " + std::to_string(dmx) + ".");
}
[[noreturn]] void err_construction() {
  fail(TPL_ERR_DATA_LOADER, "Internal error: Failed to construct the sparse matrix from triplets.");
}
[[noreturn]] void err_node_index(const std::string& s) {
  fail(TPL_ERR_DATA_LOADER, "Format error: Invalid node index '" + s +
                                "'. DIMACS format requires 1-based positive integers.");
}

// Rust's `str::parse::<usize>()`: optional '+', then ASCII digits only, no overflow.
bool parse_usize(const std::string& s, size_t& out) {
  size_t i = 0;
  if (i < s.size() && s[i] == '+') ++i;
  if (i == s.size()) return false;
  unsigned long long v = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    const unsigned d = (unsigned)(s[i] - '0');
    if (v > (~0ull - d) / 10) return false;
    v = v * 10 + d;
  }
  out = (size_t)v;
  return true;
}

// Rust's `str::parse::<f64>()`: decimal/scientific, inf/infinity/nan (any case),
// optional sign; no surrounding whitespace, no hex.
bool parse_f64(const std::string& s, double& out) {
  if (s.empty()) return false;
  for (char c : s)
    if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v' || c == 'x' ||
        c == 'X' || c == 'p' || c == 'P')
      return false;
  const char* b = s.c_str();
  char* e = nullptr;
  errno = 0;
  const double v = std::strtod(b, &e);
  if (e != b + s.size()) return false;
  out = v; // overflow -> +-inf, as Rust
  return true;
}

std::vector<std::string> split_ws(const std::string& line) {
  std::vector<std::string> parts;
  size_t i = 0;
  while (i < line.size()) {
    while (i < line.size() && std::isspace((unsigned char)line[i])) ++i;
    if (i >= line.size()) break;
    size_t j = i;
    while (j < line.size() && !std::isspace((unsigned char)line[j])) ++j;
    parts.emplace_back(line.substr(i, j - i));
    i = j;
  }
  return parts;
}

// BufRead::lines(): split on '\n', drop one trailing '\r'.
bool next_line(std::FILE* f, std::string& line) {
  line.clear();
  int c;
  bool any = false;
  while ((c = std::fgetc(f)) != EOF) {
    any = true;
    if (c == '\n') break;
    line.push_back((char)c);
  }
  if (!any) return false;
  if (!line.empty() && line.back() == '\r') line.pop_back();
  return true;
}

struct FileGuard {
  std::FILE* f;
  ~FileGuard() {
    if (f) std::fclose(f);
  }
};

struct Trip {
  int64_t r, c;
  double v;
};

// CSR of A = [[D, E^T], [E, 0]] (load_kkt_system, src/utils/data_loader.rs:211-259):
// arc j has tail eu[j] (+1) and head ev[j] (-1); arcs j >= arc_counter are absent;
// qcost holds the D diagonal entries present (the 3-line qfc yields none).
void assemble_kkt(size_t num_nodes, size_t num_arcs, size_t arc_counter,
                  const std::vector<int64_t>& eu, const std::vector<int64_t>& ev,
                  const std::vector<double>& qcost, tpl_csr_host* out) {
    const int64_t m = (int64_t)num_arcs, p = (int64_t)num_nodes, n = m + p;
    if (n >= INT32_MAX) fail(TPL_ERR_UNSUPPORTED, "n must be < 2^31");
    // E column j holds rows eu[j] (+1) and ev[j] (-1), summed if equal (faer sums duplicates).
    // Arc row j of A: D[j] (if present) at column j, then E column j at columns m + node.
    // Node row m + r of A: E row r, i.e. the arcs touching node r, ascending arc index.
    std::vector<int64_t> deg(p, 0);
    for (int64_t j = 0; j < m; ++j) {
      if (j >= (int64_t)arc_counter) continue;
      deg[eu[j]]++;
      if (ev[j] != eu[j]) deg[ev[j]]++;
    }
    std::vector<int64_t> rp(n + 1, 0);
    for (int64_t j = 0; j < m; ++j) {
      int64_t c = (j < (int64_t)qcost.size()) ? 1 : 0;
      if (j < (int64_t)arc_counter) c += (eu[j] == ev[j]) ? 1 : 2;
      rp[j + 1] = c;
    }
    for (int64_t r = 0; r < p; ++r) rp[m + r + 1] = deg[r];
    for (int64_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
    const int64_t nnz = rp[n];
    if (nnz >= INT32_MAX) fail(TPL_ERR_UNSUPPORTED, "nnz must be < 2^31");
    std::vector<int32_t> col(nnz);
    std::vector<double> val(nnz);
    for (int64_t j = 0; j < m; ++j) {
      int64_t q = rp[j];
      if (j < (int64_t)qcost.size()) {
        col[q] = (int32_t)j;
        val[q] = qcost[j];
        ++q;
      }
      if (j < (int64_t)arc_counter) {
        const int64_t u = eu[j], v = ev[j];
        if (u == v) {
          col[q] = (int32_t)(m + u);
          val[q] = 1.0 + -1.0;
        } else {
          const int64_t lo = u < v ? u : v, hi = u < v ? v : u;
          col[q] = (int32_t)(m + lo);
          val[q] = (lo == u) ? 1.0 : -1.0;
          col[q + 1] = (int32_t)(m + hi);
          val[q + 1] = (hi == u) ? 1.0 : -1.0;
        }
      }
    }
    std::vector<int64_t> fill(p);
    for (int64_t r = 0; r < p; ++r) fill[r] = rp[m + r];
    for (int64_t j = 0; j < (int64_t)arc_counter && j < m; ++j) { // ascending arc j
      const int64_t u = eu[j], v = ev[j];
      if (u == v) {
        col[fill[u]] = (int32_t)j;
        val[fill[u]++] = 1.0 + -1.0;
      } else {
        col[fill[u]] = (int32_t)j;
        val[fill[u]++] = 1.0;
        col[fill[v]] = (int32_t)j;
        val[fill[v]++] = -1.0;
      }
    }
    out->n = n;
    out->nnz = nnz;
    out->num_nodes = p;
    out->num_arcs = m;
    out->row_ptr = (int64_t*)std::malloc((n + 1) * sizeof(int64_t));
    out->col_idx = (int32_t*)std::malloc(std::max<int64_t>(nnz, 1) * sizeof(int32_t));
    out->vals = (double*)std::malloc(std::max<int64_t>(nnz, 1) * sizeof(double));
    if (!out->row_ptr || !out->col_idx || !out->vals) {
      tpl_csr_host_free(out);
      fail(TPL_ERR_OUT_OF_MEMORY, "host allocation failed");
    }
    std::memcpy(out->row_ptr, rp.data(), (n + 1) * sizeof(int64_t));
    if (nnz) {
      std::memcpy(out->col_idx, col.data(), nnz * sizeof(int32_t));
      std::memcpy(out->vals, val.data(), nnz * sizeof(double));
    }
}

} // namespace

extern "C" {

tpl_status tpl_load_kkt_system(const char* dmx_path, const char* qfc_path, tpl_csr_host* out) {
  try {
    if (!dmx_path || !qfc_path || !out) fail(TPL_ERR_INVALID_ARGUMENT, "NULL argument");
    std::memset(out, 0, sizeof(*out));
    // ---- parse_dmx (:68-156)
    std::FILE* fd = std::fopen(dmx_path, "rb");
    if (!fd) err_io(errno);
    FileGuard gd{fd};
    std::setvbuf(fd, nullptr, _IOFBF, 1 << 20);
    size_t num_nodes = 0, num_arcs = 0, arc_counter = 0;
    bool found = false;
    std::vector<int64_t> eu, ev; // per arc: row of +1, row of -1
    std::string line;
    while (next_line(fd, line)) {
      const std::vector<std::string> parts = split_ws(line);
      if (parts.empty()) continue;
      const std::string& t = parts[0];
      if (t == "c") continue;
      if (t == "p") {
        if (parts.size() >= 4 && parts[1] == "min") {
          if (!parse_usize(parts[2], num_nodes)) err_parse_int(parts[2]);
          if (!parse_usize(parts[3], num_arcs)) err_parse_int(parts[3]);
          found = true;
        } else {
          err_problem_line();
        }
      } else if (t == "a") {
        // (the reference indexes parts[1], parts[2] unchecked and would panic)
        const std::string su = parts.size() > 1 ? parts[1] : std::string();
        const std::string sv = parts.size() > 2 ? parts[2] : std::string();
        size_t u, v;
        if (!parse_usize(su, u)) err_parse_int(su);
        if (u == 0) err_node_index(su);
        if (!parse_usize(sv, v)) err_parse_int(sv);
        if (v == 0) err_node_index(sv);
        eu.push_back((int64_t)u - 1);
        ev.push_back((int64_t)v - 1);
        ++arc_counter;
      }
    }
    if (std::ferror(fd)) err_io(EIO);
    if (!found) err_problem_line();
    // SparseColMat::try_new_from_triplets(num_nodes, num_arcs, ...) bounds check (:152-153)
    for (size_t j = 0; j < arc_counter; ++j)
      if (j >= num_arcs || (size_t)eu[j] >= num_nodes || (size_t)ev[j] >= num_nodes)
        err_construction();

    // ---- parse_qfc (:166-198)
    std::FILE* fq = std::fopen(qfc_path, "rb");
    if (!fq) err_io(errno);
    FileGuard gq{fq};
    if (!next_line(fq, line)) err_eof();
    size_t m_from_file;
    if (!parse_usize(line, m_from_file)) err_parse_int("m");
    if (m_from_file != num_arcs) err_arc_mismatch(m_from_file, num_arcs);
    for (size_t s = 0; s < num_arcs; ++s)
      if (!next_line(fq, line)) break;
    std::vector<double> qcost;
    for (size_t s = 0; s < num_arcs; ++s) {
      if (!next_line(fq, line)) break;
      double c;
      if (!parse_f64(line, c)) err_parse_float(line);
      qcost.push_back(c);
    }

    assemble_kkt(num_nodes, num_arcs, arc_counter, eu, ev, qcost, out);
    tpl::set_last_error("");
    return TPL_OK;
  } catch (const tpl::Error& e) {
    tpl::set_last_error(e.code, e.msg, e.det);
    return e.code;
  } catch (const std::bad_alloc&) {
    tpl::set_last_error(TPL_ERR_OUT_OF_MEMORY, "host allocation failed", {});
    return TPL_ERR_OUT_OF_MEMORY;
  }
}

tpl_status tpl_generate_kkt(int64_t num_arcs, int64_t num_nodes, uint64_t seed,
                            tpl_csr_host* out) {
  try {
    if (!out) fail(TPL_ERR_INVALID_ARGUMENT, "out is NULL");
    *out = tpl_csr_host{};
    if (num_arcs < 1 || num_nodes < 2) fail(TPL_ERR_INVALID_ARGUMENT, "need >= 1 arc and >= 2 nodes");
    // Arcs (u, v), u != v, from a splitmix64 stream, then ordered by tail node and head
    // like netgen's output (each node's outgoing arcs contiguous). Degrees follow the
    // netgen instances' spread (measured on the 5k / 50k / 500k fixtures:
    // total degree / mean from 0.5 at the 5th percentile to 1.55-1.74 at the maximum,
    // out-degrees 0.2-1.9x the mean at the 10th / 90th percentiles, in-degrees within
    // 0.9-1.2x): node i draws an integer out-weight in [100, 1900] and an in-weight in
    // [800, 1200]; a tail is drawn with probability proportional to its out-weight, a head
    // (redrawn until it differs from the tail) proportional to its in-weight. Integer
    // weights and cumulative sums: the instance is the same on every platform.
    uint64_t st = seed;
    auto next = [&st]() {
      uint64_t z = (st += 0x9E3779B97F4A7C15ULL);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
      return z ^ (z >> 31);
    };
    const size_t p = (size_t)num_nodes;
    std::vector<uint64_t> cum_out(p + 1, 0), cum_in(p + 1, 0);
    for (size_t i = 0; i < p; ++i) {
      cum_out[i + 1] = cum_out[i] + 100 + next() % 1801;
      cum_in[i + 1] = cum_in[i] + 800 + next() % 401;
    }
    // node whose cumulative range holds r in [0, cum[p])
    auto pick = [p](const std::vector<uint64_t>& cum, uint64_t r) {
      return (int64_t)(std::upper_bound(cum.begin() + 1, cum.begin() + p + 1, r) -
                       (cum.begin() + 1));
    };
    std::vector<std::pair<int64_t, int64_t>> arcs((size_t)num_arcs);
    for (auto& a : arcs) {
      const int64_t u = pick(cum_out, next() % cum_out[p]);
      int64_t v;
      do v = pick(cum_in, next() % cum_in[p]);
      while (v == u);
      a = {u, v};
    }
    std::sort(arcs.begin(), arcs.end());
    std::vector<int64_t> eu((size_t)num_arcs), ev((size_t)num_arcs);
    for (size_t j = 0; j < arcs.size(); ++j) {
      eu[j] = arcs[j].first;
      ev[j] = arcs[j].second;
    }
    assemble_kkt((size_t)num_nodes, (size_t)num_arcs, (size_t)num_arcs, eu, ev, {}, out);
    tpl::set_last_error("");
    return TPL_OK;
  } catch (const tpl::Error& e) {
    tpl::set_last_error(e.code, e.msg, e.det);
    return e.code;
  } catch (const std::bad_alloc&) {
    tpl::set_last_error(TPL_ERR_OUT_OF_MEMORY, "host allocation failed", {});
    return TPL_ERR_OUT_OF_MEMORY;
  }
}

void tpl_csr_host_free(tpl_csr_host* csr) {
  if (!csr) return;
  std::free(csr->row_ptr);
  std::free(csr->col_idx);
  std::free(csr->vals);
  csr->row_ptr = nullptr;
  csr->col_idx = nullptr;
  csr->vals = nullptr;
}

} // extern "C"
