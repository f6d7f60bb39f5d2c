// sanitize_driver.cpp — the engine's host C++ (the .dmx/.qfc loader, the f(T_k) solvers,
// the SpMV layout builder) built with -fsanitize=address,undefined on the CPU and driven
// over the committed fixture, malformed and random inputs (sanitizers on
// host code; tpl_loader.cpp parses untrusted files). Any sanitizer report aborts the run;
// the layout checks also verify that every nonzero lands exactly once in the layout.
//
//   sanitize_driver <netgen-5000-3.dmx> <qfc> <scratch dir>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "tpl.h"
#include "tpl_internal.h"
#include "tpl_layout.h"

static int g_fail = 0;
#define CHECK(cond, ...)                                \
  do {                                                  \
    if (!(cond)) {                                      \
      std::printf("FAIL %s:%d: ", __FILE__, __LINE__);  \
      std::printf(__VA_ARGS__);                         \
      std::printf("\n");                                \
      ++g_fail;                                         \
    }                                                   \
  } while (0)

static void write_file(const std::string& path, const std::string& text) {
  FILE* f = std::fopen(path.c_str(), "wb");
  std::fwrite(text.data(), 1, text.size(), f);
  std::fclose(f);
}

static void loader_checks(const char* dmx, const char* qfc, const std::string& dir) {
  tpl_csr_host A{};
  CHECK(tpl_load_kkt_system(dmx, qfc, &A) == TPL_OK, "fixture: %s", tpl_last_error());
  CHECK(A.n == 5115 && A.nnz == 20000, "fixture sizes");
  tpl_csr_host_free(&A);
  // malformed inputs: every one must fail cleanly (status + message), never crash
  const char* bad[][2] = {
      {"p min 2 1\na 0 1\n", "1\n"},   {"a 1 2\n", "1\n"},          {"p min 2 1\na 1 x\n", "1\n"},
      {"p min 2 1\na 1 2\n", "2\n"},   {"p min 2 1\na 1 2\n", ""},  {"p min 2 1\na 1 99999999999\n", "1\n"},
      {"p min 2 1\na 1 2\n", "1\n1\nabc\n"}, {"p min -5 -1\n", "1\n"}, {"p min 2 1\na 1\n", "1\n"},
      {"p min 3 2\na 1 2\na 3 -1\n", "2\n"}, {"p min 2 1\na 2 1\na 1 2\n", "2\n"},
  };
  for (auto& t : bad) {
    write_file(dir + "/m.dmx", t[0]);
    write_file(dir + "/m.qfc", t[1]);
    tpl_csr_host B{};
    const tpl_status st = tpl_load_kkt_system((dir + "/m.dmx").c_str(), (dir + "/m.qfc").c_str(), &B);
    if (st == TPL_OK) tpl_csr_host_free(&B);
    else CHECK(std::strlen(tpl_last_error()) > 0, "error without message");
  }
  // random mutations of small valid files
  std::mt19937_64 rng(7);
  const std::string good = "c x\np min 4 5\na 1 2 0 1 1\na 2 3 0 1 2\na 3 4 0 1 3\na 4 1 0 1 4\na 1 3 0 1 5\n";
  const std::string qgood = "5\n1\n2\n3\n4\n5\n0.5\n1.5\n2.5\n3.5\n4.5\n";
  const char alphabet[] = "0123456789 -+.eExap\n\tmin";
  for (int it = 0; it < 400; ++it) {
    std::string d = good, q = qgood;
    const int edits = 1 + (int)(rng() % 6);
    for (int e = 0; e < edits; ++e) {
      std::string& s = (rng() % 3 == 0) ? q : d;
      if (s.empty()) continue;
      const size_t pos = rng() % s.size();
      switch (rng() % 3) {
        case 0: s[pos] = alphabet[rng() % (sizeof alphabet - 1)]; break;
        case 1: s.erase(pos, 1 + rng() % 4); break;
        default: s.insert(pos, 1, alphabet[rng() % (sizeof alphabet - 1)]);
      }
    }
    write_file(dir + "/r.dmx", d);
    write_file(dir + "/r.qfc", q);
    tpl_csr_host B{};
    if (tpl_load_kkt_system((dir + "/r.dmx").c_str(), (dir + "/r.qfc").c_str(), &B) == TPL_OK) {
      for (int64_t i = 0; i < B.n; ++i) CHECK(B.row_ptr[i] <= B.row_ptr[i + 1], "row_ptr");
      for (int64_t q2 = 0; q2 < B.nnz; ++q2) CHECK(B.col_idx[q2] >= 0 && B.col_idx[q2] < B.n, "col");
      tpl_csr_host_free(&B);
    }
  }
  tpl_csr_host G{};
  CHECK(tpl_generate_kkt(3000, 80, 11, &G) == TPL_OK, "generate");
  tpl_csr_host_free(&G);
  CHECK(tpl_generate_kkt(0, 80, 11, &G) != TPL_OK, "generate: bad sizes accepted");
}

static void ftk_checks() {
  std::mt19937_64 rng(3);
  std::uniform_real_distribution<double> U(-2.0, 2.0);
  for (size_t k : {1, 2, 3, 10, 57, 200, 333}) {
    std::vector<double> a(k), b(k > 1 ? k - 1 : 0), y(k);
    for (auto& v : a) v = U(rng);
    for (auto& v : b) v = 0.1 + std::fabs(U(rng));
    size_t len = 0;
    char err[64];
    for (auto fn : {tpl_ftk_inv, tpl_ftk_exp, tpl_ftk_sq}) {
      const int rc = fn(a.data(), k, b.data(), b.size(), y.data(), k, &len, err, sizeof err, nullptr);
      CHECK(rc == 0 && len == k, "ftk rc %d k %zu", rc, k);
    }
    // inv: residual of T y = e1
    tpl_ftk_inv(a.data(), k, b.data(), b.size(), y.data(), k, &len, err, sizeof err, nullptr);
    double r = 0, s = 0;
    for (size_t i = 0; i < k; ++i) {
      double t = a[i] * y[i] - (i == 0 ? 1.0 : 0.0);
      if (i > 0) t += b[i - 1] * y[i - 1];
      if (i + 1 < k) t += b[i] * y[i + 1];
      r += t * t;
      s += y[i] * y[i];
    }
    CHECK(std::sqrt(r) <= 1e-9 * std::max(1.0, std::sqrt(s)), "inv residual %g (k %zu)", std::sqrt(r), k);
  }
  // capacity errors write the message within err_cap
  double a1[3] = {1, 2, 3}, y1[3];
  size_t len = 0;
  char tiny[4];
  CHECK(tpl_ftk_exp(a1, 3, a1, 0, y1, 3, &len, tiny, sizeof tiny, nullptr) != 0 && tiny[3] == '\0',
        "exp size error");
}

// Symmetric random matrix: `hubs` rows of `hub_len` entries, the rest short.
static void random_csr(int64_t n, int hubs, int hub_len, uint64_t seed, std::vector<int32_t>& rp,
                       std::vector<int32_t>& col, std::vector<double>& val) {
  std::mt19937_64 rng(seed);
  std::map<std::pair<int32_t, int32_t>, double> m;
  for (int64_t i = 0; i < n; ++i) {
    const int k = (int)(rng() % 4);
    for (int e = 0; e < k; ++e) {
      const int32_t j = (int32_t)(rng() % n);
      const double v = (double)((int)(rng() % 5) - 2);
      m[{(int32_t)i, j}] = v;
      m[{j, (int32_t)i}] = v;
    }
  }
  for (int h = 0; h < hubs && n > 1; ++h) {
    const int32_t r = (int32_t)(rng() % n);
    for (int e = 0; e < hub_len; ++e) {
      const int32_t j = (int32_t)(rng() % n);
      m[{r, j}] = 1.0;
      m[{j, r}] = 1.0;
    }
  }
  rp.assign(n + 1, 0);
  col.clear();
  val.clear();
  for (auto& kv : m) rp[kv.first.first + 1]++;
  for (int64_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
  for (auto& kv : m) {
    col.push_back(kv.first.second);
    val.push_back(kv.second);
  }
}

static void layout_checks() {
  struct Case { int64_t n; int hubs, hub_len; int slices, srm; bool compress; };
  const Case cases[] = {{1, 0, 0, 0, -1, true},      {2, 1, 1, 0, -1, true},     {7, 1, 5, 0, -1, false},
                        {1000, 3, 300, 0, -1, true}, {1000, 3, 300, 8, 2, false}, {20000, 2, 9000, 0, -1, true},
                        {20000, 40, 700, 2, -1, true}, {5000, 0, 0, 4, 6, true},
                        // 8 slices and more than 32 bins per slice: crowded CU positions
                        {20000, 600, 1000, 8, -1, true}};
  // every bin packing: the first fit, the balanced cut (even and crowd-weighted caps),
  // the first fit with its lightest bins on the crowded positions
  const std::pair<int, double> packings[] = {{0, 1.0}, {1, 1.0}, {1, 0.5}, {2, 1.0}};
  for (const Case& c : cases)
  for (const auto& pk : packings) {
    std::vector<int32_t> rp, col;
    std::vector<double> val;
    random_csr(c.n, c.hubs, c.hub_len, 1234 + c.n, rp, col, val);
    tpl::SchedParams sp;
    sp.bin_balance = pk.first;
    sp.bin_crowd = pk.second;
    sp.slices = c.slices;
    sp.short_row_max = c.srm;
    sp.compress_values = sp.compress_cols = c.compress;
    tpl::Layout L;
    try {
      L = tpl::build_layout(c.n, c.n, rp, col, val, sp, tpl::ColMap{});
    } catch (const tpl::Error& e) {
      std::printf("FAIL layout n=%lld: %s\n", (long long)c.n, e.msg.c_str());
      ++g_fail;
      continue;
    }
    // every nonzero exactly once: short rows through the chunks, long rows through bins
    CHECK((int64_t)(L.srows.size() + L.lrows.size()) == c.n, "row split");
    int64_t seen_short = 0, seen_long = 0;
    const bool c16 = L.s_col16, b16 = L.b_col16;
    const int64_t nch = (int64_t)L.c_base.size();
    for (int64_t ch = 0; ch < nch; ++ch)
      for (int64_t k = 0; k < L.c_width[ch]; ++k)
        for (int p = 0; p < tpl::kChunkRows; ++p) {
          const int64_t e = L.c_base[ch] + k * tpl::kChunkRows + p;
          const bool pad = c16 ? L.s_col16v[e] == 0xFFFF : L.s_col[e] < 0;
          seen_short += !pad;
        }
    const size_t nbins = L.b_hdr.size();
    for (size_t bin = 0; bin < nbins && !L.lrows.empty(); ++bin)
      for (int32_t e = 0; e < L.bin_cap; ++e) {
        const size_t q = bin * L.bin_cap + e;
        const bool pad = b16 ? L.b_col16v[q] == 0xFFFF : L.b_col[q] < 0;
        seen_long += !pad;
      }
    int64_t want_short = 0, want_long = 0;
    for (int32_t r : L.srows) want_short += rp[r + 1] - rp[r];
    for (int32_t r : L.lrows) want_long += rp[r + 1] - rp[r];
    CHECK(seen_short == want_short && seen_long == want_long, "entries n=%lld: short %lld/%lld long %lld/%lld",
          (long long)c.n, (long long)seen_short, (long long)want_short, (long long)seen_long,
          (long long)want_long);
    // the bin tables: each long row's packed pieces are its pieces with entries (one
    // empty piece for a row with none), every one carrying that count - 1 (its arrival
    // count, BinSeg::pad)
    {
      std::vector<int32_t> got(L.lrows.size(), 0), pad(L.lrows.size(), -1);
      bool pad_ok = true;
      for (size_t bin = 0; bin < nbins && !L.lrows.empty(); ++bin)
        for (int j = 0; j < tpl::kTPB; ++j) {
          const tpl::BinSeg& g = L.b_seg[bin * tpl::kTPB + j];
          if (g.ri < 0) continue;
          ++got[g.ri];
          pad_ok = pad_ok && (pad[g.ri] < 0 || pad[g.ri] == g.pad);
          pad[g.ri] = g.pad;
        }
      for (size_t r = 0; r < L.lrows.size(); ++r) {
        const int32_t row = L.lrows[r];
        int want = 0;
        for (int s = 0; s < L.nslices; ++s) {
          const int64_t lo = (int64_t)c.n * s / L.nslices, hi = (int64_t)c.n * (s + 1) / L.nslices;
          int cnt = 0;
          for (int32_t q = rp[row]; q < rp[row + 1]; ++q) cnt += col[q] >= lo && col[q] < hi;
          want += cnt > 0;
        }
        want = std::max(want, 1);
        pad_ok = pad_ok && got[r] == want && pad[r] == want - 1;
      }
      CHECK(pad_ok, "bin pieces / arrival counts n=%lld", (long long)c.n);
    }
    // the locality order (a permutation, long rows last) and P A P^T (same entries,
    // columns ascending), then the layout of P A P^T
    for (int groups : {1, 16, 1000}) {
      tpl::SchedParams so = sp;
      so.order_groups = groups;
      const std::vector<int32_t> perm = tpl::locality_order(c.n, rp, col, so);
      if (perm.empty()) continue;
      std::vector<int32_t> iperm(c.n, -1);
      bool is_perm = (int64_t)perm.size() == c.n;
      for (int64_t i = 0; is_perm && i < c.n; ++i) {
        is_perm = perm[i] >= 0 && perm[i] < c.n && iperm[perm[i]] < 0;
        if (is_perm) iperm[perm[i]] = (int32_t)i;
      }
      CHECK(is_perm, "locality order n=%lld is not a permutation", (long long)c.n);
      if (!is_perm) continue;
      std::vector<int32_t> prp, pcol;
      std::vector<double> pval;
      tpl::permute_csr(c.n, rp, col, val, perm, iperm, prp, pcol, pval);
      bool ok = prp.size() == rp.size() && pcol.size() == col.size();
      for (int64_t i = 0; ok && i < c.n; ++i) {
        const int32_t e = perm[i];
        ok = prp[i + 1] - prp[i] == rp[e + 1] - rp[e];
        for (int32_t q = prp[i] + 1; ok && q < prp[i + 1]; ++q) ok = pcol[q] > pcol[q - 1];
      }
      CHECK(ok, "permuted CSR n=%lld", (long long)c.n);
      try {
        (void)tpl::build_layout(c.n, c.n, prp, pcol, pval, sp, tpl::ColMap{});
      } catch (const tpl::Error& e) {
        std::printf("FAIL permuted layout n=%lld: %s\n", (long long)c.n, e.msg.c_str());
        ++g_fail;
      }
    }
  }
}

// tpl_locality_order (host-only C ABI entry): malformed CSRs are rejected before any
// indexing (decreasing row_ptr, row_ptr[0] != 0, columns out of range or not ascending,
// NULL columns), and 300 random mutations of valid CSRs never read out of bounds —
// either rejected or a permutation.
static void locality_abi_checks() {
  int32_t perm[8], applied = -1;
  const int64_t rp_dec[4] = {0, 3, 1, 4}, rp_start[4] = {1, 2, 3, 4}, rp_ok[4] = {0, 2, 3, 4};
  const int32_t col_ok[4] = {1, 2, 0, 0}, col_neg[4] = {-1, 2, 0, 0}, col_big[4] = {1, 9, 0, 0},
                col_desc[4] = {2, 1, 0, 0};
  CHECK(tpl_locality_order(3, rp_dec, col_ok, 0, 0, perm, &applied) == TPL_ERR_INVALID_ARGUMENT,
        "decreasing row_ptr accepted");
  CHECK(tpl_locality_order(3, rp_start, col_ok, 0, 0, perm, &applied) == TPL_ERR_INVALID_ARGUMENT,
        "row_ptr[0] != 0 accepted");
  CHECK(tpl_locality_order(3, rp_ok, col_neg, 0, 0, perm, &applied) == TPL_ERR_INVALID_ARGUMENT,
        "negative column accepted");
  CHECK(tpl_locality_order(3, rp_ok, col_big, 0, 0, perm, &applied) == TPL_ERR_INVALID_ARGUMENT,
        "column >= n accepted");
  CHECK(tpl_locality_order(3, rp_ok, col_desc, 0, 0, perm, &applied) == TPL_ERR_INVALID_ARGUMENT,
        "descending columns accepted");
  CHECK(tpl_locality_order(3, rp_ok, nullptr, 0, 0, perm, &applied) == TPL_ERR_INVALID_ARGUMENT,
        "NULL columns accepted");
  CHECK(tpl_locality_order(3, rp_ok, col_ok, 0, 0, perm, &applied) == TPL_OK, "valid CSR: %s",
        tpl_last_error());
  std::mt19937_64 rng(77);
  int accepted = 0;
  for (int it = 0; it < 300; ++it) {
    std::vector<int32_t> rp32, col;
    std::vector<double> val;
    const int64_t n = 2 + (int64_t)(rng() % 400);
    random_csr(n, (int)(rng() % 3), 40 + (int)(rng() % 100), rng(), rp32, col, val);
    std::vector<int64_t> rp(rp32.begin(), rp32.end());
    const int kind = (int)(rng() % 4);  // 0: none, 1: row_ptr, 2: column value, 3: swap
    if (kind == 1) rp[1 + rng() % n] += (int64_t)(rng() % 7) - 3;
    if (kind == 2 && !col.empty()) col[rng() % col.size()] = (int32_t)(rng() % (3 * n)) - (int32_t)n;
    if (kind == 3 && col.size() > 1) {
      const size_t q = rng() % (col.size() - 1);
      std::swap(col[q], col[q + 1]);
    }
    if (rp[n] > (int64_t)col.size()) continue;  // row_ptr[n] is the caller's nnz: keep it readable
    std::vector<int32_t> pm(n, -1);
    const tpl_status st = tpl_locality_order(n, rp.data(), col.empty() ? nullptr : col.data(), 0,
                                             (int)(rng() % 20), pm.data(), &applied);
    CHECK(st == TPL_OK || st == TPL_ERR_INVALID_ARGUMENT, "mutation %d: status %d", it, (int)st);
    if (st != TPL_OK) continue;
    ++accepted;
    std::vector<char> seen(n, 0);
    bool ok = true;
    for (int64_t i = 0; ok && i < n; ++i) ok = pm[i] >= 0 && pm[i] < n && !seen[pm[i]]++;
    CHECK(ok, "mutation %d: not a permutation", it);
  }
  CHECK(accepted > 50, "only %d valid mutations", accepted);
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::printf("usage: sanitize_driver <dmx> <qfc> <scratch dir>\n");
    return 2;
  }
  loader_checks(argv[1], argv[2], argv[3]);
  ftk_checks();
  layout_checks();
  locality_abi_checks();
  std::printf("%s (%d failures)\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
