// tpl_layout.h — the SpMV layout of an operator (host side): short rows as sliced ELL,
// long rows cut into column slices and packed into bins (tpl_device.h describes the
// device view). Pure host code, built by tpl_layout.cpp; the runtime uploads the result.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

#include "tpl_device.h"

namespace tpl {

struct SchedParams {
  int short_row_max = -1;           // rows longer than this are sliced; -1 = auto
  int max_g2 = 1024;                // element-wise workgroups (== #norm partials)
  int64_t long_from = -1;           // >= 0: rows [long_from, n) are long, the rest short
  bool compress_values = true;      // int8 values when all values are small integers
  bool compress_cols = true;        // uint16 column offsets when the spans allow
  int slices = 0;                   // long-row column slices (1, 2, 4, 8); 0 = auto
  bool window = true;               // stage the short chunks' column window in LDS
  int order_groups = 16;            // locality order: long-row rank groups (tpl_layout.h)
  int elem_rows = 0;                // rows per element-wise workgroup (multiple of 512;
                                    // 0: kElemRows)
  int bin_lines = 0;                // > 0: also close a bin once its gathers would touch
                                    // more than this many distinct 128-B lines (lab)
  int bin_segs = 0;                 // > 0: at most this many pieces per bin (0: kBinSegs)
  int bin_big = 0;                  // > 0: at most this many pieces longer than kBigPiece
                                    // per bin (their 16-lane sums run kTPB / 16 per pass)
  int bin_small = 0;                // > 0: at most this many other pieces per bin (their
                                    // 8-lane sums run kTPB / 8 per pass)
  int bin_balance = 2;              // bins per slice after the first fit (tpl_layout.cpp):
                                    // 0 the first fit, 1 the cost-balanced contiguous cut
                                    // (lab; measured slower), 2 the first fit with its
                                    // lightest bins on the crowded CU positions (default)
  double bin_crowd = 1.0;           // bin_balance 1: cost cap of a crowded position / of
                                    // the others
};

// Host copy of the SpMV layout (tpl_device.h).
struct Layout {
  std::vector<int32_t> srows;       // short rows, ascending
  std::vector<int32_t> s_col;       // sliced ELL entries (col = -1: padding)
  std::vector<double> s_val;
  std::vector<int32_t> c_base, c_width;
  int32_t s_width = 0;              // uniform chunk width (0: per-chunk)
  int32_t s_identity = 0;
  std::vector<int32_t> lrows;       // long rows, ascending
  std::vector<int32_t> b_col;       // long-row bins: n_bins x bin_cap entries
  std::vector<double> b_val;
  bool val_i8 = false;              // every value a small integer: stored as int8
  std::vector<int8_t> s_val8, b_val8;
  bool s_col16 = false, b_col16 = false;  // uint16 column offsets from a per-chunk/bin base
  std::vector<uint16_t> s_col16v, b_col16v;
  std::vector<int32_t> s_cbase, b_cbase;
  int32_t nslices = 1;              // column slices of the long rows
  std::vector<BinSeg> b_seg;        // n_bins x kTPB table slots
  std::vector<int32_t> b_hdr;       // per bin: pieces | long pieces << 16
  int32_t bin_cap = kBinMin;
  int32_t M = 0;                    // bins per slice
  int G2 = 1;
  int64_t E = 512;
  int32_t s_win = 0, s_win_max = 0;  // short-chunk column window (tpl_device.h)
};

// Column index as stored on the device: the identity on one GPU; with the rows
// partitioned over ranks, global column c (owned by rank r, rows [starts[r],
// starts[r+1])) lives at r * ld + (c - starts[r]) of the all-gathered vector.
// Halo-exchange row blocks: an explicit table (global column -> position in
// [own block | nranks x halo slots]).
struct ColMap {
  const std::vector<int64_t>* starts = nullptr;  // row partition (nullptr: see table)
  int64_t ld = 0;
  const std::vector<int32_t>* table = nullptr;   // halo partition
  int32_t operator()(int32_t c) const {
    if (table) return (*table)[c];
    if (!starts) return c;
    const auto it = std::upper_bound(starts->begin(), starts->end(), (int64_t)c);
    const int64_t r = (it - starts->begin()) - 1;
    return (int32_t)(r * ld + (c - (*starts)[r]));
  }
};

// Device order of the entry arrays (tpl_device.h kPackedEntries): the device index of
// canonical entry i of the bins (bin_cap entries per bin) / of the sliced-ELL chunks of
// uniform width W (packed_chunk_width(W)).
inline int64_t packed_bin_index(int64_t i, int32_t bin_cap) {
  const int64_t bin = i / bin_cap, off = i % bin_cap;
  const int64_t u0 = off / kBinMin * kBinMin, r = off % kBinMin;
  return bin * bin_cap + u0 + (r % kTPB) * kBinBatch + r / kTPB;
}
inline int64_t packed_chunk_index(int64_t i, int32_t W) {
  const int64_t per = (int64_t)W * kChunkRows, c = i / per, off = i % per;
  const int64_t k = off / kChunkRows, p = off % kChunkRows, q = p / kTPB, t = p % kTPB;
  return c * per + t * (kRowsPerThread * W) + q * W + k;
}
// v (canonical order) in the device order idx(i).
template <class T, class Idx>
std::vector<T> to_device_order(const std::vector<T>& v, Idx idx) {
  std::vector<T> out(v.size());
  for (size_t i = 0; i < v.size(); ++i) out[(size_t)idx((int64_t)i)] = v[i];
  return out;
}

// Short-row threshold: requested (> 0), or the auto rule T = clamp(2 * median row nnz,
// 4, kShortRowMax).
int32_t short_row_threshold(int64_t n, const std::vector<int32_t>& rp, int requested);

// Locality order of the rows (an internal symmetric permutation, single-GPU operators):
// perm[i] = the caller's row placed at internal position i, or an empty vector when
// the order would not change (no long rows). Short rows first, keyed by the long
// columns they reference — (tail, group(lo), group(hi), rank(lo), rank(hi), row) with
// lo / hi the smallest / largest referenced long column, rank = its position among the
// long rows, group = rank / ceil(n_long / G) (G = SchedParams::order_groups, 16 by
// default; tpl_op_tune_order tries others), and tail = 1 for rows that also
// reference another short row (they go last, next to the long columns, so the chunks
// that hold them keep the narrow column spans of uint16 columns and the LDS window) —
// then the long rows, ascending. For the
// KKT matrices this orders the arcs by (endpoint group, endpoint group, endpoints):
// the arcs of each node then lie in a few compact runs, so the long-row bins' gathers
// of a node's arcs hit lines their neighbours have just fetched.
std::vector<int32_t> locality_order(int64_t n, const std::vector<int32_t>& rp,
                                    const std::vector<int32_t>& col, const SchedParams& sp);

// The locality order's sort of short rows (shared by locality_order and the replicated
// partition's per-rank order, tpl_dist_op_create_replicated): `rows` (indices into the
// CSR rp / col, columns ascending per row) are sorted by the key above, given lrank[c] =
// the rank of column c among the n_long long rows (-1: a short row) and G groups.
template <class RowPtr, class Row>
void locality_sort(std::vector<Row>& rows, const RowPtr* rp, const int32_t* col,
                   const int32_t* lrank, int32_t n_long, int32_t G) {
  const int32_t gsize = (n_long + std::max(1, G) - 1) / std::max(1, G);  // ranks per group
  struct Key {
    int32_t tail, glo, ghi, rlo, rhi;
    Row row;
  };
  std::vector<Key> keys;
  keys.reserve(rows.size());
  for (const Row i : rows) {
    int32_t lo = INT32_MAX, hi = INT32_MAX;  // no long reference: after the others
    int32_t tail = 0;
    for (RowPtr q = rp[i]; q < rp[i + 1]; ++q) {
      const int32_t r = lrank[col[q]];
      if (r < 0) {
        tail |= (Row)col[q] != i;  // references another short row
        continue;
      }
      if (lo == INT32_MAX) lo = r;
      hi = r;  // columns ascend and ranks follow the row order
    }
    auto grp = [&](int32_t r) { return r == INT32_MAX ? INT32_MAX : r / gsize; };
    keys.push_back(Key{tail, grp(lo), grp(hi), lo, hi, i});
  }
  std::sort(keys.begin(), keys.end(), [](const Key& x, const Key& y) {
    if (x.tail != y.tail) return x.tail < y.tail;
    if (x.glo != y.glo) return x.glo < y.glo;
    if (x.ghi != y.ghi) return x.ghi < y.ghi;
    if (x.rlo != y.rlo) return x.rlo < y.rlo;
    if (x.rhi != y.rhi) return x.rhi < y.rhi;
    return x.row < y.row;
  });
  for (size_t p = 0; p < keys.size(); ++p) rows[p] = keys[p].row;
}
// P A P^T in CSR: internal row i = the caller's row perm[i], columns mapped through
// iperm (the inverse) and re-sorted ascending.
void permute_csr(int64_t n, const std::vector<int32_t>& rp, const std::vector<int32_t>& col,
                 const std::vector<double>& val, const std::vector<int32_t>& perm,
                 const std::vector<int32_t>& iperm, std::vector<int32_t>& prp,
                 std::vector<int32_t>& pcol, std::vector<double>& pval);

// Throws tpl::Error (TPL_ERR_INVALID_ARGUMENT) unless row_ptr (n + 1 entries) starts at
// 0 and is monotone, col_idx is non-NULL when row_ptr[n] > 0, and every row's columns lie
// in [0, n_cols) strictly ascending.
void check_csr(int64_t n, int64_t n_cols, const int64_t* row_ptr, const int32_t* col_idx);

// Element-wise workgroups of an operator of n rows (build_layout's rule): G2 blocks of E
// rows each. Every rank of a partition can compute every other rank's count.
void elem_geometry(int64_t n, const SchedParams& sp, int32_t& G2, int64_t& E);

// n: rows of this operator (this rank's block); n_glob: columns of A (slice bounds are
// taken on global column indices, so a partition of one rank reproduces the single-GPU
// layout exactly). Throws tpl::Error (TPL_ERR_UNSUPPORTED) for layouts the device
// kernels cannot hold.
Layout build_layout(int64_t n, int64_t n_glob, const std::vector<int32_t>& rp,
                    const std::vector<int32_t>& col, const std::vector<double>& val,
                    const SchedParams& sp, const ColMap& cmap);

} // namespace tpl
