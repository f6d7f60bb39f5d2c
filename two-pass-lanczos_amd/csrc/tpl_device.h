// tpl_device.h — structures shared by the HIP kernels (tpl_kernels.hip) and the
// host runtime (tpl_runtime.cpp). Everything here is plain data: the kernels take
// these structs by value as kernel arguments.
//
// SpMV layout (built once per operator, tpl_runtime.cpp build_layout):
//   * SHORT rows (<= T nnz, T = clamp(2 * median row nnz, 4, kShortRowMax) unless
//     set explicitly), taken in ascending order, are stored as sliced ELL: chunk c
//     holds short-row positions [C*c, C*c + C) (C = kChunkRows); entry k of position
//     p sits at chunk_base[c] + k*C + (p - C*c) (column-major inside the chunk,
//     padded to the chunk's widest row with col = -1). One workgroup per chunk,
//     thread t owns positions C*c + t + 256q: every load is coalesced and no row
//     pointer is chased. When every chunk has the same width W the chunk bases are
//     computed, not loaded, and the kernel is specialised for W.
//   * LONG rows are cut into S column slices [floor(n*s/S), floor(n*(s+1)/S)), S in
//     {1, 2, 4, 8} (tpl_runtime.cpp auto_slices: the fewest whose share of the
//     gathered vector fits an eighth of an L2). The (row, slice) pieces of slice s that
//     hold entries (a row with none keeps its slice-0 piece), long rows ascending, are
//     packed whole into BINS of bin_cap entries (padding
//     col = -1) with at most kBinSegs pieces each; every slice gets the same number
//     M of bins. Bin m of slice s is workgroup S*m + s of the slice part of the
//     grid: under the round-robin dispatch of workgroups to XCDs the bins of a slice
//     run on 8/S XCDs, whose L2s then only cache 1/S of the gathered vector (speed
//     only, never correctness). A bin's entries are read at computed addresses
//     (thread t: entries t + 256u), the products are staged in LDS, and each piece
//     is summed by 8 lanes (by a whole wave when longer than kBigPiece; those
//     pieces lead the table). A row with one packed piece (always with S = 1) is
//     finished in place by that piece's thread. Otherwise every piece sum is published
//     write-through into the row's slot (the slots of unpacked pieces are never written:
//     they hold the +0.0 an empty piece sums to); after its store drains, the publisher
//     increments the row's arrival counter (agent-scope atomic_inc wrapping at the row's
//     packed-piece count, BinSeg::pad), and the one whose increment returns the row's last
//     count reads the S slots and finalises the row (sums the slots, runs the epilogue).
//     Nobody waits on anybody.
//
// Canonical reduction order (reproduced bit for bit by oracle/lanczos_oracle.c):
//   * tree256(a[256])  : per 64-lane wave an xor butterfly (offsets 1,2,4,8,16,32,
//                        a_l <- a_l + a_{l^off}), then (S0 + S1) + (S2 + S3).
//   * partials(P[N])   : thread t: s_t = 0; s_t += P[t + 256q] (q ascending); tree256.
//   * short row        : s = 0; s += round(a_k x_k), k ascending.
//   * long row         : per slice s, its L entries form a piece. L <= kBigPiece: lane
//                        g (0..7): p_g = 0; p_g += round(a_k x_k) for the piece's
//                        entries k = g + 8q (q ascending); P_s = xor butterfly of p over
//                        8 lanes (offsets 1, 2, 4). L > kBigPiece: the same with 16
//                        lanes (k = g + 16q) and a 16-lane butterfly (1, 2, 4, 8).
//                        y = 0; y += P_s, s = 0..S-1.
//   * alpha partials   : Pa[c] (short chunk c): thread t: acc = fma(v, w, acc) over its
//                        positions C*c + t + 256q (q ascending), tree256 (C = kChunkRows);
//                        Pa[n_chunks + r] (long row r) = round(v * w).
//                        alpha = partials(Pa[0 .. n_chunks + n_long)).
//   * norm partial     : workgroup b (of G2) owns [bE, min(n,(b+1)E)); thread t visits
//                        i0 = bE + 2t + 512q, then i0, i0+1: acc = fma(x,x,acc); tree256.
#pragma once
#include <stdint.h>

namespace tpl {

constexpr int kTPB = 256;            // threads per workgroup (4 waves of 64)
#ifndef TPL_CHUNK_ROWS
#define TPL_CHUNK_ROWS 512
#endif
constexpr int kChunkRows = TPL_CHUNK_ROWS; // short-row positions per SELL chunk
constexpr int kRowsPerThread = kChunkRows / kTPB;
#ifndef TPL_ELEM_ROWS
#define TPL_ELEM_ROWS 2048
#endif
// rows per workgroup of the element-wise kernels (k_p1_axpy, ...): G2 = ceil(n / this)
// workgroups, a multiple of kChunkRows (chunk_of_block keeps a chunk on its element
// block's XCD). 2048 at 500k arcs: k_p1_axpy 3.97 us vs 4.24 at 1024 (each workgroup
// re-reduces the ~2.1k alpha partials; fewer workgroups, less of that), 4.94 at 4096
// (too few workgroups to stream); solve 12.58 vs 12.69 ms.
constexpr int kElemRows = TPL_ELEM_ROWS;
constexpr int kElemMinBlocks = 192;  // below this many blocks, kElemRows is halved (to 512)
constexpr int kShortRowMax = 32;     // upper bound of the short-row threshold
#ifndef TPL_MAX_SLICES
#define TPL_MAX_SLICES 8
#endif
constexpr int kSlices = TPL_MAX_SLICES;  // most column slices of a long row (8 = XCDs)
#ifndef TPL_SLOT_STRIDE
#define TPL_SLOT_STRIDE TPL_MAX_SLICES
#endif
constexpr int kSlotStride = TPL_SLOT_STRIDE;  // doubles between two long rows' slot arrays
constexpr int kBinSegs = kTPB - 1;   // pieces per bin (+1 end marker = kTPB table slots)
// Pieces longer than this are summed by 16 lanes, the others by 8 lanes;
// the long pieces of a bin come first in its table (CsrDev::b_hdr holds their count).
constexpr int kBigPiece = 64;
#ifndef TPL_BIN_MIN
#define TPL_BIN_MIN 2048
#endif
constexpr int kBinMin = TPL_BIN_MIN; // default entries per bin
constexpr int kBinBatch = kBinMin / kTPB;  // entries per thread per load batch
// Device order of the stored entries (speed only; positions, and so every sum, are
// unchanged): the kBinBatch entries thread t reads from a bin's load batch (positions
// u0 + 256u + t) are stored consecutively at u0 + kBinBatch t + u, and the
// kRowsPerThread x W entries of a chunk of uniform width W in {1, 2, 4} (entry k of
// position C c + 256q + t) at C W c + kRowsPerThread W t + W q + k — one 16-B load of
// uint16 columns and one 8-B load of int8 values per thread instead of 16 strided
// 2-B / 1-B loads (tpl_layout.h packed_bin_index / packed_chunk_index).
#ifndef TPL_PACKED_ENTRIES
#define TPL_PACKED_ENTRIES 1
#endif
constexpr bool kPackedEntries = TPL_PACKED_ENTRIES != 0;
constexpr bool packed_chunk_width(int w) { return kPackedEntries && (w == 1 || w == 2 || w == 4); }
constexpr int kLongEpiRows = kTPB;  // one replicated long row per thread (k_long_epi_*)
constexpr int kPbRanks = 8;          // most ranks whose norm partials k_p1_spmv reduces itself
constexpr int kWinMax = 2048;        // short-chunk column window in LDS: at most this many columns
constexpr int kWinLoads = kWinMax / 256;  // window loads per thread
constexpr int kBinMax = 7936;        // LDS bound: 62 KiB of staged products (+1 KiB starts)
// Arrival counters of the sliced long rows: one uint32 per row, kCntStride apart (one
// 64-B segment each, so the atomics of different rows never share a segment).
constexpr int kCntStride = 16;
constexpr double kBreakdownTol = 2.220446049250313080847263336181640625e-13; // 1000*f64::EPSILON, src/algorithms/mod.rs:140-143

// One bin-table slot: piece start (offset in the bin), long-row index, global row, and
// the row's packed pieces - 1 (its last arrival count; 0: the piece is the whole row).
// Slot j < pieces describes piece j (its end is slot j+1's start); the slot after
// the last piece holds the bin's fill with ri = row = -1, and so do all later slots.
// x terms pass-two step j (1 .. last) applies (EpiPass2): the terms pending since the
// previous flush, at every third step and at the last one.
inline int p2_flush(int j, int last) {
  return (j % 3 == 0 || j == last) ? j - ((j - 1) / 3) * 3 : 0;
}

struct BinSeg {
  int32_t start, ri, row, pad;
};

// Device view of the operator plus its layout.
struct CsrDev {
  // short rows: sliced ELL
  const int32_t* srows;     // n_short short-row indices (ascending); unused if s_identity
  const void* s_col;        // padded entries: int32 (col = -1 for padding), or uint16
                            // offsets from s_cbase[chunk] (0xFFFF padding) when s_col16
  const int32_t* s_cbase;   // per-chunk column base (s_col16)
  const void* s_val;        // double, or int8_t when val_i8
  const int32_t* c_base;    // n_chunks chunk base offsets; unused if s_width > 0
  const int32_t* c_width;   // n_chunks chunk widths; unused if s_width > 0
  // long rows: bins (bin b = 8m + s holds pieces of slice s)
  const void* b_col;        // n_bins x bin_cap entries: int32 (-1: padding), or uint16
                            // offsets from b_cbase[bin] (0xFFFF padding) when b_col16
  const int32_t* b_cbase;   // per-bin column base (b_col16)
  const void* b_val;        // double, or int8_t when val_i8
  const BinSeg* b_seg;      // n_bins x kTPB table slots (pieces, then the end marker)
  const int32_t* b_hdr;     // per bin: number of pieces | long pieces (first) << 16
  double* P;                // n_long x kSlices piece partials (slot s: slice s)
  unsigned int* Pcnt;       // n_long arrival counters, kCntStride apart (never reset)
  int32_t val_i8;           // 1: every stored value is a small integer, kept as int8
  int32_t s_col16;          // 1: chunk columns as uint16 offsets
  int32_t b_col16;          // 1: bin columns as uint16 offsets
  int32_t s_width;          // > 0: every chunk has this width (bases computed)
  int32_t s_identity;       // 1: short rows are exactly 0 .. n_short-1
  int32_t n_short;
  int32_t n_chunks;
  int32_t n_long;
  int32_t bin_cap;          // entries per bin (multiple of kTPB)
  int32_t n_slice_blocks;   // n_slices * M; SpMV grid = n_chunks + n_slice_blocks
  int32_t G2;               // workgroups of the element-wise kernels == #norm partials
  int32_t NA;               // #alpha partials = n_chunks + n_long
  int32_t NA_r;             // #alpha partials the reducing kernel reads (NA, or more, see DevState)
  int32_t G2_r;             // #norm partials the reducing kernel reads (G2, or #ranks)
  int32_t pb_ld;            // > 0 (replicated partition, round 6): Pb_r holds every rank's
                            // G2 norm partials, pb_ld apart (zero-padded), all-gathered;
                            // k_p1_spmv reduces each rank's to its total itself (no
                            // rank-total launch). 0: Pb_r holds G2_r partials / totals
  int32_t n_slices;         // column slices of the long rows (1, 2, 4 or 8 <= kSlices)
  int64_t n;
  int64_t E;                // elements per workgroup of the element-wise kernels
  // Replicated-long-row partition (tpl_runtime.cpp, "hybrid"): the SpMV stores each
  // long row's rank-local partial in ypart[ri] instead of finishing the row, and the
  // norm partials cover elements [0, norm_n) only (replicated entries count once).
  double* ypart;            // n_long partials of this rank (own slice of the all-gather)
  int32_t long_defer;       // 1: long rows deferred to k_long_epi_*
  int32_t y_ld;             // stride of the all-gathered segments. Pass one: n_long
                            // partials + the rank's short-chunk alpha partials
                            // (yall[r * y_ld + n_long + c], nch[r] of them); pass two and
                            // the plain product: n_long + 1
  const int32_t* nch;       // chunk (alpha partial) count of every rank (hybrid)
  int64_t norm_n;           // == n except on ranks that do not own the replicated rows
  // Short-chunk column window (s_win > 0: every chunk's columns lie in [cbase, cbase +
  // s_win), s_win <= kWinMax; the window is staged in LDS). s_win_max: the largest
  // column of any chunk (window loads past it are clamped there).
  int32_t s_win;
  int32_t s_win_max;
};

// Device-resident solver state (one per operator).
constexpr int kFlagBytes = 32;       // DevState::flags: 8 int32
struct DevState {
  int32_t* flags;   // [0] stop, [1] error (1 = zero b), [2] steps_taken, [3] second
                    // Gram-Schmidt passes, [4] device f(T_k) handed back to the host,
                    // [5] rows of T_k's LU eliminated during pass one (k_p1_axpy)
  double* norms;    // [0] = ||b||, [j] = beta_j                         (kcap+1)
  double* alphas;   // alphas[j-1] = alpha_j                              (kcap)
  double* betas;    // betas[j-1]  = beta_j                               (kcap)
  double* y;        // pass-two coefficients y_k (already * ||b||), or y' (kcap)
  double* p2c;      // pass-two step records, 8 doubles per step (k_p2_coefs, EpiPass2R)
  double* lu;       // T_k's LU built during pass one (one-graph inv): D | DU | DU2 | B
                    // (kcap each), then the running row (d, du, b)        (4 kcap + 3)
  int32_t kcap;     // capacity of the k-sized arrays
  double* Pa;       // alpha partials (NA) — written by this rank's kernels
  double* Pb;       // ||.||^2 partials (G2)
  // What the reducing kernels read: Pa / Pb on one GPU; with the rows partitioned
  // over R ranks, the R per-rank totals (each = partials() of that rank's Pa / Pb),
  // all-gathered in rank order.
  const double* Pa_r;
  const double* Pb_r;
};

} // namespace tpl
