// tpl_layout.cpp — builds the SpMV layout of an operator (tpl_layout.h). Host only.
#include "tpl_layout.h"

#include <algorithm>
#include <cmath>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "tpl_internal.h"

namespace tpl {

// Column slices of the long rows (auto rule): the fewest (1, 2, 4, 8) whose share of
// the gathered vector fits in an eighth of an XCD's 4 MiB L2 (measured at 500k arcs with
// the arrival-counter hand-off: 8 slices 11.91 ms per k = 500 solve, 4 slices 12.23, 2
// slices 13.61; at 50k: 1 slice 7.1 ms, 2 slices 9.1) — slice s runs on the XCDs
// b % 8 == s (mod slices), so each L2 caches only its slice's columns — and, when a
// (row, slice) piece would exceed one bin, more slices until every piece fits.
static int auto_slices(int64_t n_cols) {
  int s = 1;
  while (s < kSlices && (double)n_cols * 8.0 / s > 0.5 * 1024.0 * 1024.0) s *= 2;
  return s;
}


// Auto rule: T = clamp(2 * median row length, 4, kShortRowMax). A sliced-ELL chunk
// costs as much as its widest row, so the few rows far above the typical length
// (e.g. the short node rows of a KKT matrix) go to the sliced long-row path instead
// of widening a chunk.
int32_t short_row_threshold(int64_t n, const std::vector<int32_t>& rp, int requested) {
  if (requested > 0) return requested;
  if (n == 0) return kShortRowMax;
  std::vector<int32_t> hist(kShortRowMax + 2, 0);
  for (int64_t i = 0; i < n; ++i) hist[std::min<int32_t>(rp[i + 1] - rp[i], kShortRowMax + 1)]++;
  int64_t seen = 0;
  int32_t median = kShortRowMax + 1;
  for (int32_t l = 0; l <= kShortRowMax + 1; ++l) {
    seen += hist[l];
    if (2 * seen >= n) {  // lower median
      median = l;
      break;
    }
  }
  return std::max<int32_t>(4, std::min<int32_t>(kShortRowMax, 2 * median));
}

std::vector<int32_t> locality_order(int64_t n, const std::vector<int32_t>& rp,
                                    const std::vector<int32_t>& col, const SchedParams& sp) {
  const int32_t T = short_row_threshold(n, rp, sp.short_row_max);
  std::vector<int32_t> rank(n, -1);  // long row -> its rank among the long rows
  int32_t n_long = 0;
  for (int64_t i = 0; i < n; ++i) {
    const bool is_long = sp.long_from >= 0 ? i >= sp.long_from : rp[i + 1] - rp[i] > T;
    if (is_long) rank[i] = n_long++;
  }
  if (n_long == 0) return {};
  std::vector<int32_t> perm;
  perm.reserve(n);
  for (int64_t i = 0; i < n; ++i)
    if (rank[i] < 0) perm.push_back((int32_t)i);
  locality_sort(perm, rp.data(), col.data(), rank.data(), n_long, sp.order_groups);
  for (int64_t i = 0; i < n; ++i)
    if (rank[i] >= 0) perm.push_back((int32_t)i);
  bool identity = true;
  for (int64_t i = 0; i < n && identity; ++i) identity = perm[i] == i;
  if (identity) return {};
  return perm;
}

void permute_csr(int64_t n, const std::vector<int32_t>& rp, const std::vector<int32_t>& col,
                 const std::vector<double>& val, const std::vector<int32_t>& perm,
                 const std::vector<int32_t>& iperm, std::vector<int32_t>& prp,
                 std::vector<int32_t>& pcol, std::vector<double>& pval) {
  prp.assign(1, 0);
  pcol.clear();
  pval.clear();
  pcol.reserve(col.size());
  pval.reserve(val.size());
  std::vector<std::pair<int32_t, double>> row;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t e = perm[i];
    row.clear();
    for (int32_t q = rp[e]; q < rp[e + 1]; ++q) row.emplace_back(iperm[col[q]], val[q]);
    std::sort(row.begin(), row.end(),
              [](const std::pair<int32_t, double>& a, const std::pair<int32_t, double>& b) {
                return a.first < b.first;
              });
    for (const auto& x : row) {
      pcol.push_back(x.first);
      pval.push_back(x.second);
    }
    prp.push_back((int32_t)pcol.size());
  }
}

Layout build_layout(int64_t n, int64_t n_glob, const std::vector<int32_t>& rp,
                           const std::vector<int32_t>& col, const std::vector<double>& val,
                           const SchedParams& sp, const ColMap& cmap) {
  Layout L;
  const int32_t T = short_row_threshold(n, rp, sp.short_row_max);
  for (int64_t i = 0; i < n; ++i) {
    if (sp.long_from >= 0 ? i >= sp.long_from : rp[i + 1] - rp[i] > T) L.lrows.push_back((int32_t)i);
    else L.srows.push_back((int32_t)i);
  }
  const int64_t ns = (int64_t)L.srows.size();
  L.s_identity = 1;
  for (int64_t p = 0; p < ns; ++p)
    if (L.srows[p] != p) {
      L.s_identity = 0;
      break;
    }
  const int64_t nchunks = (ns + kChunkRows - 1) / kChunkRows;
  L.c_base.resize(nchunks);
  L.c_width.resize(nchunks);
  int64_t total = 0;
  for (int64_t c = 0; c < nchunks; ++c) {
    int32_t w = 0;
    for (int64_t p = c * kChunkRows; p < std::min(ns, (c + 1) * kChunkRows); ++p)
      w = std::max<int32_t>(w, rp[L.srows[p] + 1] - rp[L.srows[p]]);
    L.c_base[c] = (int32_t)total;
    L.c_width[c] = w;
    total += (int64_t)w * kChunkRows;
  }
  if (total >= INT32_MAX) fail(TPL_ERR_UNSUPPORTED, "sliced-ELL storage exceeds 2^31 entries");
  L.s_col.assign(std::max<int64_t>(total, 1), -1);
  L.s_val.assign(std::max<int64_t>(total, 1), 0.0);
  for (int64_t c = 0; c < nchunks; ++c)
    for (int64_t p = c * kChunkRows; p < std::min(ns, (c + 1) * kChunkRows); ++p) {
      const int32_t r = L.srows[p];
      for (int32_t k = 0; k < rp[r + 1] - rp[r]; ++k) {
        const int64_t e = L.c_base[c] + (int64_t)k * kChunkRows + (p - c * kChunkRows);
        L.s_col[e] = cmap(col[rp[r] + k]);
        L.s_val[e] = val[rp[r] + k];
      }
    }
  L.s_width = 0;
  if (nchunks > 0) {
    bool uni = true;
    for (int64_t c = 0; c < nchunks; ++c) uni = uni && L.c_width[c] == L.c_width[0];
    if (uni && L.c_width[0] > 0) L.s_width = L.c_width[0];
  }
  const size_t nl = L.lrows.size();
  // Long rows: piece (r, s) = entries of long row r with columns in slice s (columns
  // [n_glob s / S, n_glob (s+1) / S)); the pieces of slice s, r ascending, are packed
  // whole into bins (first fit in order).
  const size_t nlb = nl;
  int S = sp.slices > 0 ? sp.slices : auto_slices(n_glob);
  std::vector<int32_t> poff;
  int32_t widest = 0;
  auto cut = [&](int ns) {
    poff.assign(nlb * (ns + 1), 0);
    widest = 0;
    for (size_t r = 0; r < nlb; ++r) {
      const int32_t row = L.lrows[r];
      int32_t q = rp[row];
      for (int s = 0; s <= ns; ++s) {
        const int64_t bound = n_glob * s / ns;
        while (q < rp[row + 1] && col[q] < bound) ++q;
        poff[r * (ns + 1) + s] = (s == ns) ? rp[row + 1] : q;
        if (s > 0) widest = std::max(widest, poff[r * (ns + 1) + s] - poff[r * (ns + 1) + s - 1]);
      }
    }
  };
  cut(S);
  while (widest > kBinMax && sp.slices <= 0 && S < kSlices) cut(S *= 2);
  if (widest > kBinMax)
    fail(TPL_ERR_UNSUPPORTED, "a long row has " + std::to_string(widest) +
                                  " nonzeros in one of its " + std::to_string(S) +
                                  " column slices (limit " + std::to_string(kBinMax) + ")");
  L.nslices = S;
  L.bin_cap = std::max<int32_t>(kBinMin, ((widest + kTPB - 1) / kTPB) * kTPB);
  L.bin_cap = ((L.bin_cap + kBinMin - 1) / kBinMin) * kBinMin;  // whole load batches
  std::vector<std::vector<std::vector<std::pair<int32_t, int32_t>>>> bins(S); // (r, fill-at-start)
  std::vector<std::vector<int32_t>> fill(S);
  const int segs = sp.bin_segs > 0 && sp.bin_segs < kBinSegs ? sp.bin_segs : kBinSegs;
  // Only the pieces with entries are packed (a row's empty pieces would only publish
  // +0.0, which its never-written slot already holds; a row with no entries at all keeps
  // its slice-0 piece); pieces_of[r] = the row's packed pieces, its arrival count.
  std::vector<int32_t> pieces_of(nlb, 0);
  for (size_t r = 0; r < nlb; ++r) {
    for (int s = 0; s < S; ++s)
      pieces_of[r] += poff[r * (S + 1) + s + 1] > poff[r * (S + 1) + s];
    pieces_of[r] = std::max(pieces_of[r], 1);
  }
  // Distinct 128-B lines of the gathered vector a bin touches, counted with stamps: line l
  // belongs to the open bin when bstamp[l] == its epoch, to the piece being weighed when
  // pstamp[l] == the piece's epoch (epochs only grow, so nothing is ever reset).
  int64_t max_line = 0;
  for (size_t r = 0; r < nlb; ++r)
    for (int32_t q = poff[r * (S + 1)]; q < poff[r * (S + 1) + S]; ++q)
      max_line = std::max<int64_t>(max_line, cmap(col[q]) >> 4);
  std::vector<int32_t> bstamp(nlb > 0 ? max_line + 1 : 0, -1), pstamp(bstamp.size(), -1);
  int32_t bin_epoch = -1, piece_epoch = -1;
  // Bin packing of slice s: its pieces in row order, cut into contiguous runs (a run of
  // consecutive rows keeps the locality order's shared lines in one bin). A bin closes
  // when the next piece would overflow its entries (bin_cap) or pieces (segs), a lab cap,
  // or — cost >= 0 — the bin's predicted cost. The cost model (fitted to the per-bin
  // end times of round-5 stamp timelines, scripts/lab/bin_cost.py: end ≈ 3.1 µs + 0.41 µs
  // per piece-sum round + 1.8 ns per distinct line) in line units: kRoundCost per round
  // of the wave tasks (long_bin: ceil(big / 4) + ceil(small / 8) tasks, 4 per round) plus
  // the lines.
  constexpr int64_t kRoundCost = 228;
  auto rounds = [](int32_t nbig, int32_t nsmall) {
    return (int64_t)(((nbig + 3) / 4 + (nsmall + 7) / 8 + 3) / 4);
  };
  // Bins that share a CU: with S = 8 the bins of slice s are XCD s's first M workgroups,
  // and a fully resident grid deals workgroup q of an XCD to CU class q mod 32
  // (scripts/lab/cu_map.hip, profiles/r02_cu_map.txt) — so when M is not a multiple of 32
  // the first M mod 32 classes hold one bin more than the others (at 500k: M = 68, classes
  // 0-3 hold three bins and three chunks, the rest two bins and four chunks). Those
  // positions m (m mod 32 < M mod 32) are "crowded"; the cut gives them a smaller cost cap
  // (crowd x the others').
  // With S = 8 TX > 8 slices an XCD runs TX slices, bin m of slice s as its workgroup
  // TX m + s mod TX (tpl_kcommon.h spmv_block_impl), TX M bins per XCD.
  constexpr int kCuClasses = 32;  // CUs per XCD (MI355X: 256 CUs / 8 XCDs)
  const int TX = S >= 8 ? S / 8 : 0;  // slices per XCD (0: S < 8, no crowding rule)
  auto crowded = [&](int32_t m, int s) {
    const int32_t Q = TX * L.M, q = TX * m + (TX > 0 ? s % TX : 0);
    return TX > 0 && Q > kCuClasses && Q % kCuClasses != 0 && q % kCuClasses < Q % kCuClasses;
  };
  auto pack = [&](int s, int64_t cost_cap, double crowd,
                  std::vector<std::vector<std::pair<int32_t, int32_t>>>& out,
                  std::vector<int32_t>& fl) {
    out.clear();
    fl.clear();
    int32_t nbig = 0, nsmall = 0;
    int64_t nlines = 0;
    // distinct lines of piece rows [q0, q1) not in the open bin (all of them: open = false)
    auto fresh_lines = [&](int32_t q0, int32_t q1, bool open) {
      int64_t f = 0;
      ++piece_epoch;
      for (int32_t q = q0; q < q1; ++q) {
        const int64_t l = cmap(col[q]) >> 4;
        if ((!open || bstamp[l] != bin_epoch) && pstamp[l] != piece_epoch) {
          pstamp[l] = piece_epoch;
          ++f;
        }
      }
      return f;
    };
    for (size_t r = 0; r < nlb; ++r) {
      const int32_t q0 = poff[r * (S + 1) + s], q1 = poff[r * (S + 1) + s + 1], cnt = q1 - q0;
      if (cnt == 0 && !(s == 0 && pieces_of[r] == 1 && poff[r * (S + 1) + S] == poff[r * (S + 1)]))
        continue;
      const bool big = cnt > kBigPiece;
      int64_t fresh = fresh_lines(q0, q1, !out.empty());
      bool close = out.empty();
      if (!close) {
        const int32_t nb = nbig + big, ns = nsmall + !big;
        close = fl.back() + cnt > L.bin_cap || (int)out.back().size() == segs ||
                (sp.bin_lines > 0 && nlines + fresh > sp.bin_lines) ||
                (big && sp.bin_big > 0 && nbig == sp.bin_big) ||
                (!big && sp.bin_small > 0 && nsmall == sp.bin_small) ||
                (cost_cap >= 0 &&
                 rounds(nb, ns) * kRoundCost + nlines + fresh >
                     (crowded((int32_t)out.size() - 1, s) ? (int64_t)(crowd * (double)cost_cap)
                                                       : cost_cap));
        if (close) fresh = fresh_lines(q0, q1, false);  // the piece against an empty bin
      }
      if (close) {
        out.emplace_back();
        fl.push_back(0);
        ++bin_epoch;
        nbig = nsmall = 0;
        nlines = 0;
      }
      for (int32_t q = q0; q < q1; ++q) bstamp[cmap(col[q]) >> 4] = bin_epoch;
      nlines += fresh;
      out.back().emplace_back((int32_t)r, fl.back());
      fl.back() += cnt;
      (big ? nbig : nsmall)++;
    }
  };
  // predicted cost of bin m of slice s (line units)
  auto bin_cost = [&](int s, const std::vector<std::pair<int32_t, int32_t>>& bin) {
    int32_t nb = 0, ns = 0;
    ++piece_epoch;
    int64_t nl = 0;
    for (const auto& p : bin) {
      const int32_t r = p.first, q0 = poff[r * (S + 1) + s], q1 = poff[r * (S + 1) + s + 1];
      (q1 - q0 > kBigPiece ? nb : ns)++;
      for (int32_t q = q0; q < q1; ++q) {
        const int64_t l = cmap(col[q]) >> 4;
        if (pstamp[l] != piece_epoch) {
          pstamp[l] = piece_epoch;
          ++nl;
        }
      }
    }
    return bin.empty() ? (int64_t)0 : rounds(nb, ns) * kRoundCost + nl;
  };
  // First fit in row order sets M, the bins per slice (the grid never grows). Then
  // (bin_balance 1) each slice is re-cut into at most M runs whose largest predicted cost
  // — on crowded positions scaled by 1 / crowd — is the smallest a contiguous cut allows
  // (the greedy cut under a cost cap uses the fewest bins for that cap, and more cap never
  // needs more bins: bisect the cap); or (bin_balance 2) the first fit's bins stay and the
  // lightest of each slice move to its crowded positions. Piece sums are per (row, slice)
  // and a row's slots are summed in slice order, so which bin holds a piece, and where
  // that bin runs, never changes a bit.
  std::vector<std::vector<std::pair<int32_t, int32_t>>> tb;
  std::vector<int32_t> tf;
  for (int s = 0; s < S && nlb > 0; ++s) pack(s, -1, 1.0, bins[s], fill[s]);
  L.M = 0;
  for (int s = 0; s < S; ++s) L.M = std::max<int32_t>(L.M, (int32_t)bins[s].size());
  for (int s = 0; s < S && nlb > 0 && sp.bin_balance == 1; ++s) {
    int64_t lo = 0, hi = 0;  // hi: a cap the first fit's cut meets on every position
    for (size_t m = 0; m < bins[s].size(); ++m) {
      const int64_t c = bin_cost(s, bins[s][m]);
      hi = std::max(hi, crowded((int32_t)m, s) ? (int64_t)std::ceil((double)c / sp.bin_crowd) + 1 : c);
    }
    while (lo < hi) {
      const int64_t mid = lo + (hi - lo) / 2;
      pack(s, mid, sp.bin_crowd, tb, tf);
      if ((int32_t)tb.size() <= L.M) hi = mid;
      else lo = mid + 1;
    }
    pack(s, hi, sp.bin_crowd, bins[s], fill[s]);
  }
  if (sp.bin_balance == 2 && nlb > 0 && TX > 0 && TX * L.M > kCuClasses &&
      (TX * L.M) % kCuClasses != 0) {
    for (int s = 0; s < S; ++s) {
      bins[s].resize(L.M);
      fill[s].resize(L.M, 0);
      std::vector<int32_t> ord(L.M);
      std::vector<int64_t> cost(L.M);
      for (int32_t m = 0; m < L.M; ++m) {
        ord[m] = m;
        cost[m] = bin_cost(s, bins[s][m]);
      }
      std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return cost[a] < cost[b]; });
      int32_t ncrowd = 0;
      for (int32_t m = 0; m < L.M; ++m) ncrowd += crowded(m, s);
      std::vector<int32_t> light(ord.begin(), ord.begin() + ncrowd), rest(ord.begin() + ncrowd, ord.end());
      std::sort(light.begin(), light.end());
      std::sort(rest.begin(), rest.end());
      std::vector<std::vector<std::pair<int32_t, int32_t>>> nb(L.M);
      std::vector<int32_t> nf(L.M);
      size_t il = 0, ir = 0;
      for (int32_t m = 0; m < L.M; ++m) {
        const int32_t from = crowded(m, s) ? light[il++] : rest[ir++];
        nb[m] = std::move(bins[s][from]);
        nf[m] = fill[s][from];
      }
      bins[s] = std::move(nb);
      fill[s] = std::move(nf);
    }
  }
  for (int s = 0; s < S; ++s) L.M = std::max<int32_t>(L.M, (int32_t)bins[s].size());
  const size_t nbins = (size_t)S * L.M;
  L.b_col.assign(std::max<size_t>(nbins * L.bin_cap, 1), -1);
  L.b_val.assign(std::max<size_t>(nbins * L.bin_cap, 1), 0.0);
  L.b_seg.assign(std::max<size_t>(nbins * kTPB, 1), BinSeg{0, -1, -1, 0});
  L.b_hdr.assign(std::max<size_t>(nbins, 1), 0);
  for (int s = 0; s < S; ++s)
    for (int32_t m = 0; m < L.M; ++m) {
      const size_t bin = (size_t)m * S + s;
      int32_t f = 0;
      if (m < (int32_t)bins[s].size()) {
        // the pieces longer than kBigPiece first (summed a wave each), then the rest;
        // entries are laid out in that table order
        auto pieces = bins[s][m];
        auto len = [&](int32_t r) {
          return poff[r * (S + 1) + s + 1] - poff[r * (S + 1) + s];
        };
        std::stable_partition(pieces.begin(), pieces.end(),
                              [&](const std::pair<int32_t, int32_t>& p) { return len(p.first) > kBigPiece; });
        int32_t nbig = 0, at = 0;
        for (auto& p : pieces) {
          nbig += len(p.first) > kBigPiece;
          p.second = at;
          at += len(p.first);
        }
        for (size_t j = 0; j < pieces.size(); ++j) {
          const int32_t r = pieces[j].first, start = pieces[j].second;
          const int32_t q0 = poff[r * (S + 1) + s], q1 = poff[r * (S + 1) + s + 1];
          L.b_seg[bin * kTPB + j] = BinSeg{start, r, L.lrows[r], pieces_of[r] - 1};
          for (int32_t q = q0; q < q1; ++q) {
            L.b_col[bin * L.bin_cap + start + (q - q0)] = cmap(col[q]);
            L.b_val[bin * L.bin_cap + start + (q - q0)] = val[q];
          }
        }
        f = fill[s][m];
        for (size_t j = pieces.size(); j < (size_t)kTPB; ++j)
          L.b_seg[bin * kTPB + j] = BinSeg{f, -1, -1, 0};
        L.b_hdr[bin] = (int32_t)pieces.size() | nbig << 16;
      }
    }
  // Value compression: when every stored value (padding included) is an integer in
  // [-128, 127] other than -0.0, keep int8 values; the device converts them back to
  // double exactly, so every product and sum keeps its bits (the KKT values are +-1).
  auto small_int = [](double v) {
    return v >= -128.0 && v <= 127.0 && v == (double)(int8_t)v && !(v == 0.0 && std::signbit(v));
  };
  L.val_i8 = sp.compress_values;
  for (double v : L.s_val) L.val_i8 = L.val_i8 && small_int(v);
  for (double v : L.b_val) L.val_i8 = L.val_i8 && small_int(v);
  if (L.val_i8) {
    L.s_val8.assign(L.s_val.begin(), L.s_val.end());
    L.b_val8.assign(L.b_val.begin(), L.b_val.end());
    std::vector<double>().swap(L.s_val);
    std::vector<double>().swap(L.b_val);
  }
  // Column compression: uint16 offsets from each chunk's / bin's smallest column when
  // every chunk / bin spans fewer than 65535 columns (0xFFFF marks padding).
  auto compress_cols = [&](const std::vector<int32_t>& cols, int64_t groups, int64_t per,
                           std::vector<uint16_t>& out16, std::vector<int32_t>& base) {
    if (!sp.compress_cols || groups == 0) return false;
    base.assign(groups, 0);
    for (int64_t g = 0; g < groups; ++g) {
      int32_t lo = INT32_MAX, hi = -1;
      for (int64_t e = g * per; e < (g + 1) * per && e < (int64_t)cols.size(); ++e)
        if (cols[e] >= 0) {
          lo = std::min(lo, cols[e]);
          hi = std::max(hi, cols[e]);
        }
      if (hi < 0) lo = hi = 0;
      if (hi - lo >= 0xFFFF) return false;
      base[g] = lo;
    }
    out16.resize(cols.size());
    for (size_t e = 0; e < cols.size(); ++e)
      out16[e] = cols[e] < 0 ? 0xFFFF : (uint16_t)(cols[e] - base[e / per]);
    return true;
  };
  // chunks have a uniform stride only when the widths are uniform (else per-chunk bases)
  if (L.s_width > 0)
    L.s_col16 = compress_cols(L.s_col, nchunks, (int64_t)L.s_width * kChunkRows, L.s_col16v, L.s_cbase);
  L.b_col16 = compress_cols(L.b_col, (int64_t)L.nslices * L.M, L.bin_cap, L.b_col16v, L.b_cbase);
  // Column window of the short chunks: every chunk's columns within kWinMax of its base
  // (uint16 columns, uniform width 1..4) -> staged in LDS.
  if (sp.window && L.s_col16 && L.s_width >= 1 && L.s_width <= 4) {
    const int64_t per = (int64_t)L.s_width * kChunkRows;
    int32_t win = 0, hi = 0;
    for (int64_t c = 0; c < nchunks; ++c)
      for (int64_t e = c * per; e < (c + 1) * per; ++e)
        if (L.s_col[e] >= 0) {
          win = std::max<int32_t>(win, L.s_col[e] - L.s_cbase[c] + 1);
          hi = std::max<int32_t>(hi, L.s_col[e]);
        }
    if (win > 0 && win <= kWinMax) {
      L.s_win = win;
      L.s_win_max = hi;
    }
  }
  if (L.s_col16) std::vector<int32_t>().swap(L.s_col);
  if (L.b_col16) std::vector<int32_t>().swap(L.b_col);
  // rows per element-wise workgroup: kElemRows, halved (down to 512) while that leaves
  // fewer than kElemMinBlocks workgroups — a small operator's element-wise kernels are
  // pure latency, and more blocks in flight hide it (measured, configs[1] 50k arcs k =
  // 200: 512 rows 2.50 ms per solve, 1024 2.52, 2048 2.54; the headline 500k: 2048 9.93,
  // 1024 9.98, 512 10.42 — profiles/r03_small_n_lab.txt)
  elem_geometry(n, sp, L.G2, L.E);
  return L;
}

void elem_geometry(int64_t n, const SchedParams& sp, int32_t& G2, int64_t& E) {
  int64_t er = kElemRows;
  if (sp.elem_rows > 0) {
    er = ((sp.elem_rows + 511) / 512) * 512;
  } else {
    while (er > 512 && (n + er - 1) / er < kElemMinBlocks) er /= 2;
  }
  const int64_t g2 = (n + er - 1) / er;
  G2 = (int)std::max<int64_t>(1, std::min<int64_t>(sp.max_g2, g2));
  const int64_t per = (n + G2 - 1) / G2;
  E = std::max<int64_t>(512, ((per + 511) / 512) * 512);
}

// The CSR rules of every entry point that takes a matrix: row_ptr (n + 1 entries) starts
// at 0 and is monotone; col_idx is non-NULL when there are entries; every column lies in
// [0, n_cols) and the columns of a row ascend strictly.
void check_csr(int64_t n, int64_t n_cols, const int64_t* row_ptr, const int32_t* col_idx) {
  if (row_ptr[0] != 0) fail(TPL_ERR_INVALID_ARGUMENT, "row_ptr must start at 0 and end at nnz");
  for (int64_t i = 0; i < n; ++i)
    if (row_ptr[i + 1] < row_ptr[i]) fail(TPL_ERR_INVALID_ARGUMENT, "row_ptr not monotone");
  if (row_ptr[n] > 0 && !col_idx) fail(TPL_ERR_INVALID_ARGUMENT, "col_idx/vals is NULL");
  for (int64_t i = 0; i < n; ++i)
    for (int64_t q = row_ptr[i]; q < row_ptr[i + 1]; ++q) {
      const int32_t c = col_idx[q];
      if (c < 0 || c >= n_cols) fail(TPL_ERR_INVALID_ARGUMENT, "column index out of range");
      if (q > row_ptr[i] && c <= col_idx[q - 1])
        fail(TPL_ERR_INVALID_ARGUMENT, "column indices must be strictly ascending per row");
    }
}

} // namespace tpl

// Host-only C ABI entry (include/tpl.h): the locality order's permutation of a CSR.
extern "C" tpl_status tpl_locality_order(int64_t n, const int64_t* row_ptr,
                                         const int32_t* col_idx, int32_t short_row_max,
                                         int32_t groups, int32_t* perm, int32_t* applied) {
  using namespace tpl;
  try {
    if (n < 0 || (n > 0 && (!row_ptr || !perm)) || !applied)
      fail(TPL_ERR_INVALID_ARGUMENT, "bad argument");
    if (n >= INT32_MAX || (n > 0 && row_ptr[n] >= INT32_MAX))
      fail(TPL_ERR_UNSUPPORTED, "n and nnz must be < 2^31");
    // the operator constructors' CSR rules: row_ptr from 0, monotone; columns in range,
    // strictly ascending per row (short_row_threshold and the sort key index by them)
    if (n > 0) check_csr(n, n, row_ptr, col_idx);
    std::vector<int32_t> rp(n + 1, 0);
    for (int64_t i = 0; n > 0 && i <= n; ++i) rp[i] = (int32_t)row_ptr[i];
    std::vector<int32_t> col;
    if (n > 0 && row_ptr[n] > 0) col.assign(col_idx, col_idx + row_ptr[n]);
    SchedParams sp;
    sp.short_row_max = short_row_max > 0 ? short_row_max : -1;
    if (groups > 0) sp.order_groups = groups;
    const std::vector<int32_t> p = locality_order(n, rp, col, sp);
    *applied = p.empty() ? 0 : 1;
    for (int64_t i = 0; i < n; ++i) perm[i] = p.empty() ? (int32_t)i : p[i];
    set_last_error("");
    return TPL_OK;
  } catch (const Error& e) {
    set_last_error(e.code, e.msg, e.det);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_last_error(TPL_ERR_OUT_OF_MEMORY, "host allocation failed", {});
    return TPL_ERR_OUT_OF_MEMORY;
  }
}
