"""Per-bin cost model of the long-row bins (dev tool, CPU only).

Rebuilds the headline operator's bins on the host (500k netgen KKT, locality order with
the pinned 13 groups; first fit of each slice's pieces in row order, as
tpl_layout.cpp build_layout) and joins them with a stamp timeline of pass one's SpMV
(gpurun_out/diag/pass1_stamps.npz, scripts/stamps.py on a TPL_STAMP build: workgroup
S m + s is bin m of slice s). Prints the features that explain each bin's end time and a
least-squares fit of end time on them.

    python scripts/lab/bin_cost.py [NPZ]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))

CAP, SEGS, BIG = 2048, 255, 64


def headline_matrix(groups=13):
    import scipy.sparse as sp

    import tpl_amd
    from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
    write_qfc_3line("/tmp/bin_cost.qfc", 500000)
    a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"),
                        "/tmp/bin_cost.qfc").a.tocsr()
    plan = tpl_amd.HostPlan(a, "single", order_groups=groups)
    sch = plan.schedule()
    plan.close()
    perm = sch["perm"]
    ip = np.empty_like(perm)
    ip[perm] = np.arange(len(perm), dtype=perm.dtype)
    pa = a[perm][:, perm].tocsr()
    pa.sort_indices()
    return pa, sch


def pieces(pa, sch):
    """[(slice, row rank, start, end)] of every non-empty piece, rows ascending."""
    n = pa.shape[0]
    S = sch["slices"]
    lr = sch["long_rows"]
    bounds = [n * s // S for s in range(S + 1)]
    out = [[] for _ in range(S)]
    cnt = np.zeros(len(lr), dtype=np.int64)
    for r, row in enumerate(lr):
        q0, q1 = pa.indptr[row], pa.indptr[row + 1]
        cols = pa.indices[q0:q1]
        cuts = np.searchsorted(cols, bounds) + q0
        for s in range(S):
            if cuts[s + 1] > cuts[s]:
                out[s].append((r, int(cuts[s]), int(cuts[s + 1])))
                cnt[r] += 1
    return out, np.maximum(cnt, 1)


def first_fit(pcs):
    bins = []
    fill = 0
    for p in pcs:
        ln = p[2] - p[1]
        if not bins or fill + ln > CAP or len(bins[-1]) == SEGS:
            bins.append([])
            fill = 0
        bins[-1].append(p)
        fill += ln
    return bins


def features(pa, bins, cnt):
    f = []
    for b in bins:
        ent = sum(p[2] - p[1] for p in b)
        cols = np.concatenate([pa.indices[p[1]:p[2]] for p in b]) if b else np.zeros(0, int)
        lines = len(np.unique(cols >> 4))
        big = sum(1 for p in b if p[2] - p[1] > BIG)
        small = len(b) - big
        single = sum(1 for p in b if cnt[p[0]] == 1)
        # 8-lane sums: 32 small pieces per pass; 16-lane: 16 big pieces per pass, each
        # over ceil(len / 16) entries per lane
        passes_small = -(-small // 32)
        longest = max((p[2] - p[1] for p in b), default=0)
        f.append((ent, lines, len(b), big, small, single, passes_small, longest))
    return np.array(f, dtype=np.float64)


NAMES = ["entries", "lines", "pieces", "big", "small", "single", "passes_small", "longest"]


def layout_cost(pa, b):
    """tpl_layout.cpp's predicted bin cost (line units): 228 per piece-sum round of the
    wave tasks + the distinct lines."""
    if not b:
        return 0
    big = sum(1 for p in b if p[2] - p[1] > BIG)
    small = len(b) - big
    rounds = (-(-big // 4) + -(-small // 8) + 3) // 4
    cols = np.concatenate([pa.indices[p[1]:p[2]] for p in b])
    return 228 * rounds + len(np.unique(cols >> 4))


def place_light_on_crowded(pa, bins, M, S):
    """tpl_layout.cpp bin_balance 2: the first fit's bins, the lightest of each slice on the
    crowded CU positions (m mod 32 < M mod 32, S = 8, M > 32)."""
    if not (S == 8 and M > 32 and M % 32):
        return bins
    crowded = [m % 32 < M % 32 for m in range(M)]
    out = []
    for bs in bins:
        bs = bs + [[] for _ in range(M - len(bs))]
        cost = [layout_cost(pa, b) for b in bs]
        order = sorted(range(M), key=lambda m: cost[m])  # stable
        nc = sum(crowded)
        light, rest = sorted(order[:nc]), sorted(order[nc:])
        il = ir = 0
        nb = []
        for m in range(M):
            if crowded[m]:
                nb.append(bs[light[il]]); il += 1
            else:
                nb.append(bs[rest[ir]]); ir += 1
        out.append(nb)
    return out


def main():
    npz = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out/diag/pass1_stamps.npz")
    pa, sch = headline_matrix()
    S = sch["slices"]
    per_slice, cnt = pieces(pa, sch)
    bins = [first_fit(p) for p in per_slice]
    M = max(len(b) for b in bins)
    if os.environ.get("MODE", "2") == "2":
        bins = place_light_on_crowded(pa, bins, M, S)
    print(f"slices {S}, bins per slice {[len(b) for b in bins]}, M = {M}")
    feat = np.zeros((S * M, len(NAMES)))
    for s in range(S):
        fs = features(pa, bins[s], cnt)
        for m in range(len(bins[s])):
            feat[S * m + s] = fs[m]
    d = np.load(npz)
    raw = d["raw"]  # (launch, workgroup, mark), 100 MHz ticks
    nb = S * M
    ends, durs = [], []
    for L in range(raw.shape[0]):
        r = raw[L, :, :].copy()
        r[r == 0] = np.nan
        t0 = np.nanmin(r[:, 0])
        ends.append((r[:nb, 5] - t0) / 100.0)
        durs.append((r[:nb, 5] - r[:nb, 0]) / 100.0)
    end = np.nanmean(ends, axis=0)
    dur = np.nanmean(durs, axis=0)
    ok = feat[:, 0] > 0
    print(f"bins with entries {ok.sum()} of {nb}; end us: median {np.median(end[ok]):.2f} "
          f"max {end[ok].max():.2f}")
    for i, nm in enumerate(NAMES):
        c = np.corrcoef(feat[ok, i], dur[ok])[0, 1]
        print(f"  corr(dur, {nm:12s}) = {c:+.3f}   range {feat[ok, i].min():.0f}..{feat[ok, i].max():.0f}")
    X = np.column_stack([np.ones(ok.sum())] + [feat[ok, i] for i in range(len(NAMES))])
    coef, *_ = np.linalg.lstsq(X, dur[ok], rcond=None)
    pred = X @ coef
    print("fit dur = " + " + ".join(f"{c:.4g}*{n}" for c, n in zip(coef, ["1"] + NAMES)))
    print(f"  r = {np.corrcoef(pred, dur[ok])[0, 1]:.3f}, rms {np.sqrt(np.mean((pred - dur[ok]) ** 2)):.3f} us")
    order = np.argsort(-end)
    print("slowest bins: idx m s | end dur | " + " ".join(NAMES))
    for g in order[:20]:
        print(f"  {g:4d} {g // S:3d} {g % S} | {end[g]:.2f} {dur[g]:.2f} | "
              + " ".join(f"{v:.0f}" for v in feat[g]))
    np.savez("/tmp/bin_cost.npz", feat=feat, end=end, dur=dur, S=S, M=M)


if __name__ == "__main__":
    main()
