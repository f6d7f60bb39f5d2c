"""Lab: which bins make the SpMV's tail? Rebuilds the long-row bins of the benched
500k operator on the CPU (tpl_layout.cpp build_layout's first-fit packing, restated) and
sets each bin's features beside its end time from a stamp run
(gpurun_out/diag/pass1_stamps.npz, scripts/stamps.py). Dev tool, CPU only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import tpl_amd  # noqa: E402
from conftest import load_kkt  # noqa: E402

a = load_kkt(500000, "/tmp").a.tocsr()
plan = tpl_amd.HostPlan(a, order_groups=13)
sch = plan.schedule()
perm = sch["perm"]
n = a.shape[0]
iperm = np.empty(n, dtype=np.int64)
iperm[perm] = np.arange(n)
pa = a[perm][:, perm].tocsr()
pa.sort_indices()
S = sch["slices"]
lr = sch["long_rows"]
BIN_CAP, SEGS, BIG = 2048, int(os.environ.get("TPL_BIN_SEGS", "0")) or 255, 64
bins = [[] for _ in range(S)]  # per slice: list of (pieces, fill, cols)
for s in range(S):
    lo, hi = n * s // S, n * (s + 1) // S
    cur = None
    for r in lr:
        c = pa.indices[pa.indptr[r]:pa.indptr[r + 1]]
        c = c[(c >= lo) & (c < hi)]
        if cur is None or cur["fill"] + len(c) > BIN_CAP or len(cur["pieces"]) == SEGS:
            cur = {"pieces": [], "fill": 0, "cols": []}
            bins[s].append(cur)
        cur["pieces"].append(len(c))
        cur["fill"] += len(c)
        cur["cols"].append(c)
M = max(len(b) for b in bins)
print(f"n {n}, long rows {len(lr)}, slices {S}, bins per slice {[len(b) for b in bins]}")
# bins' gather columns for scripts/lab/bin_gather_lab.hip: per bin (block order b = 8m + s,
# bin_cap entries; -1 padding) in the canonical position order and sorted by column inside
# the bin (the same set of gathers, fewer distinct lines per wave-instruction)
if os.environ.get("DUMP"):
    nb = 8 * M
    canon = np.full((nb, BIN_CAP), -1, dtype=np.int32)
    for b in range(nb):
        m, s = b >> 3, b & 7
        if m < len(bins[s]) and bins[s][m]["cols"]:
            c = np.concatenate(bins[s][m]["cols"]).astype(np.int32)
            canon[b, :len(c)] = c
    srt = np.sort(np.where(canon < 0, np.iinfo(np.int32).max, canon), axis=1)
    srt[srt == np.iinfo(np.int32).max] = -1
    hdr = np.array([nb, BIN_CAP, n], dtype=np.int32)
    with open(os.environ["DUMP"], "wb") as f:
        f.write(hdr.tobytes()); f.write(canon.tobytes()); f.write(srt.tobytes())
    w = canon.reshape(nb, 8, 4, 64)  # (bin, u, wave, lane): position u*256 + 64*wave + lane
    def lines_per_instr(a):
        a = a.reshape(nb, 8, 4, 64)
        tot = 0
        for x in a.reshape(-1, 64):
            x = x[x >= 0]
            tot += len(np.unique(x >> 4))
        return tot / (nb * 32)
    print("distinct 128-B lines per wave-instruction: canonical %.1f, sorted %.1f"
          % (lines_per_instr(canon), lines_per_instr(srt)))
    sys.exit(0)

npz = np.load(os.environ.get("NPZ", os.path.join(ROOT, "gpurun_out", "diag", "pass1_stamps.npz")))
raw = npz["raw"].astype(np.float64)  # (3, G, K)
t0 = raw[:, :, 0].min(axis=1, keepdims=True)
end = ((raw[:, :, 5] - t0) / 100.0).mean(axis=0)
dur = ((raw[:, :, 5] - raw[:, :, 0]) / 100.0).mean(axis=0)
start = ((raw[:, :, 0] - t0) / 100.0).mean(axis=0)
rows = []
for b in range(int(npz["nbins"])):
    m, s = b >> 3, b & 7
    if m >= len(bins[s]):
        continue
    B = bins[s][m]
    cols = np.concatenate(B["cols"]) if B["cols"] else np.zeros(0, dtype=np.int64)
    lines = len(np.unique(cols >> 4))
    nbig = sum(p > BIG for p in B["pieces"])
    rows.append((b, m, s, B["fill"], len(B["pieces"]), nbig, max(B["pieces"]), lines,
                 start[b], dur[b], end[b]))
R = np.array(rows)
names = ["fill", "pieces", "nbig", "maxpiece", "lines", "m"]
idx = {"fill": 3, "pieces": 4, "nbig": 5, "maxpiece": 6, "lines": 7, "m": 1}
print("corr with duration / end:")
for nm in names:
    x = R[:, idx[nm]]
    print(f"  {nm:9s} {np.corrcoef(x, R[:, 9])[0, 1]:+.2f} {np.corrcoef(x, R[:, 10])[0, 1]:+.2f}"
          f"   range {x.min():.0f}..{x.max():.0f}")
o = np.argsort(-R[:, 10])
print(" bin   m  s  fill pcs big maxp lines | start  dur   end")
for i in list(o[:20]) + list(o[-5:]):
    r = R[i]
    print(f" {int(r[0]):4d} {int(r[1]):3d} {int(r[2]):2d} {int(r[3]):5d} {int(r[4]):3d} {int(r[5]):3d}"
          f" {int(r[6]):4d} {int(r[7]):5d} | {r[8]:5.2f} {r[9]:5.2f} {r[10]:5.2f}")
plan.close()

# linear cost model of a bin's duration: a + b pieces + c lines + d nbig + e fill
X = np.column_stack([np.ones(len(R)), R[:, 4], R[:, 7], R[:, 5], R[:, 3]])
coef, *_ = np.linalg.lstsq(X, R[:, 9], rcond=None)
pred = X @ coef
print("model dur = %.3f + %.4f pieces + %.5f lines + %.4f nbig + %.6f fill;  r = %.2f, resid sd %.2f"
      % (*coef, np.corrcoef(pred, R[:, 9])[0, 1], np.std(R[:, 9] - pred)))
np.save("/tmp/bin_model.npy", coef)

mk = ((raw - t0[:, :, None]) / 100.0).mean(axis=0)  # (G, K) mean over the 3 launches
print("marks (us from launch start): start scale products pieces publish end")
med = np.median(mk[:int(npz["nbins"]), :6], axis=0)
print("  median bin      " + " ".join(f"{v:5.2f}" for v in med))
for b in [13, 2, 23, 525, 522, 517, 527, 512, 252, 236]:
    print(f"  bin {b:4d}        " + " ".join(f"{v:5.2f}" for v in mk[b, :6]))
