"""Timeline of one SpMV-shaped launch from a TPL_STAMP build (dev tool). Marks per
workgroup: [0] start, [1] scale known, [2] products staged / row sums, [3] piece sums
staged, [4] publish drained, [5] end."""
import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
import numpy as np
import tpl_amd
from tpl_amd import _lib
from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
K = 9  # kMarks (tpl_lab.h): marks 0..5, the HW_ID / XCC_ID slot, marks 7..8 (bins' piece sums)
write_qfc_3line("/tmp/t.qfc", 500000)
a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"), "/tmp/t.qfc").a
n = a.shape[0]
b = a @ np.full(n, 1 / np.sqrt(n))
op = tpl_amd.HipCsrOp(a)
op.set_order_groups(int(os.environ.get("GROUPS", "13")))  # the benched (pinned) order
op.set_slices(int(os.environ.get("SLICES", "0")))
tpl_amd.lanczos_two_pass(op, b, 50, "inv")
sch = op.schedule()
ns = len(sch["short_rows"])
CR = int(os.environ.get("CR", "512"))
nch = (ns + CR - 1) // CR
# the chunk part of an SpMV grid is padded to 8 ceil(G2 / 8) E / 512 blocks (chunk_of_block)
NCHB = 8 * ((sch["G2"] + 7) // 8) * (sch["E"] // 512)
fn = _lib.lib.tpl_debug_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
def q(x):
    x = x[np.isfinite(x)]
    return " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 50, 90, 100])) if len(x) else "-"
for kid, name in [(3, "spmv"), (2, "p2_spmv"), (0, "p1_spmv")]:
    op.profile_kernel(kid, 20)
    st = np.zeros(K * 65536, dtype=np.uint64)
    fn(st.ctypes.data, 65536)
    G = int(np.count_nonzero(st[0:K * 60000:K]))  # below kAxpyMarkBase
    nsl = G - NCHB
    m = st[:K * G].reshape(G, K).astype(np.float64)
    m[m == 0] = np.nan
    base = np.nanmin(m[:, 0])
    t = (m - base) / 100.0  # us
    first = os.environ.get("FIRST", "slices")
    ch, sl = (slice(0, nch), slice(nch, G)) if first == "chunks" else (slice(nsl, G), slice(0, nsl))
    print(f"== {name}: grid {G} (chunks {nch}, bins {nsl}); us; pct 0/50/90/100")
    for nm, sel, marks in [("chunk", ch, [1, 2]), ("bin", sl, [1, 2, 3, 4])]:
        tt = t[sel]
        print(f"  {nm:5s} start      {q(tt[:,0])}")
        for k in marks:
            print(f"  {nm:5s} mark{k}-start {q(tt[:,k]-tt[:,0])}")
        print(f"  {nm:5s} end        {q(tt[:,5])} | dur {q(tt[:,5]-tt[:,0])}")
    # stale marks from earlier launches are possible for marks a block did not reach

# pass one as it alternates (TPL_KERNEL_PASS1_STEP: k_p1_spmv then k_p1_axpy, step 2 over
# and over): the last pair's timelines on one clock — the boundary between the two
# kernels is the gap from k_p1_spmv's last workgroup end to k_p1_axpy's first start
if os.environ.get("PASS1", "1") == "1":
    op.profile_kernel(6, 20)
    st = np.zeros(K * 65536, dtype=np.uint64)
    fn(st.ctypes.data, 65536)
    AX = 60000  # kAxpyMarkBase (tpl_lab.h)
    m = st.reshape(65536, K).astype(np.float64)
    m[m == 0] = np.nan
    sp_rows = m[:AX]
    sp_rows = sp_rows[np.isfinite(sp_rows[:, 0])]
    ax = m[AX:]
    ax = ax[np.isfinite(ax[:, 0])]
    base = np.nanmin(sp_rows[:, 0])
    ts, ta = (sp_rows - base) / 100.0, (ax - base) / 100.0
    print(f"== pass-one step (k_p1_spmv {len(ts)} workgroups, then k_p1_axpy {len(ta)}); us from the SpMV's first start")
    nchb = 8 * ((sch["G2"] + 7) // 8) * (sch["E"] // 512)  # chunk part of the grid
    ff = getattr(_lib.lib, "tpl_debug_first", None)
    if ff is not None:
        ff.argtypes = [ctypes.c_void_p, ctypes.c_int]
        fst = np.zeros(65536, dtype=np.uint64)
        ff(fst.ctypes.data, 65536)
        f0 = (fst[:len(sp_rows)].astype(np.float64) - base) / 100.0
        print(f"  first-instruction stamp (dispatch), bins {q(f0[:len(ts) - nchb])}  chunks {q(f0[len(ts) - nchb:])}")
        print(f"  mark0 - first: bins {q(ts[:len(ts) - nchb, 0] - f0[:len(ts) - nchb])}  chunks {q(ts[len(ts) - nchb:, 0] - f0[len(ts) - nchb:])}")
    nbin = len(ts) - nchb
    for nm, sel, marks in [("bin", slice(0, nbin), [1, 2, 7, 8, 3, 4]), ("chunk", slice(nbin, len(ts)), [1, 2])]:
        tt = ts[sel]
        print(f"  {nm:5s} start      {q(tt[:,0])}")
        for k in marks:
            print(f"  {nm:5s} mark{k}-start {q(tt[:,k]-tt[:,0])}")
        print(f"  {nm:5s} end        {q(tt[:,5])} | dur {q(tt[:,5]-tt[:,0])}")
    print(f"  axpy  start      {q(ta[:,0])}   (gap after the SpMV's last end: {np.nanmin(ta[:,0]) - np.nanmax(ts[:,5]):.2f})")
    for k, nm in [(1, "loads issued"), (4, "alpha partials landed"), (2, "alpha known"),
                  (3, "r stored")]:
        print(f"  axpy  mark{k}-start {q(ta[:,k]-ta[:,0])}  ({nm})")
    print(f"  axpy  end        {q(ta[:,5])} | dur {q(ta[:,5]-ta[:,0])}")

    # is the tail structural? the same pair again: per-workgroup end times of two launches
    if os.environ.get("TAIL", "1") == "1":
        ends = []
        for rep in range(3):
            op.profile_kernel(6, 20)
            st = np.zeros(K * 65536, dtype=np.uint64)
            fn(st.ctypes.data, 65536)
            mm = st.reshape(65536, K)[:AX].astype(np.float64)
            G = int(np.count_nonzero(mm[:, 0]))
            e = (mm[:G, 5] - mm[:G, 0].min()) / 100.0
            ends.append(e)
            hw = st.reshape(65536, K)[:G, 6]
            raw = mm[:G] if rep == 0 else np.concatenate([raw, mm[:G]])
        nb = G - NCHB  # bins first in the grid (FIRST=slices)
        os.makedirs(os.path.join(ROOT, "gpurun_out", "diag"), exist_ok=True)
        np.savez(os.path.join(ROOT, "gpurun_out", "diag", "pass1_stamps.npz"), raw=raw.reshape(3, G, K),
                 hw=hw, nbins=nb, nchunks=nch)
        print(f"== SpMV tail: {G} workgroups ({nb} bins then {nch} chunks), 3 launches")
        for r in range(1, 3):
            print(f"  corr(end, launch 0 vs {r}): bins {np.corrcoef(ends[0][:nb], ends[r][:nb])[0,1]:.2f}"
                  f" chunks {np.corrcoef(ends[0][nb:], ends[r][nb:])[0,1]:.2f}")
        avg = np.mean(ends, axis=0)
        order = np.argsort(-avg)[:24]
        print("  slowest (mean end over 3): idx kind xcc se cu | end0 end1 end2")
        for g in order:
            kind = "bin" if g < nb else "chunk"
            v = int(hw[g])
            print(f"   {g:5d} {kind:5s} {(v >> 32) & 15:3d} {(v >> 13) & 7:2d} {(v >> 8) & 15:2d} | "
                  + " ".join(f"{e[g]:5.2f}" for e in ends))
        for kind, sel in (("bin", slice(0, nb)), ("chunk", slice(nb, G))):
            a = avg[sel]
            print(f"  {kind}: mean end by grid index mod 8: " + " ".join(f"{a[i::8].mean():.2f}" for i in range(8)))
