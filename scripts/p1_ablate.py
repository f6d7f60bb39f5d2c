"""Dev tool: isolated k_p1_spmv / k_p2_spmv / k_p1_axpy times of experiment variants
(two-pass-lanczos_amd/variants/libtpl_<name>.so, scripts/build_variants.sh) on the 500k KKT."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.join(ROOT, "two-pass-lanczos_amd"))
    import numpy as np
    import tpl_amd
    from tpl_amd.utils.data_loader import load_kkt_system, write_qfc_3line
    write_qfc_3line("/tmp/t.qfc", 500000)
    a = load_kkt_system(os.path.join(ROOT, "tests/golden/kkt/netgen-500000-3.dmx.xz"), "/tmp/t.qfc").a
    n = a.shape[0]
    op = tpl_amd.HipCsrOp(a)
    tpl_amd.lanczos_two_pass(op, a @ np.full(n, 1 / np.sqrt(n)), 50, "inv")
    row = {"variant": sys.argv[2]}
    for kid, nm in [(0, "p1_spmv"), (1, "p1_axpy"), (2, "p2_spmv")]:
        row[nm] = round(op.profile_kernel(kid, 300)[0], 2)
    print(json.dumps(row), flush=True)
    sys.exit(0)
for name in os.environ.get("VARIANTS", "base").split(","):
    env = dict(os.environ)
    if name != "main":  # main: the in-tree libtpl_amd.so
        env["TPL_LIB_PATH"] = os.path.join(ROOT, "two-pass-lanczos_amd/variants", f"libtpl_{name}.so")
    subprocess.run([sys.executable, __file__, "--child", name], env=env, check=True, timeout=120)
