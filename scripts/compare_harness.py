"""Compare the engine's harness CSVs (profiles/r02_harness) with the reference's published
results (tests/golden/reference_results): per file, the k range where the relative error
agrees to 1e-6 relative, the worst ratio of orthogonality losses, and the drift columns."""
import csv, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ours_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r02_harness")
ref_dir = os.path.join(ROOT, "tests", "golden", "reference_results")
def rows(p):
    with open(p) as f:
        return {int(r["k"]): r for r in csv.DictReader(f)}
for name in sorted(os.listdir(ref_dir)):
    if not os.path.exists(os.path.join(ours_dir, name)):
        continue
    ref, ours = rows(os.path.join(ref_dir, name)), rows(os.path.join(ours_dir, name))
    ks = sorted(set(ref) & set(ours))
    if name.startswith("accuracy"):
        agree = [k for k in ks if abs(float(ours[k]["relative_error_standard"]) - float(ref[k]["relative_error_standard"]))
                 <= 1e-6 * float(ref[k]["relative_error_standard"]) + 1e-15]
        last = max((k for k in ks if all(kk in agree for kk in ks if kk <= k)), default=None)
        dev = max(float(ours[k]["relative_solution_deviation"]) for k in ks)
        print(f"{name}: {len(ks)} rows, relative_error_standard within 1e-6 rel for k <= {last} "
              f"({len(agree)}/{len(ks)} rows), max relative_solution_deviation {dev:.1e}")
    else:
        drift = max(float(ours[k]["basis_drift_fro"]) for k in ks) if ks else None
        dev = max(float(ours[k]["solution_deviation_l2"]) for k in ks) if ks else None
        ratio = [float(ours[k]["ortho_loss_standard"]) / float(ref[k]["ortho_loss_standard"])
                 for k in ks if float(ref[k]["ortho_loss_standard"]) > 0]
        print(f"{name}: {len(ks)} rows, basis_drift_fro max {drift}, solution_deviation_l2 max {dev}, "
              f"ortho_loss ratio ours/published {min(ratio):.2f}..{max(ratio):.2f}")
