"""The engine's tradeoff / scalability CSVs (tpl_amd.harness on the MI355X) beside the
reference's published ones (its Xeon, one thread): time per row and the ratio.
    python scripts/compare_timing.py OURS_TRADEOFF.csv OURS_SCALABILITY.csv"""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "tests", "golden", "reference_results")


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    ours_t, ours_s = sys.argv[1], sys.argv[2]
    ref = {(r["variant"], int(r["k"])): r for r in rows(os.path.join(REF, "tradeoff_arcs500k_rho3.csv"))}
    print("tradeoff, 500k arcs: variant k | reference s | MI355X ms | ratio | device MB (ours) | VmPeak MB (reference)")
    for r in rows(ours_t):
        key = (r["variant"], int(r["k"]))
        if key in ref:
            t0, t1 = float(ref[key]["time_s"]), float(r["time_s"])
            print(f"  {key[0]:9s} {key[1]:5d} | {t0:9.3f} | {1000 * t1:8.3f} | {t0 / t1:7.0f}x | "
                  f"{int(r['device_kb']) / 1024:8.1f} | {int(ref[key]['rss_kb']) / 1024:8.1f}")
    refs = rows(os.path.join(REF, "scalability_k500_rho3.csv"))
    ours = rows(ours_s)
    print("scalability, k = 500: variant | reference n, s | MI355X n, ms | ratio")
    for v in ("standard", "two-pass"):
        a = [r for r in refs if r["variant"] == v]
        b = [r for r in ours if r["variant"] == v]
        for x, y in zip(a, b):
            t0, t1 = float(x["time_s"]), float(y["time_s"])
            print(f"  {v:9s} | {int(x['n']):7d} {t0:7.3f} | {int(y['n']):7d} {1000 * t1:8.3f} | {t0 / t1:6.0f}x")


if __name__ == "__main__":
    main()
