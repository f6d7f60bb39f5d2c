"""Copy the judged profiles of a scripts/gpu_check.sh run from gpurun_out/ into
profiles/ (tracked): rocprofv3 kernel stats, PMC summary, the bench line, and the
per-launch HBM traffic of the roofline kernel (2 x FETCH_SIZE + WRITE_SIZE, KiB ->
bytes; gfx950 half-counts wide reads, MI355X_MICROARCH.md). Arg: tag (e.g. r01_v6)."""
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
out = os.path.join(ROOT, "gpurun_out")
prof = os.path.join(ROOT, "profiles")
shutil.copy(os.path.join(out, "prof", "run_kernel_stats.csv"),
            os.path.join(prof, f"{tag}_kernel_stats.csv"))
shutil.copy(os.path.join(out, "pmc_summary.txt"), os.path.join(prof, f"{tag}_pmc_summary.txt"))
# the median per-kernel time from the rocprofv3 kernel trace
trace = os.path.join(out, "prof", "run_kernel_trace.csv")
if os.path.exists(trace):
    import subprocess
    subprocess.check_call([sys.executable, os.path.join(ROOT, "scripts", "kernel_medians.py"), trace,
                           os.path.join(prof, f"{tag}_kernel_medians.json")])
with open(os.path.join(out, "bench.log")) as f:
    line = [l for l in f if l.startswith("{")][-1]
with open(os.path.join(prof, f"{tag}_bench.json"), "w") as f:
    f.write(line)
# the headline instance of k_p2_spmv: template variant 122 (500k KKT layout: uniform
# width 2, int8 values, uint16 chunk and bin columns, chunk window); the other configs of
# the same bench run (5k, 50k, 5M) instantiate other variants or share it with fewer calls
HEADLINE = sys.argv[2] if len(sys.argv) > 2 else "k_p2_spmv<58>"
blocks, cur = {}, None
for l in open(os.path.join(out, "pmc_summary.txt")):
    if not l.startswith(" "):
        cur = l.strip()
        continue
    m = re.match(r"\s+(\S+)\s+([0-9.]+)", l)
    if m and cur:
        blocks.setdefault(cur, {})[m.group(1)] = float(m.group(2))
SRC = (f"profiles/{tag}_pmc_summary.txt (rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, "
       "bench.py --headline-only 1 --steps 1 --warmup 0: every launch is the 500k headline's)")
CFG = "500k-arc KKT, lanczos_two_pass k=500, pinned locality order (bench.py --headline-only 1)"


def traffic(vals):
    return round(2 * vals["FETCH_SIZE"] * 1024 + vals["WRITE_SIZE"] * 1024)


vals = blocks[HEADLINE]
d = {"kernel": "k_p2_spmv", "config": CFG,
     "FETCH_SIZE_KiB": vals["FETCH_SIZE"], "WRITE_SIZE_KiB": vals["WRITE_SIZE"],
     "traffic_bytes_per_launch": traffic(vals),
     "correction": "2 x FETCH_SIZE (gfx950 half-count of wide reads) + WRITE_SIZE",
     "source": SRC}
with open(os.path.join(prof, "pmc_k_p2_spmv.json"), "w") as f:
    json.dump(d, f, indent=1)
print(d)
# pass one at the same size (its counters isolated from the other configs)
p1 = {"config": CFG, "correction": d["correction"], "source": SRC, "kernels": {}}
for name, vals in blocks.items():
    if name.startswith(("k_p1_spmv", "k_p1_axpy")):
        p1["kernels"][name] = {"FETCH_SIZE_KiB": vals["FETCH_SIZE"],
                               "WRITE_SIZE_KiB": vals["WRITE_SIZE"],
                               "traffic_bytes_per_launch": traffic(vals)}
with open(os.path.join(prof, "pmc_pass_one.json"), "w") as f:
    json.dump(p1, f, indent=1)
print(p1)
# in-graph average duration of both SpMV kernels of the headline (rocprofv3 --stats of
# the --headline-only run): bench.py reads it for roofline.committed_profile
stats = {}
import csv
with open(os.path.join(out, "prof", "run_kernel_stats.csv")) as f:
    for r in csv.DictReader(f):
        m = re.search(r"tpl::(k_p[12]_spmv|k_p1_axpy)(<\d+>)", r["Name"])
        if m and m.group(1) + m.group(2) in ("k_p1_spmv<58>", "k_p2_spmv<58>", "k_p1_axpy<12>"):
            stats[m.group(1)] = {"avg_ns": float(r["AverageNs"]), "calls": int(r["Calls"]),
                                 "percentage": float(r["Percentage"])}
med = {}
mpath = os.path.join(prof, f"{tag}_kernel_medians.json")
if os.path.exists(mpath):
    for name, v in json.load(open(mpath)).items():
        for k in ("k_p1_spmv<58>", "k_p2_spmv<58>", "k_p1_axpy<12>"):
            if name == k:
                med[k.split("<")[0]] = round(1000.0 * v["median_us"], 1)
sys.path.insert(0, ROOT)
from bench import kernel_src_digest  # noqa: E402  (the profile's kernels: this tree's)
bline = json.loads(line)
b_spmv = (bline.get("roofline_live") or bline["roofline"])["bytes_per_launch"]
rj = {"config": CFG, "kernel_src_sha16": kernel_src_digest(),
      "bytes_per_launch": b_spmv,  # SURVEY §8(d) B_spmv of the headline (the bench line's)
      "avg_ns": {k: v["avg_ns"] for k, v in stats.items()}, "median_ns": med,
      "calls": {k: v["calls"] for k, v in stats.items()},
      "percentage_of_gpu_time": {k: v["percentage"] for k, v in stats.items()},
      "source": f"profiles/{tag}_kernel_stats.csv (rocprofv3 --kernel-trace --stats, bench.py "
                "--headline-only 1 --steps 5 --warmup 1)"}
with open(os.path.join(prof, "rocprof_headline.json"), "w") as f:
    json.dump(rj, f, indent=1)
print(rj)
