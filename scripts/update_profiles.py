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
with open(os.path.join(out, "bench.log")) as f:
    line = [l for l in f if l.startswith("{")][-1]
with open(os.path.join(prof, f"{tag}_bench.json"), "w") as f:
    f.write(line)
# the headline instance of k_p2_spmv: template variant 122 (500k KKT layout: uniform
# width 2, int8 values, uint16 chunk and bin columns, chunk window); the other configs of
# the same bench run (5k, 50k, 5M) instantiate other variants or share it with fewer calls
HEADLINE = sys.argv[2] if len(sys.argv) > 2 else "k_p2_spmv<122>"
blocks, cur = {}, None
for l in open(os.path.join(out, "pmc_summary.txt")):
    if not l.startswith(" "):
        cur = l.strip()
        continue
    m = re.match(r"\s+(\S+)\s+([0-9.]+)", l)
    if m and cur and cur.startswith("k_p2_spmv"):
        blocks.setdefault(cur, {})[m.group(1)] = float(m.group(2))
vals = blocks[HEADLINE]
d = {"kernel": "k_p2_spmv", "config": "500k-arc KKT, lanczos_two_pass k=500 (bench.py --steps 1 --warmup 0)",
     "FETCH_SIZE_KiB": vals["FETCH_SIZE"], "WRITE_SIZE_KiB": vals["WRITE_SIZE"],
     "traffic_bytes_per_launch": round(2 * vals["FETCH_SIZE"] * 1024 + vals["WRITE_SIZE"] * 1024),
     "correction": "2 x FETCH_SIZE (gfx950 half-count of wide reads) + WRITE_SIZE",
     "source": f"profiles/{tag}_pmc_summary.txt (rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE)"}
with open(os.path.join(prof, "pmc_k_p2_spmv.json"), "w") as f:
    json.dump(d, f, indent=1)
print(d)
