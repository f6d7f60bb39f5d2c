"""Per-kernel median / min / mean dispatch durations (µs) from a rocprofv3 --kernel-trace
CSV ("median per-kernel time from rocprofv3 kernel trace").
Usage: python scripts/kernel_medians.py run_kernel_trace.csv [out.json]"""
import csv
import json
import statistics
import sys

dur = {}
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tpl::", "")
    dur.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
out = {k: {"calls": len(v), "median_us": round(statistics.median(v), 3),
           "min_us": round(min(v), 3), "mean_us": round(statistics.fmean(v), 3)}
       for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))}
for k, v in out.items():
    print(f"{k:40s} {v['calls']:7d} median {v['median_us']:9.3f}  min {v['min_us']:9.3f}  mean {v['mean_us']:9.3f}")
if len(sys.argv) > 2:
    with open(sys.argv[2], "w") as f:
        json.dump(out, f, indent=1)
