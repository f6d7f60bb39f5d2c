"""Boundaries between consecutive kernels in a rocprofv3 --kernel-trace CSV: for each
(previous kernel -> next kernel) pair on one queue, the median of start(next) - end(prev).
A negative gap means rocprofv3's intervals of the two kernels overlap, i.e. the next
kernel's recorded duration also covers part of the previous one's tail (so per-kernel
durations of a graph can sum to more than the wall time of the sequence).
Usage: python scripts/trace_gaps.py run_kernel_trace.csv [min_calls]"""
import csv
import statistics
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tpl::", "")
    q = (r.get("Agent_Id", ""), r.get("Queue_Id", ""))
    rows.append((q, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
pairs = {}
for a, b in zip(rows, rows[1:]):
    if a[0] != b[0]:
        continue
    pairs.setdefault((a[3], b[3]), []).append((b[1] - a[2]) / 1000.0)
mc = int(sys.argv[2]) if len(sys.argv) > 2 else 100
print(f"{'previous -> next':70s} {'calls':>6s} {'median gap us':>14s} {'min':>8s} {'max':>8s}")
for (pa, pb), g in sorted(pairs.items(), key=lambda kv: -len(kv[1])):
    if len(g) >= mc:
        print(f"{pa[:34]:34s} -> {pb[:32]:32s} {len(g):6d} {statistics.median(g):14.3f} "
              f"{min(g):8.3f} {max(g):8.3f}")
