"""Average rocprofv3 --pmc counter values per kernel (dev tool). Args: counter csv files."""
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    with open(path) as f:
        for r in csv.DictReader(f):
            k = r.get("Kernel_Name", "?")
            k = k.split("(")[0].replace("void tpl::", "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v)/len(v):16.1f}  (n={len(v)})")
