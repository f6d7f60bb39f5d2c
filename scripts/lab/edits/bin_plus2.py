"""Lab probe (timing only, bits unchanged): two extra 4-B loads per thread in the long-row
bins (the bin table's starts of two pieces), waited on after the piece sums. Separates
scripts/lab/edits/preload_starts.py's cost into its loads and its use (round 6)."""
p = "tpl_kcommon.h"
s = open(p).read()
OLD1 = """  const BinSeg sg = A.b_seg[bin * kTPB + (t < npieces ? t : npieces)];
"""
NEW1 = """  const BinSeg sg = A.b_seg[bin * kTPB + (t < npieces ? t : npieces)];
  const int dj = (t >> 3) < npieces ? (t >> 3) : npieces;
  const int dmy0 = A.b_seg[bin * kTPB + dj].start, dmy1 = A.b_seg[bin * kTPB + (dj + 1 < npieces ? dj + 1 : npieces)].start;
"""
assert OLD1 in s
s = s.replace(OLD1, NEW1)
OLD2 = """  TPL_MARK(3);
  // the finalising thread's row entries"""
NEW2 = """  TPL_MARK(3);
  asm volatile("" ::"v"(dmy0), "v"(dmy1));
  // the finalising thread's row entries"""
assert OLD2 in s
s = s.replace(OLD2, NEW2)
open(p, "w").write(s)
