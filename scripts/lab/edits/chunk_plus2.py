"""Lab probe (timing only, bits unchanged): two extra 8-B loads per thread in the short
chunks (xsrc at the rows' neighbours), waited on with the rows' own entries. Measures how
much one more memory instruction per chunk wave costs the SpMV (round 6)."""
p = "tpl_kcommon.h"
s = open(p).read()
OLD = """  for (int q = 0; q < kRowsPerThread; ++q) pre[q] = epi.pre(row[q]);
  const Scale sc = scale_of();
  TPL_MARK(1);
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q) keep_pre(pre[q]);
"""
NEW = """  for (int q = 0; q < kRowsPerThread; ++q) pre[q] = epi.pre(row[q]);
  double dmy[kRowsPerThread];
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q) dmy[q] = xsrc[row[q] ^ 1];
  const Scale sc = scale_of();
  TPL_MARK(1);
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q) keep_pre(pre[q]);
#pragma unroll
  for (int q = 0; q < kRowsPerThread; ++q) asm volatile("" ::"v"(dmy[q]));
"""
assert OLD in s
s = s.replace(OLD, NEW)
open(p, "w").write(s)
