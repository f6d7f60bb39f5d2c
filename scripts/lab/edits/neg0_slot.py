"""Lab edit (scripts/build_variant_src.sh neg0 scripts/lab/edits/neg0_slot.py): the bins'
piece sums read -0.0 from a reserved LDS slot for the entries past a piece's end (the
address select stays, the two value selects per entry go). x + (-0.0) is x bit for bit,
as with the select it replaces. One more double of dynamic LDS per bin workgroup."""
p = "tpl_kcommon.h"
s = open(p).read()

OLD0 = """  starts[t] = sg.ri < 0 ? -1 - sg.start : sg.start;  // < 0: no piece (value encodes the fill)
"""
NEW0 = """  starts[t] = sg.ri < 0 ? -1 - sg.start : sg.start;  // < 0: no piece (value encodes the fill)
  const int kNeg0 = A.bin_cap + kTPB / 2 + kTPB;  // one double of -0.0 after the piece sums
  if (t == 0) lds[kNeg0] = -0.0;
"""
assert OLD0 in s
s = s.replace(OLD0, NEW0)

OLD1 = """          for (int u = 0; u < 8; ++u) v[u] = lds[u < rem ? k + 16 * u : k];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc = acc + (u < rem ? v[u] : -0.0);"""
NEW1 = """          for (int u = 0; u < 8; ++u) v[u] = lds[u < rem ? k + 16 * u : kNeg0];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc = acc + v[u];"""
assert OLD1 in s
s = s.replace(OLD1, NEW1)

OLD2 = """          for (int u = 0; u < 8; ++u) v[u] = lds[k0 + 8 * u < en ? k0 + 8 * u : k0];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc = acc + (k0 + 8 * u < en ? v[u] : -0.0);"""
NEW2 = """          for (int u = 0; u < 8; ++u) v[u] = lds[k0 + 8 * u < en ? k0 + 8 * u : kNeg0];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc = acc + v[u];"""
assert OLD2 in s
s = s.replace(OLD2, NEW2)
open(p, "w").write(s)

p = "tpl_kernels.hip"
s = open(p).read()
OLD3 = "? (size_t)A.bin_cap * sizeof(double) + kTPB * sizeof(int) + kTPB * sizeof(double)"
NEW3 = "? (size_t)A.bin_cap * sizeof(double) + kTPB * sizeof(int) + (kTPB + 1) * sizeof(double)"
assert OLD3 in s
s = s.replace(OLD3, NEW3)
open(p, "w").write(s)
