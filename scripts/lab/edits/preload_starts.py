"""Lab edit (scripts/build_variant_src.sh pst scripts/lab/edits/preload_starts.py): the
long-row bins' first round of piece sums takes its piece bounds from registers — each
lane loads b_seg[j].start and b_seg[j + 1].start of its first-round piece j from global
memory with the entries — instead of two dependent LDS reads of `starts` after the
staging barrier. Later rounds still read `starts`. No arithmetic changes."""
p = "tpl_kcommon.h"
s = open(p).read()

OLD1 = """  const int npieces = hdr & 0xFFFF, nbig = hdr >> 16;
  const BinSeg sg = A.b_seg[bin * kTPB + (t < npieces ? t : npieces)];
"""
NEW1 = """  const int npieces = hdr & 0xFFFF, nbig = hdr >> 16;
  const BinSeg sg = A.b_seg[bin * kTPB + (t < npieces ? t : npieces)];
  // first-round piece bounds in registers (the wave's task wv: see the piece sums below)
  int pj0, pj1;
  {
    const int lane0 = t & 63, wv0 = t >> 6;
    const int tb0 = (nbig + 3) >> 2;
    const int j0 = wv0 < tb0 ? 4 * wv0 + (lane0 >> 4) : nbig + 8 * (wv0 - tb0) + (lane0 >> 3);
    const int jc0 = j0 < npieces ? j0 : npieces;
    const int jn0 = jc0 + 1 < npieces ? jc0 + 1 : npieces;
    pj0 = A.b_seg[bin * kTPB + jc0].start;
    pj1 = A.b_seg[bin * kTPB + jn0].start;
  }
"""
assert OLD1 in s
s = s.replace(OLD1, NEW1)

OLD2 = """        const int jc = valid ? j : 0;
        const int st = starts[jc], nx = starts[jc + 1];
        const int b0 = valid ? st : 0;
        const int en = valid ? (nx >= 0 ? nx : -1 - nx) : 0;
        // this lane's entries k + 16q"""
NEW2 = """        const int jc = valid ? j : 0;
        int b0, en;
        if (task == wv) {  // first round: preloaded
          b0 = valid ? pj0 : 0;
          en = valid ? pj1 : 0;
        } else {
          const int st = starts[jc], nx = starts[jc + 1];
          b0 = valid ? st : 0;
          en = valid ? (nx >= 0 ? nx : -1 - nx) : 0;
        }
        // this lane's entries k + 16q"""
assert OLD2 in s
s = s.replace(OLD2, NEW2)

OLD3 = """        const int jc = j < kTPB - 2 ? j : kTPB - 2;
        const int st = starts[jc], nx = starts[jc + 1];
        const bool valid = j < npieces;
        const int b0 = valid ? st : 0;
        const int en = valid ? (nx >= 0 ? nx : -1 - nx) : 0;"""
NEW3 = """        const int jc = j < kTPB - 2 ? j : kTPB - 2;
        const bool valid = j < npieces;
        int b0, en;
        if (task == wv) {  // first round: preloaded
          b0 = valid ? pj0 : 0;
          en = valid ? pj1 : 0;
        } else {
          const int st = starts[jc], nx = starts[jc + 1];
          b0 = valid ? st : 0;
          en = valid ? (nx >= 0 ? nx : -1 - nx) : 0;
        }"""
assert OLD3 in s
s = s.replace(OLD3, NEW3)
open(p, "w").write(s)
