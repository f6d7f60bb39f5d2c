"""Lab edit: scripts/lab/edits/neg0_slot.py, plus both task paths of the bins' piece sums
read a piece's two bounds unconditionally (one ds_read2 instead of a read and a second
one inside the validity branch). No arithmetic changes."""
import os
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "neg0_slot.py")).read())
p = "tpl_kcommon.h"
s = open(p).read()
OLD1 = """        const int jc = valid ? j : 0;
        const int st = starts[jc], nx = starts[jc + 1];
        const int b0 = valid ? st : 0;"""
NEW1 = """        const int jc = valid ? j : 0;
        int st = starts[jc], nx = starts[jc + 1];
        asm volatile("" : "+v"(st), "+v"(nx));
        const int b0 = valid ? st : 0;"""
assert OLD1 in s
s = s.replace(OLD1, NEW1)
OLD2 = """        const int jc = j < kTPB - 2 ? j : kTPB - 2;
        const int st = starts[jc], nx = starts[jc + 1];"""
NEW2 = """        const int jc = j < kTPB - 2 ? j : kTPB - 2;
        int st = starts[jc], nx = starts[jc + 1];
        asm volatile("" : "+v"(st), "+v"(nx));"""
assert OLD2 in s
s = s.replace(OLD2, NEW2)
open(p, "w").write(s)
