# Lab edit: pass one's w stored plain (kept in the writing XCD's L2 for k_p1_axpy).
s = open("tpl_kcommon.h").read()
a = "    st_out(W + i, w);\n"
assert a in s
s = s.replace(a, "    W[i] = w;\n", 1)
open("tpl_kcommon.h", "w").write(s)
