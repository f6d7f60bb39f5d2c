# Lab edit: pass one's w stored non-temporal.
s = open("tpl_kcommon.h").read()
a = "    st_out(W + i, w);\n"
assert a in s
s = s.replace(a, "    __builtin_nontemporal_store(w, W + i);\n", 1)
open("tpl_kcommon.h", "w").write(s)
