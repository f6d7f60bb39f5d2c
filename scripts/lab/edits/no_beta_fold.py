# Lab edit: the replicated partition's beta rank total as its own launch (k_reorth_reduce)
# again, instead of k_p1_axpy's last workgroup (the round-5 fold) — the A/B for it.
s = open("tpl_runtime.cpp").read()
a = "bool beta_folded(const tpl_op_s* op, const CsrDev& A) { return op->hybrid && A.G2 <= 1024; }"
assert a in s
s = s.replace(a, "bool beta_folded(const tpl_op_s*, const CsrDev&) { return false; }", 1)
open("tpl_runtime.cpp", "w").write(s)
