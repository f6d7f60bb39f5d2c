# Lab edit: k_p1_axpy's norm partials stored write-through (read next by every k_p1_spmv
# workgroup on all XCDs).
s = open("tpl_kernels.hip").read()
a = "  if (threadIdx.x == 0) S.Pb[rb] = p;  // plain: write-through measured +0.35 us here\n"
assert a in s
s = s.replace(a, "  if (threadIdx.x == 0) st_out(S.Pb + rb, p);\n", 1)
open("tpl_kernels.hip", "w").write(s)
