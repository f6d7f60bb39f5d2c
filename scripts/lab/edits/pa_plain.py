# Lab edit: k_p1_spmv's alpha partials (chunk totals and long-row products) stored plain.
s = open("tpl_kernels.hip").read()
a = "  if (threadIdx.x == 0) st_out(S.Pa + slot, p);\n}"
assert a in s
s = s.replace(a, "  if (threadIdx.x == 0) S.Pa[slot] = p;\n}", 1)
open("tpl_kernels.hip", "w").write(s)
k = open("tpl_kcommon.h").read()
a = "  __device__ __forceinline__ void long_alpha(int r, double acc) const { st_out(Pa_long + r, acc); }"
assert a in k
k = k.replace(a, "  __device__ __forceinline__ void long_alpha(int r, double acc) const { Pa_long[r] = acc; }", 1)
open("tpl_kcommon.h", "w").write(k)
