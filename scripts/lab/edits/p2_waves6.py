# Lab edit: k_p2_spmv built for at least 6 waves per SIMD (the 5M layout's int32-column
# variant takes 82 VGPRs, 5 waves, by default; 74 and 6 waves this way, no scratch).
s = open('tpl_kernels.hip').read()
a = '__launch_bounds__(kTPB, kSpmvMinWaves) void k_p2_spmv'
assert a in s
s = s.replace(a, '__launch_bounds__(kTPB, 6) void k_p2_spmv')
open('tpl_kernels.hip', 'w').write(s)
