# Lab edit: beta of k_p1_spmv from ONE norm partial per thread (thread t loads P[t], G2 <= 256
# assumed), wave sums exchanged through LDS behind an lgkmcnt-only barrier — the same tree
# (bitwise), 6 fewer VGPRs live across the gathers than four loads per lane.
s = open("tpl_kernels.hip").read()
a = "  PartialRegs<4> pr;           // G2 <= 1024\n"
assert a in s
s = s.replace(a, "  double pr1;\n", 1)
a = "  load_partials_sel(S.Pb_r, A.G2_r, wave_red, pr);\n"
assert a in s
s = s.replace(a, "  pr1 = S.Pb_r[clampi(threadIdx.x, A.G2_r - 1)];\n  (void)wave_red;\n", 1)
a = """    const double beta = sqrt(wave_red ? finish_partials_wave(A.G2_r, pr)
                                      : finish_partials(S.Pb_r, A.G2_r, pr, red));"""
assert a in s
s = s.replace(a, """    double sv = 0.0;
    if ((int)threadIdx.x < A.G2_r) sv = sv + pr1;
    sv = wave_sum(sv);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sv;
    asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory");
    const double beta = sqrt((red[0] + red[1]) + (red[2] + red[3]));""", 1)
# red is also used by the alpha tail (block_sum_tail): separate the two uses
a = "  __shared__ double red[4];\n  extern __shared__ double lds[];\n  pin_layout_args(A);\n  asm volatile(\"\" ::\"s\"(S.Pb_r)"
assert a in s
s = s.replace(a, "  __shared__ double red[4];\n  __shared__ double redb[4];\n  extern __shared__ double lds[];\n  pin_layout_args(A);\n  asm volatile(\"\" ::\"s\"(S.Pb_r)", 1)
s = s.replace("    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sv;", "    if ((threadIdx.x & 63) == 0) redb[threadIdx.x >> 6] = sv;", 1)
s = s.replace("    const double beta = sqrt((red[0] + red[1]) + (red[2] + red[3]));", "    const double beta = sqrt((redb[0] + redb[1]) + (redb[2] + redb[3]));", 1)
open("tpl_kernels.hip", "w").write(s)
