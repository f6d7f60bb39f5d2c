# Lab edit (timing bound only, WRONG results): k_p1_spmv takes beta = 1 without loading or
# reducing the norm partials — what pass one would cost with beta as a ready scalar.
s = open("tpl_kernels.hip").read()
a = "  load_partials_sel(S.Pb_r, A.G2_r, wave_red, pr);\n"
assert a in s
s = s.replace(a, "  (void)pr;\n", 1)
a = """    const double beta = sqrt(wave_red ? finish_partials_wave(A.G2_r, pr)
                                      : finish_partials(S.Pb_r, A.G2_r, pr, red));"""
assert a in s
s = s.replace(a, "    const double beta = 1.0 + 0.0 * (double)j;\n    (void)wave_red;", 1)
open("tpl_kernels.hip", "w").write(s)
