mkdir -p gpurun_out
L=$PWD/two-pass-lanczos_amd/ab/libtpl_lab.so
REPS=3 timeout -k 10 600 bash scripts/env_ab.sh base "TPL_LIB_PATH=$L TPL_BIN_BIG=16" "TPL_LIB_PATH=$L TPL_BIN_BIG=16 TPL_BIN_SMALL=32" > gpurun_out/ab_bincap2.txt 2>&1
cat gpurun_out/ab_bincap2.txt
