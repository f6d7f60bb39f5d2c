set -e
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/pp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/tune.py > $GRAFT_REPO_ROOT/gpurun_out/pp.log 2>&1
cut -d, -f1-4 $GRAFT_REPO_ROOT/gpurun_out/pp/run_kernel_stats.csv | cut -c1-150
