set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TPL_DEVICE=0 TPL_DIST_TRANSPORT=host timeout -k 10 500 python bench.py --gpus 2 --steps 1 --warmup 1 --profile-iters 5 --child-timeout 450 --rank-timeout 440 > gpurun_out/reh2.log 2>&1 || { echo "failed"; tail -20 gpurun_out/reh2.log; exit 2; }
grep '^{' gpurun_out/reh2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); pc=d.get('partitioned_configs4', {}); print(d.get('value'), d.get('scaling'), pc.get('value'), pc.get('scaling'), d['parity']['all_ok'], list(d['parity']['workloads']))"
