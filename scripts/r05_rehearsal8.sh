#!/bin/bash
# Round-5 rehearsal of `bench.py --gpus 8` on a one-GPU box: eight ranks share GPU 0, the
# exchanges staged through host memory (TPL_DIST_TRANSPORT=host: a protocol check, not a
# rate). The line's parity block checks the assembled x against configs4_replicated_N8 and
# its `predicted` block is the N = 8 row of profiles/rank_share.json.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
echo "== N=8 host transport, replicated"
TPL_DEVICE=0 TPL_DIST_TRANSPORT=host timeout -k 10 900 python bench.py --gpus 8 --steps 1 --warmup 1 --profile-iters 3 --child-timeout 840 --rank-timeout 830 > "$OUT/rehearsal8.log" 2>&1 || { echo "rehearsal8 failed"; tail -30 "$OUT/rehearsal8.log"; exit 2; }
grep '^{' "$OUT/rehearsal8.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); pc=d.get('partitioned_configs4', d); print(d.get('status','ok'), 'value', d.get('value'), d.get('scaling'), d['ms_per_step'], '| partitioned', pc.get('value'), pc.get('ms_per_step'), pc['config']['parallelism'], '| parity', json.dumps(d.get('parity',{}).get('workloads')), '| predicted', json.dumps(pc.get('predicted'))[:300])"
