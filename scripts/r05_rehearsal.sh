#!/bin/bash
# Round-5 rehearsal of the N > 1 bench path on a one-GPU box: two ranks share GPU 0, the
# exchanges staged through host memory (TPL_DIST_TRANSPORT=host: a protocol check, not a
# rate). Both partitions; each line's parity block checks the assembled x against the
# partition oracle's digest, and the replicated line carries the `predicted` block.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
for mode in ${MODES:-replicated rows}; do
  echo "== N=2 host transport, $mode"
  TPL_DEVICE=0 TPL_DIST_TRANSPORT=host timeout -k 10 500 python bench.py --gpus 2 --steps 1 --warmup 1 --profile-iters 5 --dist-mode $mode --child-timeout 450 --rank-timeout 440 > "$OUT/rehearsal_$mode.log" 2>&1 || { echo "rehearsal $mode failed"; tail -20 "$OUT/rehearsal_$mode.log"; exit 2; }
  grep '^{' "$OUT/rehearsal_$mode.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); pc=d.get('partitioned_configs4', d); print(d.get('status','ok'), 'value', d.get('value'), d.get('scaling'), d['ms_per_step'], '| partitioned', pc.get('value'), pc.get('ms_per_step'), pc['config']['parallelism'], '| parity', json.dumps(d.get('parity',{}).get('workloads')), '| predicted', json.dumps(pc.get('predicted'))[:300])"
done
