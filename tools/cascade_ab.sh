#!/bin/bash
# Cascade decode attention A/B on one MI355X: batched decisions on one cluster snapshot with the cluster-first
# prompt layout (every prompt of a step shares the cluster block), K8S_DECODE_CASCADE=1 (default) vs 0, then a
# rocprofv3 per-layer view of the cascade run.  NODES / BATCH pick the config; output gpurun_out/$OUT/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-cascade}; mkdir -p "$O"
N=${NODES:-64}; B=${BATCH:-16}; ML=${MAXLEN:-8192}
ARGS="--nodes $N --batch $B --prompt-layout cluster_first --max-model-len $ML --steps ${STEPS:-3} --warmup 1"
for c in 1 0; do
  K8S_DECODE_CASCADE=$c timeout -k 10 600 python -u bench.py $ARGS > "$O/cas$c.json" 2> "$O/cas$c.err"
  rc=$?; echo "cascade=$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/cas$c.err"; exit $rc; }
  python -c "import json; d=json.loads(open('$O/cas$c.json').read().strip().splitlines()[-1]); print('cascade=$c', d['value'], 'decisions/s decode', d['decode_ms_per_step'], 'ms prefill', d['prefill_ms_per_decision'])"
done
[ -n "$PROF" ] && timeout -k 10 700 bash tools/gpu_prof.sh "cas_n${N}_b${B}" "--nodes $N --batch $B --prompt-layout cluster_first --max-model-len $ML"
true
