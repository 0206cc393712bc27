#!/bin/bash
# Decode attention route A/B: the small-grid split kernel (one wave per 64-token chunk) up to K8S_ATTN_SPLIT_PAIRS
# (sequence, kv head) pairs vs the one-workgroup kernel; bench.py at a few batch sizes.  gpurun_out/$OUT/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-splitab}; mkdir -p "$O"
for B in ${BATCHES:-8 16}; do
  for P in ${PAIRS:-32 128}; do
    K8S_ATTN_SPLIT_PAIRS=$P timeout -k 10 400 python -u bench.py --batch $B --steps ${STEPS:-5} --warmup 1 > "$O/b${B}_p$P.json" 2> "$O/b${B}_p$P.err" || exit $?
    python -c "import json; d=json.loads(open('$O/b${B}_p$P.json').read().strip().splitlines()[-1]); print('batch $B pairs $P', d['value'], d['decode_ms_per_step'])"
  done
done
