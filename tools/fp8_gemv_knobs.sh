#!/bin/bash
# fp8 TP=1 decode (bench.py --dtype fp8) under the GEMV row-set knobs, one box, each row its own process.
# gpurun_out/$OUT/knobs.txt: "<knobs> decisions/s decode-ms".
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-fp8knobs}; mkdir -p "$O"
run() {  # run <tag> <env assignments...>
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --dtype fp8 --steps ${STEPS:-6} --warmup 2 > "$O/$tag.json" 2> "$O/$tag.err" || exit $?
  python -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', '$*', d['value'], d['decode_ms_per_step'])" | tee -a "$O/knobs.txt"
}
run base K8S_NONE=1
run loop0 K8S_GEMV_LOOP=0
run loop1 K8S_GEMV_LOOP=1
run loop3 K8S_GEMV_LOOP=3
run minmi64 K8S_GEMV_LOOP_MIN_MI=64
run kw2 K8S_GEMV_KW=2
run base2 K8S_NONE=1
