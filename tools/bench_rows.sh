#!/bin/bash
# The bench rows docs/PERF.md and docs/STATUS.md quote, on one MI355X (one gpurun call, each row under its own
# limit): default (the driver's N=1 run), --simulate-tp 8 (one TP=8 rank's shapes), --batch 64 (config 4 at N=1),
# --batch 8, --dtype fp8.  ROWS picks a subset; output: gpurun_out/$OUT/rows.jsonl (one tagged JSON line per row).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-rows}; mkdir -p "$O"
row() {  # row <tag> <seconds> <bench args...>
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "$O/$tag.json" 2> "$O/$tag.err"
  local rc=$?
  echo "$tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$O/$tag.err"; [ $rc -ne 1 ] && exit $rc; return 0; fi
  python -c "import json,sys; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); d['row']='$tag'; print(json.dumps(d))" >> "$O/rows.jsonl"
  tail -1 "$O/rows.jsonl" | cut -c1-300
}
for r in ${ROWS:-default tp8sim b64 b8 fp8}; do
  case $r in
    default) row default 300 --steps 10 --warmup 2 ;;
    tp8sim)  row tp8sim 240 --simulate-tp 8 --steps 10 --warmup 2 ;;
    tp8sim_b64) row tp8sim_b64 300 --simulate-tp 8 --batch 64 --steps 3 --warmup 1 ;;
    b64)     row b64 400 --batch 64 --steps 3 --warmup 1 ;;
    b8)      row b8 300 --batch 8 --steps 5 --warmup 1 ;;
    fp8)     row fp8 300 --dtype fp8 --steps 10 --warmup 2 ;;
    fp8_b64) row fp8_b64 400 --dtype fp8 --batch 64 --steps 3 --warmup 1 ;;
    nodes256) row nodes256 900 --nodes 256 --max-model-len 32768 --steps 10 --warmup 1 ;;
    gen200)  row gen200 400 --gen-tokens 200 --steps 5 --warmup 1 ;;
    *) echo "unknown row $r"; exit 2 ;;
  esac
done
