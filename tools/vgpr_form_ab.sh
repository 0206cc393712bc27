# GPU suite, then bench.py defaults and --batch 64 / --batch 8 rows (one box) -- the A/B arm for a build-flag change.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-vgpr_ab}; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > "$O/tests.log" 2>&1; rc=$?
tail -n 1 "$O/tests.log"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for args in "--steps 6 --warmup 2" "--batch 64 --steps 3 --warmup 1" "--batch 8 --steps 5 --warmup 1"; do
  timeout -k 10 400 python -u bench.py $args > "$O/b.json" 2> "$O/b.err" || exit 1
  python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$args', d['value'], d['decode_ms_per_step'], d['prefill_ms_per_decision'], d['prefill_ms_per_step'])" | tee -a "$O/summary.txt"
done
