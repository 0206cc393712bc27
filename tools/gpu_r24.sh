set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r24; mkdir -p $O
for R in 2 3; do
timeout -k 10 300 python -u bench.py --arrival-rate $R --steps 40 --warmup 4 --batch 16 --json-out $O/arrival_r$R.json > $O/arrival_r$R.log 2>&1 && cat $O/arrival_r$R.json || exit 1
done
