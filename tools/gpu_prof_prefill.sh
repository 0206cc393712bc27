# rocprofv3 kernel statistics of the prefill probe (one TP=8 rank's shapes, 256-token chunks).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPO="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_prefill" -o run -- python3 "$REPO/tools/prefill_probe.py" --simulate-tp ${TP:-8} > "$REPO/gpurun_out/prof_prefill.log" 2>&1 || { tail -20 "$REPO/gpurun_out/prof_prefill.log"; exit 1; }
f=$(find "$REPO/gpurun_out/prof_prefill" -name "*kernel_stats.csv" | head -1)
python3 "$REPO/tools/prof_summary.py" "$f" 40 > "$REPO/gpurun_out/rocprof_prefill_tp${TP:-8}.txt" && cat "$REPO/gpurun_out/rocprof_prefill_tp${TP:-8}.txt"
