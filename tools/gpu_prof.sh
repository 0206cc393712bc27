# rocprofv3 kernel statistics of the decode path (one TP=8 rank's shapes, and TP=1), plus the
# 64-pod batched bench.  Summaries land in gpurun_out/rocprof_*.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPO="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_tp8" -o run -- python3 "$REPO/bench.py" --steps 2 --warmup 1 --simulate-tp 8 > "$REPO/gpurun_out/prof_tp8.log" 2>&1 || { tail -20 "$REPO/gpurun_out/prof_tp8.log"; exit 1; }
f=$(find "$REPO/gpurun_out/prof_tp8" -name "*kernel_stats.csv" | head -1)
python3 "$REPO/tools/prof_summary.py" "$f" 22 > "$REPO/gpurun_out/rocprof_70b_tp8sim_decode_kernels.txt" && cat "$REPO/gpurun_out/rocprof_70b_tp8sim_decode_kernels.txt"
cd "$REPO"
true
