# rocprofv3 kernel statistics of a short bench run.  $1 = tag, $2 = extra bench args (default: one TP=8
# rank's shapes).  Summary lands in gpurun_out/rocprof_70b_<tag>_kernels.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPO="$GRAFT_REPO_ROOT"
TAG="${1:-tp8sim}"
ARGS="${2---simulate-tp 8}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_$TAG" -o run -- python3 "$REPO/bench.py" --steps 2 --warmup 1 $ARGS > "$REPO/gpurun_out/prof_$TAG.log" 2>&1 || { tail -20 "$REPO/gpurun_out/prof_$TAG.log"; exit 1; }
f=$(find "$REPO/gpurun_out/prof_$TAG" -name "*kernel_stats.csv" | head -1)
python3 "$REPO/tools/prof_summary.py" "$f" 30 > "$REPO/gpurun_out/rocprof_70b_${TAG}_kernels.txt" && cat "$REPO/gpurun_out/rocprof_70b_${TAG}_kernels.txt"
t=$(find "$REPO/gpurun_out/prof_$TAG" -name "*kernel_trace.csv" | head -1)
[ -n "$t" ] && python3 "$REPO/tools/last_forward.py" "$t" > "$REPO/gpurun_out/lastfwd_${TAG}.txt" 2>&1
rm -rf "$REPO/gpurun_out/prof_$TAG"   # raw traces stay on the box (gpurun copies back at most 64 MiB)
cd "$REPO"
true
