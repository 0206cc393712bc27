set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/m1_trace; mkdir -p $O
K8S_SGEMV_MFMA_MIN_M=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 tools/probes/m1_trace.py > $O/m1.log 2>&1 || { tail -5 $O/m1.log; exit 1; }
python3 tools/probes/m1_parse.py $(ls $O/t/*kernel_trace.csv $O/t/*/*kernel_trace.csv 2>/dev/null | head -1) $O/m1.log
