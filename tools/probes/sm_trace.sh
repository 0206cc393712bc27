# kernel-trace (no counters) of the small-batch sgemv forms on the 70B TP=1 shapes, M rows, both forms
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sm_trace; mkdir -p $O
for M in ${MS:-8 16}; do
  for form in ${FORMS:-5 17}; do
    [ $M -gt 8 ] && [ $form -gt 16 ] && continue
    tag=m${M}_f${form}
    M=$M K8S_SGEMV_MFMA_MIN_M=$form timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- python3 tools/probes/sm_trace.py > $O/$tag.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$tag rc=$rc"; tail -5 $O/$tag.log; exit $rc; }
    echo "== M=$M form=$( [ $form -le $M ] && echo mfma || echo dot2 )"
    python3 tools/probes/sm_trace_parse.py $(ls $O/$tag/*kernel_trace.csv $O/$tag/*/*kernel_trace.csv 2>/dev/null | head -1) $O/$tag.log
  done
done
