# A/B of the one-GPU TP rehearsals (tests/test_multigpu.py) with and without sgemv (K8S_SGEMV), one step per arm,
# each under its own time limit; results in gpurun_out/r4/mg*.log
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r4
for spec in ${ARMS:-"4 1" "2 1"}; do
  set -- $spec
  K8S_SGEMV=$2 timeout -k 10 300 python -u -m pytest "tests/test_multigpu.py::test_tp_rehearsal_ranks_share_one_gpu[$1]" -x -q -s --timeout 280 --timeout-method thread > gpurun_out/r4/mg$1_sgemv$2.log 2>&1
  rc=$?
  echo "world $1 sgemv $2 rc=$rc"; grep -E "passed|failed|timed out" gpurun_out/r4/mg$1_sgemv$2.log | head -3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
