set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r45; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests_full.log 2>&1 || { tail -40 $O/gpu_tests_full.log; exit 1; }
tail -2 $O/gpu_tests_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log | cut -c1-100
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err && cat $O/bench_default.json
bash tools/gpu_prof.sh tp1_r2_final "" > /dev/null && head -14 gpurun_out/rocprof_70b_tp1_r2_final_kernels.txt
