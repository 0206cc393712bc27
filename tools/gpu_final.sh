# End-of-round verification: full GPU suite, smoke(), the driver's default bench, rocprof kernel table of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/final; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; grep -E "FAILED|Error" $O/gpu_tests.log | head -20; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
K8S_SMOKE=1 timeout -k 10 300 python -u __graft_entry__.py > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
bash tools/gpu_prof.sh tp1_final "" > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
head -16 gpurun_out/rocprof_70b_tp1_final_kernels.txt
timeout -k 10 600 python -u tools/spec_probe.py --preset llama-3.3-70b --reps 2 > $O/spec_probe_70b.jsonl 2> $O/spec_probe_70b.err || { tail -20 $O/spec_probe_70b.err; exit 1; }
cat $O/spec_probe_70b.jsonl
timeout -k 10 400 python -u tools/spec_probe.py --preset llama-3-8b > $O/spec_probe_8b.jsonl 2> $O/spec_probe_8b.err || { tail -20 $O/spec_probe_8b.err; exit 1; }
cat $O/spec_probe_8b.jsonl
