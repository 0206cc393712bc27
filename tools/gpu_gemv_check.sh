# After a GEMV launch change: kernel + model tests, then TP=8-shape and 8B benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/gemv_check; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_mgemm_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --simulate-tp 8 --steps 15 --warmup 2 > $O/tp8sim.json 2> $O/tp8sim.err || { tail -20 $O/tp8sim.err; exit 1; }
timeout -k 10 300 python -u bench.py --preset llama-3-8b --steps 10 --warmup 2 > $O/8b.json 2> $O/8b.err || { tail -20 $O/8b.err; exit 1; }
for f in tp8sim 8b; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decode_ms_per_step'], d['p50_decision_latency_ms'])" $O/$f.json $f; done
