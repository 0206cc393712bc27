# GEMV default change + speculative decoding: tests, then benches (TP=8 shapes, 8B, 70B TP=1 with and without drafts).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/spec; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_speculative_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_mgemm_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  timeout -k 10 400 python -u bench.py $2 > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['decode_ms_per_step'], d['p50_decision_latency_ms'], d.get('speculative'))" $O/$1.json $1
}
run tp8sim "--simulate-tp 8 --steps 15 --warmup 2"
run 8b "--preset llama-3-8b --steps 10 --warmup 2"
run 8b_spec4 "--preset llama-3-8b --steps 10 --warmup 2 --speculative 4"
run tp1 "--steps 5 --warmup 1"
run tp1_spec4 "--steps 5 --warmup 1 --speculative 4"
