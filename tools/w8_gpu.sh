set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/w8; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mgemm_gpu.py -k "w8" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/mgemm_tune.py --w8 --tp 1 4 --m 32 64 128 --only qkv o_proj gate_up down --write --json-out $O/tune.json > $O/tune.log 2>&1; rc=$?; cat $O/tune.log | grep -v "^    cand"; [ $rc -eq 0 ] || exit $rc
cp k8s_llm_scheduler_amd/engine/assets/mgemm_gfx950.json $O/
for w in 0 1; do
  K8S_MGEMM_W8=$w timeout -k 10 600 python -u bench.py --dtype fp8 --batch 64 --steps 3 --warmup 1 > $O/bench_fp8_b64_w8_$w.json 2>&1; rc=$?; tail -1 $O/bench_fp8_b64_w8_$w.json | cut -c1-600; [ $rc -eq 0 ] || exit $rc
done
