set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r46; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_multigpu.py > $O/test_multigpu.log 2>&1 || { tail -40 $O/test_multigpu.log; exit 1; }
grep -E "PASS|SKIP|FAIL|rehearsal" $O/test_multigpu.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "graph or engine" > $O/test_model.log 2>&1 || { tail -30 $O/test_model.log; exit 1; }
tail -1 $O/test_model.log
K8S_TP_BACKEND=gloo K8S_TP_COMM=xgmi timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29519 \
  bench.py --gpus 8 --preset tiny-tp8 --gen-tokens 16 --steps 2 --warmup 1 --verbose --json-out $O/tiny_tp8_rehearsal.json > $O/tiny_tp8_rehearsal.log 2>&1 || { tail -30 $O/tiny_tp8_rehearsal.log; exit 1; }
cat $O/tiny_tp8_rehearsal.json
