set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r19; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sampler or nucleus" > $O/test_sampler.log 2>&1 || { tail -30 $O/test_sampler.log; exit 1; }
tail -3 $O/test_sampler.log
timeout -k 10 300 python tools/kbench.py --tp 8 > $O/kbench_tp8.txt 2>&1 && grep sampler $O/kbench_tp8.txt
timeout -k 10 300 python -u bench.py --batch 8 --steps 2 --warmup 1 --json-out $O/b8.json > $O/b8.log 2>&1 && cat $O/b8.json
timeout -k 10 300 python -u bench.py --batch 16 --steps 2 --warmup 1 --json-out $O/b16.json > $O/b16.log 2>&1 && cat $O/b16.json
timeout -k 10 300 python -u bench.py --top-p 0.9 --steps 3 --warmup 1 --json-out $O/topp.json > $O/topp.log 2>&1 && cat $O/topp.json
K8S_TP_BACKEND=gloo K8S_TP_COMM=xgmi timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29519 \
  bench.py --gpus 8 --preset tiny-tp8 --gen-tokens 16 --steps 2 --warmup 1 --verbose --json-out $O/tiny_tp8_rehearsal.json > $O/tiny_tp8_rehearsal.log 2>&1 || { tail -30 $O/tiny_tp8_rehearsal.log; exit 1; }
cat $O/tiny_tp8_rehearsal.json
