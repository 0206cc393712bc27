set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r17
timeout -k 10 300 python tools/kbench.py --tp 8 > gpurun_out/r17/kbench_tp8.txt 2>&1 && tail -6 gpurun_out/r17/kbench_tp8.txt
timeout -k 10 500 python -u bench.py --arrival-rate 3 --steps 40 --warmup 4 --batch 16 --json-out gpurun_out/r17/arrival_tp1.json > gpurun_out/r17/arrival_tp1.log 2>&1 || { tail -20 gpurun_out/r17/arrival_tp1.log; exit 1; }
cat gpurun_out/r17/arrival_tp1.json
export K8S_TP_BACKEND=gloo K8S_TP_COMM=xgmi
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 8 --steps 2 --warmup 1 > gpurun_out/r17/bench_tp8_rehearsal.json 2> gpurun_out/r17/bench_tp8_rehearsal.err \
  || { tail -30 gpurun_out/r17/bench_tp8_rehearsal.err; exit 1; }
cat gpurun_out/r17/bench_tp8_rehearsal.json
