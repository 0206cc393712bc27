set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r18
timeout -k 10 300 python -u bench.py --arrival-rate 3 --steps 40 --warmup 4 --batch 16 --json-out gpurun_out/r18/arrival_tp1.json 2>&1 | grep --line-buffered -v "Could not parse" > gpurun_out/r18/arrival_tp1.log || { tail -20 gpurun_out/r18/arrival_tp1.log; exit 1; }
cat gpurun_out/r18/arrival_tp1.json
export K8S_TP_BACKEND=gloo K8S_TP_COMM=xgmi
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 8 --steps 2 --warmup 1 --verbose --json-out gpurun_out/r18/bench_tp8_rehearsal.json 2>&1 | grep -v "Could not parse\|amdgpu.ids\|socket.cpp" | tee gpurun_out/r18/bench_tp8_rehearsal.log
