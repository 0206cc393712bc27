# Rehearse the multi-rank bench path on a 1-GPU box: 2 ranks share the GPU (torchrun), gloo process
# group + xGMI peer-memory collectives (RCCL cannot put two ranks on one GPU).  70B at TP=2 = 2 x 70 GB.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 K8S_TP_BACKEND=gloo K8S_TP_COMM=xgmi
mkdir -p gpurun_out
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps ${STEPS:-2} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench_tp2_rehearsal.json 2> gpurun_out/bench_tp2_rehearsal.err \
  || { tail -30 gpurun_out/bench_tp2_rehearsal.err; exit 1; }
cat gpurun_out/bench_tp2_rehearsal.json
