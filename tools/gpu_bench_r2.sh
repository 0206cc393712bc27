# End-to-end benches after the mgemm / GQA-attention / comm changes (70B, one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/b2
run() { tag=$1; shift; timeout -k 10 500 python -u bench.py "$@" > gpurun_out/b2/$tag.json 2> gpurun_out/b2/$tag.err || { echo "BENCH $tag FAILED"; tail -20 gpurun_out/b2/$tag.err; return 1; }; cat gpurun_out/b2/$tag.json; }
run tp1 --steps 8 --warmup 2 && \
K8S_GEMM=mgemm run tp1_allmgemm --steps 8 --warmup 2 && \
run tp8sim --steps 8 --warmup 2 --simulate-tp 8 && \
run tp1_b64 --steps 2 --warmup 1 --batch 64 && \
K8S_GEMM=library run tp1_b64_lib --steps 2 --warmup 1 --batch 64 && \
run tp8sim_b64 --steps 2 --warmup 1 --batch 64 --simulate-tp 8
