# 1-GPU benches: 70B TP=1 single pod (the driver's N=1 run) and one TP=8 rank's shapes (simulated).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/bench_tp1.json 2> gpurun_out/bench_tp1.err || { tail -20 gpurun_out/bench_tp1.err; exit 1; }
cat gpurun_out/bench_tp1.json
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --simulate-tp 8 ${BENCH_ARGS:-} > gpurun_out/bench_tp8sim.json 2> gpurun_out/bench_tp8sim.err || { tail -20 gpurun_out/bench_tp8sim.err; exit 1; }
cat gpurun_out/bench_tp8sim.json
