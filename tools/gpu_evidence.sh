# Round-3 evidence on one MI355X: serving under Poisson arrivals, one TP=8 rank's shapes, fp8 weights, the
# 256-node prompt, and rocprof kernel tables of the prefill-heavy (256 nodes) and fp8 batch-64 benches (no
# library GEMM may appear).  Each GPU step has its own limit; a timeout / abort / fault ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ev; mkdir -p $O
step() {  # step <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1
  local rc=$?
  echo "$log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$O/$log"; exit $rc; fi
  grep -h '"metric"' "$O/$log" | cut -c1-700
  return 0
}
for spec in ${RUNS:-arrivals tp8sim fp8 nodes256 prof256 proffp8b64}; do
  case $spec in
    default) step 300 bench_default.json python -u bench.py --steps 6 --warmup 2 ;;
    arrivals) step 420 bench_arrivals_rate3.json python -u bench.py --arrival-rate 3 --steps 40 --warmup 5 ;;
    tp8sim) step 300 bench_tp8sim.json python -u bench.py --simulate-tp 8 --steps 10 --warmup 2 ;;
    pf8) K8S_DECODE_PREFETCH_MB=48 step 300 bench_tp8sim_prefetch48.json python -u bench.py --simulate-tp 8 --steps 10 --warmup 2 ;;
    pf8b) K8S_DECODE_PREFETCH_MB=24 step 300 bench_tp8sim_prefetch24.json python -u bench.py --simulate-tp 8 --steps 10 --warmup 2 ;;
    pf1) K8S_DECODE_PREFETCH_MB=64 step 300 bench_tp1_prefetch64.json python -u bench.py --steps 4 --warmup 1 ;;
    fp8) step 300 bench_fp8_tp1.json python -u bench.py --dtype fp8 --steps 6 --warmup 2 ;;
    fp8b64) step 400 bench_fp8_tp1_b64.json python -u bench.py --dtype fp8 --batch 64 --steps 3 --warmup 1 ;;
    b64) step 400 bench_tp1_b64.json python -u bench.py --batch 64 --steps 3 --warmup 1 ;;
    nodes256) step 400 bench_nodes256.json python -u bench.py --nodes 256 --max-model-len 32768 --steps 3 --warmup 1 ;;
    prof256) bash tools/gpu_prof.sh tp1_nodes256 "--nodes 256 --max-model-len 32768" > $O/prof256.log 2>&1 || { tail -20 $O/prof256.log; exit 1; }
             head -16 gpurun_out/rocprof_70b_tp1_nodes256_kernels.txt ;;
    proftp1) bash tools/gpu_prof.sh tp1_default "" > $O/proftp1.log 2>&1 || { tail -20 $O/proftp1.log; exit 1; }
             cat gpurun_out/lastfwd_tp1_default.txt | head -60 ;;
    proftp8) bash tools/gpu_prof.sh tp8sim "--simulate-tp 8" > $O/proftp8.log 2>&1 || { tail -20 $O/proftp8.log; exit 1; }
             cat gpurun_out/lastfwd_tp8sim.txt | head -60 ;;
    proffp8b64) bash tools/gpu_prof.sh tp1_fp8_b64 "--dtype fp8 --batch 64" > $O/proffp8.log 2>&1 || { tail -20 $O/proffp8.log; exit 1; }
             head -16 gpurun_out/rocprof_70b_tp1_fp8_b64_kernels.txt ;;
  esac
done
