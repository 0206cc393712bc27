# GPU steps for one MI355X box (run through gpurun): RUNS="step step ..." picks them, default "tests smoke bench".
#   tests       pytest -m gpu (the driver's round-end suite)
#   smoke       __graft_entry__.smoke()
#   bench       bench.py defaults (the driver's N=1 run)
#   tp8sim      bench.py --simulate-tp 8 (one TP=8 rank's shapes, collectives skipped)
#   b64         bench.py --batch 64 (config 4 at N=1)
#   fp8         bench.py --dtype fp8 (config 5 shapes at TP=1) and --dtype fp8 --simulate-tp 4
#   prof        rocprofv3 kernel stats + last-forward timeline of the default bench (tools/gpu_prof.sh)
#   proftp8     the same for --simulate-tp 8
#   kbench      tools/kbench.py per-kernel microbench at TP=1 and TP=8 shapes
#   nodes256    bench.py --nodes 256 (22k-token prompts), 10 timed steps
#   gen200      bench.py --gen-tokens 200 (the reference's max_tokens) at TP=1 and --simulate-tp 8
# Each step has its own time limit; test failures (rc 1) do not stop later steps, a timeout / abort / fault (any other
# rc) ends the script.  Logs land in gpurun_out/$OUT (default run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${OUT:-run}; mkdir -p "$O"
step() {  # step <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1
  local rc=$?
  echo "$log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$O/$log"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
for spec in ${RUNS:-tests smoke bench}; do
  case $spec in
    tests)   step 1100 gpu_tests.log $PT -m gpu tests; tail -3 "$O/gpu_tests.log" ;;
    smoke)   step 300 smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"; tail -2 "$O/smoke.log" ;;
    bench)   step 400 bench_default.json python -u bench.py --steps ${STEPS:-10} --warmup 2; tail -1 "$O/bench_default.json" ;;
    tp8sim)  step 400 bench_tp8sim.json python -u bench.py --simulate-tp 8 --steps ${STEPS:-10} --warmup 2
             tail -1 "$O/bench_tp8sim.json" ;;
    b64)     step 600 bench_b64.json python -u bench.py --batch 64 --steps ${STEPS:-3} --warmup 1; tail -1 "$O/bench_b64.json" ;;
    fp8)     step 400 bench_fp8.json python -u bench.py --dtype fp8 --steps ${STEPS:-10} --warmup 2; tail -1 "$O/bench_fp8.json"
             step 400 bench_fp8_tp4sim.json python -u bench.py --dtype fp8 --simulate-tp 4 --steps ${STEPS:-10} --warmup 2
             tail -1 "$O/bench_fp8_tp4sim.json" ;;
    prof)    step 700 prof_default.log bash tools/gpu_prof.sh default ""; cat "$O/prof_default.log" | head -25 ;;
    proftp8) step 700 prof_tp8sim.log bash tools/gpu_prof.sh tp8sim "--simulate-tp 8"
             head -25 "$O/prof_tp8sim.log" ;;
    nodes256) step 900 bench_nodes256.json python -u bench.py --nodes 256 --max-model-len 32768 --steps ${STEPS:-10} --warmup 1
             tail -1 "$O/bench_nodes256.json" ;;
    gen200)  step 600 bench_gen200.json python -u bench.py --gen-tokens 200 --steps ${STEPS:-10} --warmup 2
             tail -1 "$O/bench_gen200.json"
             step 400 bench_tp8sim_gen200.json python -u bench.py --gen-tokens 200 --simulate-tp 8 --steps ${STEPS:-10} --warmup 2
             tail -1 "$O/bench_tp8sim_gen200.json" ;;
    kbench)  step 300 kbench_tp1.txt python -u tools/kbench.py --tp 1; step 300 kbench_tp8.txt python -u tools/kbench.py --tp 8 ;;
    *) echo "unknown step $spec"; exit 2 ;;
  esac
done
