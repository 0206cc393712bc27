#!/bin/bash
# the headline's full-depth 70B engine as 8 rank processes sharing the ONE GPU of a gpurun box
# (correctness and exit code only; time-shared ranks say nothing about speed): the 70B-shape rehearsal test at fp8
# TP = 4, then `bench.py --gpus 8` (TP = 8) and `bench.py --gpus 8 --tp 4 --dtype fp8` (two TP = 4 replicas).
# Eight processes time-sharing one GPU stall the fused GEMV all-reduce's 70B-shape launches at random
# (profiles/fused_ar_70b_shapes_r6.txt), so these runs take the separate GEMV + xGMI all-reduce (K8S_FUSED_AR=0).
#   gpurun --timeout 1200 -- 'bash tools/rehearsal_full_depth.sh'
mkdir -p gpurun_out/g5 && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -v -s --timeout 290 --timeout-method thread tests/test_multigpu_70b.py -k fp8 > gpurun_out/g5/r70fp8.log 2>&1
echo "fp8 test rc=$?"
K8S_FUSED_AR=0 timeout -k 10 900 python -u bench.py --gpus 8 --gen-tokens 4 --steps 2 --warmup 1 > gpurun_out/g5/bench_tp8_full.json 2> gpurun_out/g5/bench_tp8_full.err
rc=$?; echo "tp8 full-depth rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
K8S_FUSED_AR=0 timeout -k 10 900 python -u bench.py --gpus 8 --tp 4 --dtype fp8 --gen-tokens 4 --steps 2 --warmup 1 > gpurun_out/g5/bench_dp2tp4_fp8.json 2> gpurun_out/g5/bench_dp2tp4_fp8.err
echo "dp2-tp4 fp8 rc=$?"
