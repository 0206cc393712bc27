# PMC counters of pgemm vs the library GEMM on one shape (one counter pass per rocprofv3 run), then a
# verbose tuning sweep of the given shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPO="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
ARGS="${PROBE_ARGS:---m 2048 --n 8192 --k 8192}"
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --stats -d "$REPO/gpurun_out/pmc/p$i" -o run --output-format csv -- python3 "$REPO/tools/pgemm_pmc_probe.py" $ARGS > "$REPO/gpurun_out/pmc/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$REPO/gpurun_out/pmc/p$i.log"; }
done
cd "$REPO"
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt 2>&1; cat gpurun_out/pmc/summary.txt
timeout -k 10 ${TUNE_TIMEOUT:-300} python -u tools/pgemm_tune.py ${TUNE_ARGS:---tp 1 --m 256 --only qkv o_proj --verbose} > gpurun_out/pgemm_tune_v.txt 2>&1 || { tail -30 gpurun_out/pgemm_tune_v.txt; exit 1; }
cat gpurun_out/pgemm_tune_v.txt
