# PMC counters of mgemm vs the library GEMM on one prefill shape (one counter pass per rocprofv3 run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPO="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
ARGS="${PROBE_ARGS:---m 256 --n 10240 --k 8192}"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$REPO/gpurun_out/pmc/counters.txt" 2>&1 || true
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --stats -d "$REPO/gpurun_out/pmc/p$i" -o run --output-format csv -- python3 "$REPO/tools/gemm_pmc_probe.py" $ARGS > "$REPO/gpurun_out/pmc/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$REPO/gpurun_out/pmc/p$i.log"; }
done
cd "$REPO"
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt 2>&1; cat gpurun_out/pmc/summary.txt
