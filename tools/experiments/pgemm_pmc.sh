# PMC passes over tools/experiments/pgemm_m256_probe.py (the prefill projections at ROWS rows, default 245; ROWS=64: the
# batched-decode mgemm shapes), each pass in its own
# rocprofv3 run (no trace domains beside the counters), summarised per kernel by tools/pmc_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPO="$GRAFT_REPO_ROOT"
O="$REPO/gpurun_out/pmc${ROWS:-}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$O/p$i" -o run -- python3 "$REPO/tools/experiments/pgemm_m256_probe.py" --rows ${ROWS:-245} > "$O/p$i.log" 2>&1 || { tail -5 "$O/p$i.log"; exit 1; }
done
python3 "$REPO/tools/pmc_summary.py" "$O" > "$O/summary.txt" && cat "$O/summary.txt"
rm -rf "$O/p1" "$O/p2"
