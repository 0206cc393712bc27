# Tune mgemm's MX modes as the fp8 decode layer runs them (TP = 1 / 4, 32-256 rows), write the table rows, then the
# fp8 batch-64 / 32 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/mgemm_tune.py --mx --tp 1 4 --m 32 64 128 256 --write --verbose > gpurun_out/mx_tune.txt 2>&1 || { tail -20 gpurun_out/mx_tune.txt; exit 1; }
cp k8s_llm_scheduler_amd/engine/assets/mgemm_gfx950.json gpurun_out/mgemm_gfx950.json
grep -v cand gpurun_out/mx_tune.txt | tail -22
bash tools/experiments/mx_ab.sh
