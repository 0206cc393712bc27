set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_prof.sh tp8sim_b64 "--simulate-tp 8 --batch 64" > /dev/null && \
bash tools/gpu_prof.sh tp1_b64 "--batch 64" > /dev/null && \
bash tools/gpu_prof.sh tp1_single "" > /dev/null
for t in tp8sim_b64 tp1_b64 tp1_single; do echo "== $t"; head -28 gpurun_out/rocprof_70b_${t}_kernels.txt; done
