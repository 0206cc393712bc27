# Full mgemm tuning sweep (bf16 at TP 1/2/4/8, fp8 at TP 4 and 1) -> engine/assets/mgemm_gfx950.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
rm -f k8s_llm_scheduler_amd/engine/assets/mgemm_gfx950.json
timeout -k 10 900 python -u tools/mgemm_tune.py --tp 8 1 4 2 --all-buckets --write --json-out gpurun_out/mgemm_full_bf16.json > gpurun_out/mgemm_full_bf16.txt 2>&1 || { tail -20 gpurun_out/mgemm_full_bf16.txt; exit 1; }
tail -3 gpurun_out/mgemm_full_bf16.txt
timeout -k 10 600 python -u tools/mgemm_tune.py --tp 4 1 --fp8 --m 16 32 48 64 96 128 192 256 320 384 448 512 640 768 896 1024 2048 --write --json-out gpurun_out/mgemm_full_fp8.json > gpurun_out/mgemm_full_fp8.txt 2>&1 || { tail -20 gpurun_out/mgemm_full_fp8.txt; exit 1; }
tail -3 gpurun_out/mgemm_full_fp8.txt
mkdir -p gpurun_out/assets && cp k8s_llm_scheduler_amd/engine/assets/mgemm_gfx950.json gpurun_out/assets/
