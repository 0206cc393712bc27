set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/prefill_probe.py --simulate-tp 8 > gpurun_out/prefill_probe.txt 2>&1 || { tail -30 gpurun_out/prefill_probe.txt; exit 1; }
timeout -k 10 300 python -u tools/prefill_probe.py --simulate-tp 0 >> gpurun_out/prefill_probe.txt 2>&1 || { tail -30 gpurun_out/prefill_probe.txt; exit 1; }
grep -v Warning gpurun_out/prefill_probe.txt | tail -4
