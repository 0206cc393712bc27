# Speculative decoding: cost when nothing is drafted (random weights) and gain when drafts hit (cycle workload).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/spec2; mkdir -p $O
timeout -k 10 400 python -u tools/spec_probe.py --preset llama-3-8b > $O/probe_8b.jsonl 2> $O/probe_8b.err || { tail -20 $O/probe_8b.err; exit 1; }
cat $O/probe_8b.jsonl
timeout -k 10 600 python -u tools/spec_probe.py --preset llama-3.3-70b --reps 2 > $O/probe_70b.jsonl 2> $O/probe_70b.err || { tail -20 $O/probe_70b.err; exit 1; }
cat $O/probe_70b.jsonl
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --speculative 4 > $O/tp1_spec4.json 2> $O/tp1_spec4.err || { tail -20 $O/tp1_spec4.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench tp1 spec4', d['value'], d['decode_ms_per_step'], d['speculative'])" $O/tp1_spec4.json
