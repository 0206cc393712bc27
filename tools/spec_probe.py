#!/usr/bin/env python3
"""Speculative decoding cost and gain on one GPU (engine.speculative_tokens).

Two workloads, each decoded plainly (captured one-token decode graphs) and with prompt-lookup drafts:
* ``random``: the random-init model as bench.py runs it -- drafts almost never exist, so this measures what
  speculation costs when it cannot help;
* ``cycle``: the same model with its logits forced to a 5-token cycle (tests/test_speculative_cpu.CycleModel), so
  nearly every draft is accepted -- the upper bound of the gain, reached when the answer copies earlier text.

    python tools/spec_probe.py --preset llama-3.3-70b --tokens 64 --spec 4
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="llama-3.3-70b")
    ap.add_argument("--tokens", type=int, default=64)
    ap.add_argument("--spec", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from k8s_llm_scheduler_amd.engine import SamplingParams, _load_gemm_table
    from k8s_llm_scheduler_amd.engine.engine import LLMEngine
    from k8s_llm_scheduler_amd.engine.tokenizer import Tokenizer
    from k8s_llm_scheduler_amd.models.config import PRESETS
    from k8s_llm_scheduler_amd.models.llama import LlamaModel
    from test_speculative_cpu import CycleModel

    _load_gemm_table()
    prompt = [(37 * i) % 5000 + 200 for i in range(400)]
    params = SamplingParams(max_tokens=a.tokens, temperature=0.3, seed=3, ignore_eos=True)
    out = []
    for workload, cls in (("random", LlamaModel), ("cycle", CycleModel)):
        m = cls(PRESETS[a.preset], device="cuda", seed=1, max_model_len=2048)
        for spec in (0, a.spec):
            eng = LLMEngine(m, Tokenizer(None, model_vocab=m.cfg.vocab), max_batch=4, num_blocks=400,
                            max_model_len=2048, seed=1, speculative_tokens=spec, prefix_caching=False)
            eng.capture_graphs([1])
            eng.generate([prompt], params)                       # warm-up
            best, toks = 1e9, None
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                o = eng.generate([prompt], params)[0]
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
                toks = o.token_ids
            st = eng.stats
            row = {"probe": "speculative", "preset": a.preset, "workload": workload, "spec_tokens": spec,
                   "ms_per_answer": round(best * 1e3, 1), "tokens": len(toks),
                   "verify_forwards": st["spec_steps"], "verify_graph_replays": st["spec_graph_replays"], "drafted": st["spec_drafted"], "accepted": st["spec_accepted"]}
            out.append((workload, spec, toks))
            print(json.dumps(row), flush=True)
            del eng
        del m
        torch.cuda.empty_cache()
    same = {w: [t for w2, _, t in out if w2 == w] for w in ("random", "cycle")}
    print(json.dumps({"answers_equal": {w: v[0] == v[1] for w, v in same.items()}}))


if __name__ == "__main__":
    main()
