#!/usr/bin/env python3
"""Where does a decision's prefill time go?  70B TP=1, graphs captured, prefix cache on: prompts of 464 tokens
sharing a 219-token prefix (as the bench's decisions do), 2 output tokens each.  Prints the engine's host timeline
of the prefill (K8S_ENGINE_TRACE points) and the GPU-event prefill time per decision."""
import os
import sys
import time
from pathlib import Path

os.environ["K8S_ENGINE_TRACE"] = "1"
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine  # noqa: E402

eng = build_engine("llama-3.3-70b", max_batch=1, max_model_len=2048, num_blocks=600, capture=False, decode_chunk=8)
eng.capture_graphs([1])
torch.cuda.synchronize()
prefix = [1000 + (i * 7919) % 120000 for i in range(219)]
for it in range(5):
    suffix = [2000 + ((it + 1) * 104729 + i * 31) % 120000 for i in range(245)]
    eng.recovery_trace.clear()
    pt0 = eng.stats["prefill_time"]
    t0 = time.perf_counter()
    out = eng.generate([prefix + suffix], SamplingParams(max_tokens=2, temperature=0.3, seed=it, ignore_eos=True))[0]
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    tr = list(eng.recovery_trace)
    pf = [(t, m) for t, m in tr if m.startswith("prefill")]
    steps = " | ".join(f"{m.split(': ', 1)[1]} +{(t - pf[0][0]) * 1e3:.1f}" for t, m in pf[1:]) if pf else "-"
    print(f"decision {it}: wall {wall:.1f} ms, GPU prefill {1e3 * (eng.stats['prefill_time'] - pt0):.1f} ms, "
          f"prefill tokens {eng.stats['prefill_tokens']}, cached {eng.stats['cached_tokens']}; host: {steps}", flush=True)
