#!/usr/bin/env python3
"""Prefill of one 256-token chunk of Llama-3.3-70B: eager forward vs the engine's padded prefill graph,
plus the engine's whole prefill step (graph replay + first-token sampling + slot setup).

    python tools/prefill_probe.py [--simulate-tp 8] [--T 256]
"""
import argparse
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from k8s_llm_scheduler_amd.engine import build_engine  # noqa: E402
from k8s_llm_scheduler_amd.engine.engine import PREFILL_GRAPH_BUCKETS  # noqa: E402
from k8s_llm_scheduler_amd.engine.sampling import SamplingParams  # noqa: E402
from k8s_llm_scheduler_amd.parallel import TPGroup  # noqa: E402


def wall(f, n=10):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / n


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--simulate-tp", type=int, default=8)
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--preset", default="llama-3.3-70b")
    a = ap.parse_args()
    tp = TPGroup(0, a.simulate_tp, None, "none", simulate=True) if a.simulate_tp > 1 else None
    eng = build_engine(a.preset, tp=tp, max_batch=1, num_blocks=600, max_model_len=4096, capture=False)
    eng.capture_graphs([1])
    m, T, dev = eng.model, a.T, eng.device
    i32 = lambda x: torch.tensor(x, dtype=torch.int32, device=dev)
    bt = torch.arange(eng.max_blocks_per_seq, dtype=torch.int32, device=dev).view(1, -1)
    ids, pos, slots = i32([7] * T), i32(list(range(T))), i32(list(range(T)))
    cu, ctx, last = i32([0, T]), i32([T]), i32([T - 1])
    eager = wall(lambda: m.forward_prefill(ids, pos, slots, cu, ctx, bt, T, last))
    Tb = next(b for b in PREFILL_GRAPH_BUCKETS if b >= T)
    eng._fill_prefill_state([7] * T, list(range(T)), list(range(T)), T, list(range(16)), Tb)
    g, _ = eng.prefill_graphs[Tb]
    replay = wall(g.replay)
    fill = wall(lambda: eng._fill_prefill_state([7] * T, list(range(T)), list(range(T)), T, list(range(16)), Tb))
    # whole engine prefill step: T-token prompt, one new token (prefix cache off by distinct prompts)
    p = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
    k = [0]

    def step():
        k[0] += 1
        eng.generate([[1000 + k[0]] + [7] * (T - 1)], p)

    step()
    eng.stats["prefill_time"], eng.stats["prefill_graph_replays"] = 0.0, 0
    for _ in range(10):
        step()
    e2e = 1e3 * eng.stats["prefill_time"] / 10
    print(f"tp{a.simulate_tp or 1} T={T}: eager forward {eager:.2f} ms | graph replay (bucket {Tb}) {replay:.2f} ms | "
          f"input fill {fill:.3f} ms | engine prefill step {e2e:.2f} ms ({eng.stats['prefill_graph_replays']} of 10 "
          f"by graph)", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
