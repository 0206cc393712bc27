#!/usr/bin/env python3
"""mgemm with and without the RMS prologue at batched-decode row counts (70B TP=1 QKV and gate/up), every tile
configuration and grid: does the tuned plan (chosen without the prologue) stay the best one with it?"""
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from k8s_llm_scheduler_amd import ops  # noqa: E402

dev = "cuda"
scrub = torch.empty(512 << 20, dtype=torch.uint8, device=dev)


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        scrub.add_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


for name, N, K, epi in (("qkv", 10240, 8192, ops.EPI_BF16), ("gate_up", 28672, 8192, ops.EPI_SWIGLU)):
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = (torch.rand(rows, K, device=dev) * 2 - 1).to(torch.bfloat16)
    for M in (32, 64):
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        plan = ops.mgemm_plan(M, N, K, epi, False)
        res = []
        for cfg in range(len(ops.mgemm_configs())):
            for grid in (1, 2, 4):
                if not ops.mgemm_valid(cfg, M, N, K, epi, False, grid):
                    continue
                try:
                    t0 = timed(lambda: ops.mgemm(x, w, epi, cfg=cfg, grid=grid))
                    t1 = timed(lambda: ops.mgemm(x, w, epi, cfg=cfg, grid=grid, rms_eps=1e-5))
                except Exception as e:  # noqa: BLE001
                    continue
                res.append((t1, t0, cfg, grid))
        res.sort()
        tp = [r for r in res if (r[2], r[3]) == tuple(plan)]
        print(f"{name} M={M}: plan {plan} -> rms {tp[0][0] if tp else float('nan'):.1f} us / plain "
              f"{tp[0][1] if tp else float('nan'):.1f}; best rms {res[0][0]:.1f} (cfg {res[0][2]}, grid {res[0][3]}, "
              f"plain {res[0][1]:.1f}); best plain {min(r[1] for r in res):.1f}", flush=True)
    del w
