"""Fused RMS prologue / residual epilogue vs the separate norm / add kernels, per projection (graph-timed)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_scheduler_amd import ops  # noqa: E402
from mgemm_tune import time_graph  # noqa: E402

H, EPS = 8192, 1e-5
print(f"{'tp':>3} {'M':>4} {'op':10} {'separate us':>12} {'fused us':>9}")
for tp in (8, 1):
    for M in (16, 64):
        for name, N, K, epi in (("qkv", 10240 // tp, H, 0), ("gate_up", 28672 // tp, H, 2)):
            rows = 2 * N if epi == 2 else N
            Ws = [torch.empty(rows, K, dtype=torch.bfloat16, device="cuda").uniform_(-.05, .05)
                  for _ in range(max(1, 600 * 2**20 // (rows * K * 2)))]
            r = torch.randn(M, K, device="cuda").bfloat16()
            ones = torch.ones(K, device="cuda", dtype=torch.bfloat16)
            sep = time_graph(lambda i: ops.mgemm(ops.rmsnorm(r, ones, EPS), Ws[i], epi), len(Ws))
            fus = time_graph(lambda i: ops.mgemm(r, Ws[i], epi, rms_eps=EPS), len(Ws))
            print(f"{tp:>3} {M:>4} {name:10} {sep:12.2f} {fus:9.2f}", flush=True)
        for name, N, K in (("o_proj", H, 8192 // tp), ("down", H, 28672 // tp)):
            Ws = [torch.empty(N, K, dtype=torch.bfloat16, device="cuda").uniform_(-.05, .05)
                  for _ in range(max(1, 600 * 2**20 // (N * K * 2)))]
            x = torch.randn(M, K, device="cuda").bfloat16()
            res = torch.randn(M, N, device="cuda").bfloat16()
            sep = time_graph(lambda i: res.add_(ops.mgemm(x, Ws[i], 0)), len(Ws))
            fus = time_graph(lambda i: ops.mgemm(x, Ws[i], 0, res=res, out=res), len(Ws))
            print(f"{tp:>3} {M:>4} {name:10} {sep:12.2f} {fus:9.2f}", flush=True)
