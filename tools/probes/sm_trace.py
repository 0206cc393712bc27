#!/usr/bin/env python3
"""Kernel-trace companion of tools/sgemv_probe.py: the 70B TP=1 projection shapes at M rows (env M, default 8),
ITERS launches each, in a fixed order, cold weights (a scrub kernel between launches).  Run under
rocprofv3 --kernel-trace; tools/probes/sm_trace_parse.py maps the trace back to the shapes."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from k8s_llm_scheduler_amd import ops  # noqa: E402

SHAPES = [("qkv", 10240, 8192, ops.EPI_BF16, True, False), ("o", 8192, 8192, ops.EPI_BF16, False, True),
          ("gate_up", 28672, 8192, ops.EPI_SWIGLU, True, False), ("down", 8192, 28672, ops.EPI_BF16, False, True)]
M = int(os.environ.get("M", "8"))
ITERS = int(os.environ.get("ITERS", "5"))
scrub = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
for fp8 in (False, True):
    for name, N, K, epi, norm, res in SHAPES:
        rows = 2 * N if epi == ops.EPI_SWIGLU else N
        w = (torch.rand(rows, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        if fp8:
            w = ops.quantize_fp8(w)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        r = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda") if res else None
        torch.cuda.synchronize()
        print(f"SHAPE {'fp8' if fp8 else 'bf16'} {name} {rows * K * (1 if fp8 else 2)}", flush=True)
        for _ in range(ITERS):
            scrub.add_(1)
            ops._sgemv(x, w, epi, res=r, rms_eps=1e-5 if norm else None, out=r)
        torch.cuda.synchronize()
        del w
