#!/usr/bin/env python3
"""One small-batch projection shape through ops._sgemv, ITERS times (for rocprofv3 --pmc passes).
Env: SHAPE=o|qkv|gate_up|down, M (rows), FP8=0|1, ITERS.  K8S_SGEMV_MFMA_MIN_M picks the kernel form."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from k8s_llm_scheduler_amd import ops  # noqa: E402

SHAPES = {"qkv": (10240, 8192, ops.EPI_BF16), "o": (8192, 8192, ops.EPI_BF16),
          "gate_up": (28672, 8192, ops.EPI_SWIGLU), "down": (8192, 28672, ops.EPI_BF16)}
N, K, epi = SHAPES[os.environ.get("SHAPE", "o")]
M = int(os.environ.get("M", "8"))
rows = 2 * N if epi == ops.EPI_SWIGLU else N
w = (torch.rand(rows, K, device="cuda") * 2 - 1).to(torch.bfloat16)
if os.environ.get("FP8", "0") == "1":
    w = ops.quantize_fp8(w)
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
scrub = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
for _ in range(int(os.environ.get("ITERS", "10"))):
    scrub.add_(1)
    ops._sgemv(x, w, epi)
torch.cuda.synchronize()
print("done", os.environ.get("SHAPE", "o"), M, flush=True)
