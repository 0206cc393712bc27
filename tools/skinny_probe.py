#!/usr/bin/env python3
"""Graph-timed skinny GEMM vs hipBLASLt at one shape (diagnostics: K8S_SKINNY_DIAG)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402
from kbench import timeit  # noqa: E402

ops.SKINNY_ENABLED = True
M, N, K = (int(v) for v in sys.argv[1:4])
epi = int(sys.argv[4]) if len(sys.argv) > 4 else 0
x = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(N * (2 if epi == 2 else 1), K, device="cuda") * 0.02).bfloat16()
fn = (lambda: ops.linear_swiglu(x, w)) if epi == 2 else (lambda: ops.linear(x, w))
us = timeit(fn, 100)
print(f"M={M} N={N} K={K} epi={epi}: {us:.2f} us  {w.numel() * 2 / us / 1e6:.2f} TB/s")
