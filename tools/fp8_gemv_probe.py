#!/usr/bin/env python3
"""Decode GEMV with fp8 weights vs bf16 weights at Llama-3.3-70B TP=1 / TP=4 shapes (us, TB/s of weight bytes)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402
from kbench import timeit  # noqa: E402

for tp in (1, 4):
    print(f"# tp={tp} M=1")
    for name, N, K, epi in (("qkv", 10240 // tp, 8192, 0), ("o_proj", 8192, 8192 // tp, 0),
                            ("gate_up", 28672 // tp, 8192, 2), ("down", 8192, 28672 // tp, 0)):
        x = torch.randn(1, K, device="cuda").bfloat16()
        w = (torch.randn(N * (2 if epi == 2 else 1), K, device="cuda") * 0.02).bfloat16()
        f8 = ops.quantize_fp8(w)
        for tag, ww, nbytes in (("bf16", w, w.numel() * 2), ("fp8", f8, f8.q.numel())):
            fn = (lambda ww=ww: ops.linear_swiglu(x, ww)) if epi == 2 else (lambda ww=ww: ops.linear(x, ww))
            us = timeit(fn, 100)
            print(f"{name:8s} {tag:5s} {us:8.2f} us {nbytes / us / 1e6:6.2f} TB/s")
