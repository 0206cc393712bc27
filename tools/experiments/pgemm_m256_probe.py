#!/usr/bin/env python3
"""The four 70B TP=1 projections at the default prefill chunk (245 rows) on their routed hand-written GEMMs, for PMC
passes (rocprofv3 --pmc): QKV and gate/up with the RMS prologue, O and down with the residual epilogue, each launched
REPS times with the weights cycled over two copies (cold, as in the prefill loop).

    rocprofv3 --pmc <counters> -d <dir> -o run -- python3 tools/experiments/pgemm_m256_probe.py [--rows 245]
"""

import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from k8s_llm_scheduler_amd import ops  # noqa: E402

H, I, NQKV = 8192, 28672, (64 + 16) * 128


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=245)
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    M, eps = a.rows, 1e-5
    dev = torch.device("cuda")
    r = (torch.randn(M, H, device=dev) * 2).to(torch.bfloat16)
    x_o = torch.randn(M, H, device=dev).to(torch.bfloat16)
    h = torch.randn(M, I, device=dev).to(torch.bfloat16)

    def w(rows, k):
        return [(torch.rand(rows, k, device=dev) * 0.1 - 0.05).to(torch.bfloat16) for _ in range(2)]

    shapes = {"qkv": w(NQKV, H), "o": w(H, H), "gate_up": w(2 * I, H), "down": w(H, I)}
    for name, ws in shapes.items():
        for i in range(a.reps):
            wt = ws[i % 2]
            if name == "qkv":
                ops.linear_rms(r, wt, eps)
            elif name == "gate_up":
                ops.linear_rms(r, wt, eps, ops.EPI_SWIGLU)
            elif name == "o":
                ops.linear_residual(x_o, wt, r.clone())
            else:
                ops.linear_residual(h, wt, r.clone())
        torch.cuda.synchronize()
        print(name, ops.gemm_route(M, ws[0].shape[0] // (2 if name == "gate_up" else 1), ws[0].shape[1],
                                   ops.EPI_SWIGLU if name == "gate_up" else ops.EPI_BF16, False), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
