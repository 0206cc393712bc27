#!/usr/bin/env python3
"""Decode GEMV A/B: one row set per wave vs the row-set loop (workgroups per CU, ops.native().gemv_set_loop).

    python tools/gemv_loop_probe.py [--tp 1 4] [--loops 0 2 4 8]

Prints us and TB/s of weight bytes for the Llama-3.3-70B decode projections (M = 1, the folded-norm prologue where
the model uses it), bf16 and fp8 weights; every loop setting's output must equal the one-row-set output bit for bit.
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402
from kbench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--loops", type=int, nargs="+", default=[0, 2, 4, 8])
    a = ap.parse_args()
    torch.manual_seed(0)
    for tp in a.tp:
        for name, N, K, epi, rms in (("qkv", 10240 // tp, 8192, 0, True), ("o_proj", 8192, 8192 // tp, 0, False),
                                     ("gate_up", 28672 // tp, 8192, 2, True), ("down", 8192, 28672 // tp, 0, False),
                                     ("lm_head", 128256 // tp, 8192, 1, True)):
            x = torch.randn(1, K, device="cuda").bfloat16()
            res = torch.randn(1, K, device="cuda").bfloat16()
            w = (torch.randn(N * (2 if epi == 2 else 1), K, device="cuda") * 0.02).bfloat16()
            f8 = ops.quantize_fp8(w)
            for dt, ww, nbytes in (("bf16", w, w.numel() * 2), ("fp8", f8, f8.q.numel())):
                if rms:
                    ro = torch.empty_like(res)
                    fn = lambda ww=ww: ops.linear_norm(x, ww, None, 1e-5, res, ro, epi=epi)  # noqa: E731
                else:
                    fn = (lambda ww=ww: ops.linear_swiglu(x, ww)) if epi == 2 else (lambda ww=ww: ops.linear(x, ww))
                base = None
                for lp in a.loops:
                    ops.native().gemv_set_loop(lp)
                    y = fn()
                    torch.cuda.synchronize()
                    if base is None:
                        base = y.clone()
                    same = bool(torch.equal(y, base))
                    us = timeit(fn, a.iters)
                    print(f"tp={tp} {name:8s} {dt:5s} loop={lp} {us:8.2f} us {nbytes / us / 1e6:6.2f} TB/s"
                          f" {'exact' if same else 'MISMATCH'}", flush=True)
                ops.native().gemv_set_loop(0)


if __name__ == "__main__":
    main()
