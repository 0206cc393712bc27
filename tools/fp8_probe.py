#!/usr/bin/env python3
"""Probe: prefill projection GEMMs at Llama-3.3-70B TP=4 shapes -- bf16 hipBLASLt vs fp8 paths.

    python tools/fp8_probe.py [--tokens 256]

Rows: bf16 F.linear; fp8 weights dequantized to bf16 then F.linear (the previous prefill path);
ops.linear on an Fp8Weight (per-token activation quantization kernel + row-wise scaled fp8 GEMM).
"""

import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=256)
    ap.add_argument("--tp", type=int, default=4)
    a = ap.parse_args()
    T, tp = a.tokens, a.tp
    shapes = {"qkv": (10240 // tp, 8192), "o": (8192, 8192 // tp), "gate_up": (57344 // tp, 8192),
              "down": (8192, 28672 // tp)}
    print(f"# T={T} tp={tp}")
    for name, (N, K) in shapes.items():
        x = (torch.randn(T, K, device="cuda") * 0.5).bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        fw = ops.quantize_fp8(w)
        flops = 2 * T * N * K
        us = timeit(lambda: torch.nn.functional.linear(x, w))
        print(f"{name:8s} N={N:6d} K={K:5d} bf16 F.linear          {us:9.1f} us {flops / us / 1e6:7.1f} TF/s")
        us = timeit(lambda: torch.nn.functional.linear(x, fw.dequant()))
        print(f"{name:8s} N={N:6d} K={K:5d} fp8 dequant+F.linear    {us:9.1f} us {flops / us / 1e6:7.1f} TF/s")
        y = ops.linear(x, fw)
        ref = torch.nn.functional.linear(x.float(), fw.dequant(torch.float32))
        err = float((y.float() - ref).abs().max() / ref.abs().max())
        us = timeit(lambda: ops.linear(x, fw))
        print(f"{name:8s} N={N:6d} K={K:5d} fp8 act-quant+scaled GEMM {us:7.1f} us {flops / us / 1e6:7.1f} TF/s"
              f"  rel.err {err:.3g}")
        xq, sx = ops.quantize_act_fp8(x)
        us = timeit(lambda: ops.quantize_act_fp8(x))
        print(f"{name:8s} {'':20s} of which act-quant       {us:9.1f} us")


if __name__ == "__main__":
    main()
