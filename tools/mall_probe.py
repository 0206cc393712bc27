#!/usr/bin/env python3
"""Probe: decode GEMV time with its weights cold (HBM) vs resident in the 256 MiB Infinity Cache.

    python tools/mall_probe.py

Each case is hipGraph-replayed as [flush, gemv] x N and [flush] x N; the difference is the GEMV time
after a 512 MiB streaming read (cold), versus [gemv] x N back to back (weights re-read: warm)."""

import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tools"))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402
from kbench import timeit  # noqa: E402


def main():
    dev, bf = "cuda", torch.bfloat16
    flush_buf = torch.ones(256 * 1024 * 1024, dtype=bf, device=dev)  # 512 MiB
    sink = torch.empty(1, dtype=torch.float32, device=dev)
    flush = lambda: flush_buf.add_(0)   # reads and writes 512 MiB
    print("# us per GEMV: warm (back to back) vs cold (after a 512 MiB read)")
    for name, N, K in (("o_proj tp8", 8192, 1024), ("down tp8", 8192, 3584), ("qkv tp8", 1280, 8192),
                       ("gate_up tp8 (rows)", 7168, 8192)):
        x = torch.randn(1, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) * 0.02).to(bf)
        f = lambda: ops.linear(x, w)
        warm = timeit(f, 100)
        both = timeit(lambda: (flush(), f()), 50)
        only = timeit(flush, 50)
        print(f"{name:20s} {N * K * 2 / 1e6:7.1f} MB  warm {warm:7.2f}  cold {both - only:7.2f}")


if __name__ == "__main__":
    main()
