#!/usr/bin/env python3
"""Probe the fused RMSNorm prologue of the decode GEMV: norm-GEMV vs plain GEMV vs (rmsnorm kernel +
plain GEMV) over N (workgroup count) at K = 8192, hipGraph-replayed.

    python tools/gemv_probe.py [--M 1]
"""

import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402
from kbench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=1)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    M, K, dev, bf = a.M, 8192, "cuda", torch.bfloat16
    x = torch.randn(M, K, device=dev).to(bf)
    res = torch.randn(M, K, device=dev).to(bf)
    ro = torch.empty_like(res)
    nw = torch.ones(K, device=dev, dtype=bf)
    print(f"# M={M} K={K}: us per call")
    print(f"{'N':>6} {'norm-gemv':>10} {'gemv':>8} {'rmsnorm+gemv':>13} {'norm-gemv, no res':>18} {'folded':>8}")
    for N in (8, 64, 256, 1280, 3584, 10240):
        w = (torch.randn(N, K, device=dev) * 0.02).to(bf)
        t_norm = timeit(lambda: ops.linear_norm(x, w, nw, 1e-5, res, ro), a.iters)
        t_plain = timeit(lambda: ops.linear(x, w), a.iters)

        def two():
            h = ops.rmsnorm(x, nw, 1e-5, residual=ro)
            return ops.linear(h, w)

        t_two = timeit(two, a.iters)
        t_nores = timeit(lambda: ops.linear_norm(x, w, nw, 1e-5, None, None), a.iters)
        t_fold = timeit(lambda: ops.linear_norm(x, w, None, 1e-5, res, ro), a.iters)
        print(f"{N:6d} {t_norm:10.2f} {t_plain:8.2f} {t_two:13.2f} {t_nores:18.2f} {t_fold:8.2f}")


if __name__ == "__main__":
    main()
