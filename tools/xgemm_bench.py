#!/usr/bin/env python3
"""xgemm.hip vs the routed mgemm plan at the batched-decode projections (cold weights: every launch reads a
different copy, > 1 GiB in rotation, so the weights come from HBM as in the decode loop).

    python tools/xgemm_bench.py [--M 64] [--tp 1]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    e0.record()
    for i in range(reps):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[32, 64])
    ap.add_argument("--tp", type=int, default=1)
    a = ap.parse_args()
    H, I = 8192, 28672 // a.tp
    shapes = [("qkv+rms", 10240 // a.tp, H, ops.EPI_BF16, "rms"), ("o+res", H, H // a.tp, ops.EPI_BF16, "res"),
              ("gate_up+swiglu+rms", I, H, ops.EPI_SWIGLU, "rms"), ("down+res", H, I, ops.EPI_BF16, "res")]
    for M in a.M:
        for name, N, K, epi, kind in shapes:
            rows = 2 * N if epi == ops.EPI_SWIGLU else N
            ncopy = max(2, int((1.2 * 2 ** 30) // (rows * K * 2)) + 1)
            ws = [torch.randn(rows, K, device="cuda").mul_(0.02).to(torch.bfloat16) for _ in range(ncopy)]
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            res = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            kw = {"rms_eps": 1e-5} if kind == "rms" else {"res": res}
            reps = 4 * ncopy
            tx = timed(lambda i: ops.xgemm(x, ws[i % ncopy], epi, **kw), reps)
            tm = timed(lambda i: ops.mgemm(x, ws[i % ncopy], epi, **kw), reps)
            gb = rows * K * 2 / 1e9
            print(f"M={M:3d} {name:20s} N={N:6d} K={K:6d}  xgemm {tx:8.1f} us ({gb / tx * 1e3:5.2f} TB/s)   "
                  f"mgemm {tm:8.1f} us ({gb / tm * 1e3:5.2f} TB/s)", flush=True)
            del ws


if __name__ == "__main__":
    main()
