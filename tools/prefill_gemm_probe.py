#!/usr/bin/env python3
"""Prefill GEMMs (M = prompt tokens) of Llama-3.3-70B: hipBLASLt's default solution vs the one PyTorch
TunableOp selects, per TP degree, plus the weight-streaming floor (bytes / 6.3 TB/s).

    python tools/prefill_gemm_probe.py [--M 256,512] [--tp 1,8] [--out table.csv]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
from kbench import timeit  # noqa: E402
from tune_gemms import shapes  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="256,512")
    ap.add_argument("--tp", default="1,8")
    ap.add_argument("--out", default="/tmp/prefill_tunableop.csv")
    a = ap.parse_args()
    t = torch.cuda.tunable
    t.set_filename(a.out)
    t.set_max_tuning_duration(60)
    names = ("qkv", "o_proj", "gate_up", "down", "lm_head")
    print(f"{'tp':>3} {'M':>5} {'gemm':8s} {'default us':>11} {'tuned us':>9} {'floor us':>9}")
    for tp in (int(x) for x in a.tp.split(",")):
        for name, (N, K) in zip(names, shapes(tp)):
            if name == "lm_head":
                continue
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            for M in (int(x) for x in a.M.split(",")):
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                f = lambda: torch.nn.functional.linear(x, w)
                t.enable(False)
                d = timeit(f, 30)
                t.enable(True)
                t.tuning_enable(True)
                f()
                torch.cuda.synchronize()
                t.tuning_enable(False)
                u = timeit(f, 30)
                t.enable(False)
                print(f"{tp:3d} {M:5d} {name:8s} {d:11.1f} {u:9.1f} {N * K * 2 / 6.3e6:9.1f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
