#!/usr/bin/env python3
"""Per-launch time of the fp8 prefill GEMMs with per-token vs MX activations (70B TP = 1 shapes, routed plans), and of
the two activation quantizers: where does an MX prefill spend more?

    python tools/experiments/mx_pgemm_bench.py [--m 245 2048 8192]
"""

import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from k8s_llm_scheduler_amd import ops  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        fn()
    t1.record()
    t1.synchronize()
    return t0.elapsed_time(t1) * 1000 / reps


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[245, 2048, 8192])
    a = ap.parse_args()
    H, I = 8192, 28672
    shapes = {"o_proj": (H, H, ops.EPI_BF16), "gate_up": (I, H, ops.EPI_SWIGLU), "down": (H, I, ops.EPI_BF16)}
    for M in a.m:
        for name, (N, K, epi) in shapes.items():
            rows = 2 * N if epi == ops.EPI_SWIGLU else N
            w = ops.quantize_fp8((torch.rand(rows, K, device="cuda") * 0.1 - 0.05).to(torch.bfloat16))
            x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
            pt = ops.quantize_act_fp8(x)
            mx = ops.quantize_act_mx(x)
            route = ops.gemm_route(M, N, K, epi, True)
            q_pt = timed(lambda: ops.quantize_act_fp8(x))
            q_mx = timed(lambda: ops.quantize_act_mx(x))
            g_pt = timed(lambda: ops._gemm(x, w, epi, act=pt))
            if epi == ops.EPI_SWIGLU:
                g_mx = timed(lambda: ops._gemm(x, w, epi, act=pt, mx_out=True))
                tag = "bf16 out / MX out"
            else:
                g_mx = timed(lambda: ops._gemm_mx(mx, w, epi))
                tag = "per-token / MX act"
            print(f"M {M:5d} {name:8s} {str(route):24s} gemm {tag}: {g_pt:8.1f} / {g_mx:8.1f} us   "
                  f"quantize per-token {q_pt:6.1f} us, MX {q_mx:6.1f} us", flush=True)
            if route[0] == "pgemm":   # every tile configuration at the routed split, per-token vs MX
                sp, gm = route[1][1], route[1][2]
                row = []
                for c in range(len(ops.pgemm_configs())):
                    if epi == ops.EPI_SWIGLU:
                        tp = timed(lambda: ops.pgemm(x, w, epi, cfg=c, splits=sp, group_m=gm, act=pt))
                        tm = timed(lambda: ops.pgemm(x, w, epi, cfg=c, splits=sp, group_m=gm, act=pt, mx_out=True))
                    else:
                        tp = timed(lambda: ops.pgemm(x, w, epi, cfg=c, splits=sp, group_m=gm, act=pt))
                        tm = timed(lambda: ops.pgemm(mx, w, epi, cfg=c, splits=sp, group_m=gm))
                    row.append(f"cfg{c} {tp:7.1f}/{tm:7.1f}")
                print("      pgemm per cfg (per-token / MX):", "  ".join(row), flush=True)
            del w, x, pt, mx
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
