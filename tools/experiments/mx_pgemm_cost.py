#!/usr/bin/env python3
"""Where pgemm's MX mode loses time against its per-token mode, per tile configuration (70B TP = 1 O / down at 2048
and 8192 rows).  profiles/mx_pgemm_cost_r5.txt was measured with a temporary K8S_PGEMM_MXDBG switch in pgemm.hip
(1: scale DMA not issued, 2: scale reads / packing skipped, 3: neither -- wrong results, timing only), since removed;
the MXDBG=0 rows are the kernel as built.

    python tools/experiments/mx_pgemm_cost.py
"""

import os
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
    dbg = os.environ.get("K8S_PGEMM_MXDBG", "0")
    H, I = 8192, 28672
    for M in (2048, 8192):
        for name, (N, K) in {"o_proj": (H, H), "down": (H, I)}.items():
            w = ops.quantize_fp8((torch.rand(N, K, device="cuda") * 0.1 - 0.05).to(torch.bfloat16))
            x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
            pt, mx = ops.quantize_act_fp8(x), ops.quantize_act_mx(x)
            row = []
            for c in (0, 1, 2, 3):
                tp = timed(lambda: ops.pgemm(x, w, ops.EPI_BF16, cfg=c, splits=1, group_m=4, act=pt))
                tm = timed(lambda: ops.pgemm(mx, w, ops.EPI_BF16, cfg=c, splits=1, group_m=4))
                row.append(f"cfg{c} {tp:7.1f}/{tm:7.1f} ({tm / tp:4.2f}x)")
            print(f"MXDBG={dbg} M {M:5d} {name:7s} per-token/MX: " + "  ".join(row), flush=True)
            del w, x, pt, mx
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
