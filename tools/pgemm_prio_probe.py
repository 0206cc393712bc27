#!/usr/bin/env python3
"""pgemm.hip main-loop wave priority A/B (ops.native().pgemm_set_prio): 0 = s_setprio 1 around every MFMA section
(default), 1 = waves 4-7 at priority 1 for the whole loop, 2 = no s_setprio.  Each shape runs its tuned plan with cold
weights (cycled over > 600 MiB), graph-timed; the outputs of the three modes must be bit-identical.

    python tools/pgemm_prio_probe.py [--m 256 2048 8192] [--tp 1] [--fp8]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_scheduler_amd import ops  # noqa: E402
from tools.mgemm_tune import COLD_BYTES, shapes, time_graph  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, nargs="+", default=[1])
    ap.add_argument("--m", type=int, nargs="+", default=[256, 2048, 8192])
    ap.add_argument("--fp8", action="store_true")
    a = ap.parse_args()
    torch.manual_seed(0)
    for tp in a.tp:
        for name, N, K, epi in shapes(tp):
            if name == "lm_head":
                continue
            rows = 2 * N if epi == ops.EPI_SWIGLU else N
            copies = max(1, -(-COLD_BYTES // (rows * K * 2)))
            Ws = [(torch.randn(rows, K, device="cuda") * 0.02).bfloat16() for _ in range(copies)]
            if a.fp8:
                Ws = [ops.quantize_fp8(w) for w in Ws]
            for M in a.m:
                (kern, cfg, sp, gm), _ = ops.pgemm_plan_for(M, N, K, epi, a.fp8)
                if kern != "pgemm":
                    continue
                x = torch.randn(M, K, device="cuda").bfloat16()
                fn = lambda i: ops.pgemm(x, Ws[i], epi, cfg=cfg, splits=sp, group_m=gm)   # noqa: E731
                outs, res = [], []
                for mode in (0, 1, 2):
                    ops.native().pgemm_set_prio(mode)
                    outs.append(fn(0))
                    res.append(time_graph(fn, copies))
                torch.cuda.synchronize()
                same = all(torch.equal(o, outs[0]) for o in outs[1:])
                print(f"tp={tp} M={M:5d} {name:8s} cfg={cfg} sp={sp} gm={gm}  prio0 {res[0]:9.1f} us  "
                      f"static {res[1]:9.1f} us ({res[0] / res[1]:.3f}x)  none {res[2]:9.1f} us ({res[0] / res[2]:.3f}x)"
                      f"  {'exact' if same else 'MISMATCH'}", flush=True)
                ops.native().pgemm_set_prio(0)
            del Ws
    return 0


if __name__ == "__main__":
    sys.exit(main())
