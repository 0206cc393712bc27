"""One 70B TP=1 projection at a prefill row count through pgemm (its tuned plan) and through the library, a few
launches each, for rocprofv3 --pmc passes (tools/pmc_summary.py averages the counters per kernel).
    python tools/pgemm_pmc_probe.py [--proj gate_up] [--m 8192] [--reps 3]"""

import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402
from tools.mgemm_tune import shapes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proj", default="gate_up")
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--plan", default=None, help="kernel,cfg,splits,group_m instead of the tuned plan (e.g. pgemm4,0,1,8)")
    a = ap.parse_args()
    name, N, K, epi = next(s for s in shapes(a.tp) if s[0] == a.proj)
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = torch.empty(rows, K, dtype=torch.bfloat16, device="cuda").uniform_(-0.05, 0.05)
    x = torch.empty(a.m, K, dtype=torch.bfloat16, device="cuda").uniform_(-1, 1)
    plan, _ = ops.pgemm_plan_for(a.m, N, K, epi, False)
    if a.plan:
        k_, c_, s_, g_ = a.plan.split(",")
        plan = (k_, int(c_), int(s_), int(g_))
    kern, cfg, sp, gm = plan
    print(f"{name} M={a.m} N={N} K={K} plan {plan}", flush=True)
    for _ in range(a.reps):
        if kern == "pgemm4":
            ops.pgemm4(x, w, epi, cfg=cfg, splits=sp, group_m=gm)
        elif kern == "pgemm":
            ops.pgemm(x, w, epi, cfg=cfg, splits=sp, group_m=gm)
        else:
            ops.pgemm(x, w, epi, cfg=0, splits=1, group_m=4)
    for _ in range(a.reps):
        y = ops._lib_linear(x, w)
        if epi == ops.EPI_SWIGLU:
            y = ops.silu_mul(y)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
