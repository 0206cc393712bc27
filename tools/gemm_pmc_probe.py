"""One GEMM shape, mgemm (given config) and the library path back to back -- a target for
`rocprofv3 --pmc ...` counter passes (tools/gpu_pgemm_pmc.sh)."""
import argparse
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from k8s_llm_scheduler_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=256)
ap.add_argument("--n", type=int, default=10240)
ap.add_argument("--k", type=int, default=8192)
ap.add_argument("--epi", type=int, default=0)
ap.add_argument("--cfg", type=int, nargs="*", default=None)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
rows = 2 * a.n if a.epi == ops.EPI_SWIGLU else a.n
w = torch.empty(rows, a.k, dtype=torch.bfloat16, device="cuda").uniform_(-0.05, 0.05)
x = torch.empty(a.m, a.k, dtype=torch.bfloat16, device="cuda").uniform_(-1, 1)
plan = ops.mgemm_plan(a.m, a.n, a.k, a.epi, False)
cfgs = a.cfg if a.cfg else [plan[0]]
for _ in range(a.reps):
    for c in cfgs:
        ops.mgemm(x, w, a.epi, cfg=c, grid=plan[1] if c == plan[0] else 1)
    y = torch.nn.functional.linear(x, w)
torch.cuda.synchronize()
print("plan", plan, "cfgs", cfgs)
