"""One GEMM shape, pgemm (given config / splits) and the library path back to back -- a target for
`rocprofv3 --pmc ...` counter passes (tools/gpu_pgemm_pmc.sh)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_llm_scheduler_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=2048)
ap.add_argument("--n", type=int, default=8192)
ap.add_argument("--k", type=int, default=8192)
ap.add_argument("--epi", type=int, default=0)
ap.add_argument("--cfg", type=int, default=0)
ap.add_argument("--splits", type=int, default=1)
ap.add_argument("--group-m", type=int, default=4)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--kernel", default="pgemm", choices=["pgemm", "pgemm4"])
a = ap.parse_args()
rows = 2 * a.n if a.epi == ops.EPI_SWIGLU else a.n
w = torch.empty(rows, a.k, dtype=torch.bfloat16, device="cuda").uniform_(-1, 1)
x = torch.empty(a.m, a.k, dtype=torch.bfloat16, device="cuda").uniform_(-1, 1)
for _ in range(a.reps):
    (ops.pgemm4 if a.kernel == "pgemm4" else ops.pgemm)(x, w, a.epi, cfg=a.cfg, splits=a.splits, group_m=a.group_m)
    torch.nn.functional.linear(x, w)
torch.cuda.synchronize()
print("done", vars(a))
