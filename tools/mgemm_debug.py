"""Correctness sweep of mgemm.hip over shapes / configs / grids (prints max error per case)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from k8s_llm_scheduler_amd import ops  # noqa: E402


def check(M, N, K, epi, cfg, grid):
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = (torch.rand(rows, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    y = ops.mgemm(x, w, epi, cfg=cfg, grid=grid).float()
    e = x.float() @ w.float().t()
    if epi == ops.EPI_SWIGLU:
        e = torch.nn.functional.silu(e[:, :N]) * e[:, N:]
    err = (y - e).abs().max().item() / (e.abs().max().item() + 1e-6)
    bad = ((y - e).abs() > 0.02 * e.abs().max()).nonzero()
    return err, bad


for (M, N, K) in [(16, 8192, 1024), (13, 8192, 1024), (16, 8192, 8192), (13, 8192, 1024), (37, 8192, 1024), (64, 8192, 1024), (130, 8192, 1024), (16, 200, 1024), (16, 1024, 1024),
                  (16, 4096, 1024), (13, 8192, 1024)]:
    for cfg in range(len(ops.mgemm_configs())):
        if not ops.mgemm_valid(cfg, M, N, K, 0, False, 1):
            continue
        err, bad = check(M, N, K, 0, cfg, 1)
        if err > 0.02:
            rows = sorted(set(bad[:, 0].tolist()))[:8]
            cols = sorted(set(bad[:, 1].tolist()))
            print(f"M={M} N={N} K={K} cfg={cfg} {ops.mgemm_configs()[cfg]} err={err:.3f} nbad={len(bad)} rows={rows} "
                  f"cols[{len(cols)}]={cols[:8]}..{cols[-4:]}", flush=True)
print("done")
