#!/usr/bin/env python3
"""One-row decode projections: the GEMV (gemv.hip, with its residual-add + norm prologue) against the MFMA sgemv
form (norm prologue / residual epilogue) on the 70B TP=1 and TP=8 shapes, M = 1 and 2.  Run under rocprofv3
--kernel-trace with K8S_SGEMV_MFMA_MIN_M=1; tools/probes/sm_trace_parse.py style output via m1_parse below."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from k8s_llm_scheduler_amd import ops  # noqa: E402

ITERS = int(os.environ.get("ITERS", "5"))
SHAPES = [  # tp, name, N, K, epi, form ("rms": residual-add + norm prologue / norm; "res": plain / residual epilogue)
    (1, "qkv", 10240, 8192, ops.EPI_BF16, "rms"), (1, "o", 8192, 8192, ops.EPI_BF16, "res"),
    (1, "gate_up", 28672, 8192, ops.EPI_SWIGLU, "rms"), (1, "down", 8192, 28672, ops.EPI_BF16, "res"),
    (8, "qkv", 1280, 8192, ops.EPI_BF16, "rms"), (8, "o", 8192, 1024, ops.EPI_BF16, "res"),
    (8, "gate_up", 3584, 8192, ops.EPI_SWIGLU, "rms"), (8, "down", 8192, 3584, ops.EPI_BF16, "res")]
scrub = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
nat = ops.native()
for tp, name, N, K, epi, form in SHAPES:
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = (torch.rand(rows, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    for M in (1, 2):
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        ra, rb = torch.zeros(M, K, dtype=torch.bfloat16, device="cuda"), torch.zeros(M, K, dtype=torch.bfloat16,
                                                                                     device="cuda")
        rN = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
        torch.cuda.synchronize()
        print(f"SHAPE tp{tp}-{name}-M{M} {rows * K * 2}", flush=True)
        for _ in range(ITERS):
            scrub.add_(1)
            if form == "rms":
                ops._gemv(x, w, epi, torch.bfloat16, eps=1e-5, res_in=ra, res_out=rb, folded=True)
            else:
                ops._gemv(x, w, epi, torch.bfloat16)
        for _ in range(ITERS):
            scrub.add_(1)
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            ws = nat.sgemv_workspace(M, N, K, epi)
            part = torch.empty(max(ws, 1), dtype=torch.float32, device="cuda")
            if form == "rms":
                nat.sgemv(out.data_ptr(), part.data_ptr(), x.data_ptr(), w.data_ptr(), 0, 0, M, N, K, epi, 1, 1e-5, -1)
            else:
                nat.sgemv(rN.data_ptr(), part.data_ptr(), x.data_ptr(), w.data_ptr(), 0, rN.data_ptr(), M, N, K, epi,
                          0, 0.0, -1)
        torch.cuda.synchronize()
    del w
