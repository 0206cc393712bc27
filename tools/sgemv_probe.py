#!/usr/bin/env python3
"""sgemv.hip vs mgemm.hip at small decode batches (4, 8, 16 rows) on the Llama-3.3-70B projection shapes (TP = 1 and
TP = 8, bf16 and fp8 weights), interleaved rounds in one process, cold weights (a 512 MiB scrub between calls so the
weights come from HBM as in a decode step).  Prints us per call and the weight-streaming rate.

    python tools/sgemv_probe.py [rounds]
"""
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = "cuda"
SHAPES = [  # name, N, K, epi, norm, residual
    ("tp1_qkv", 10240, 8192, ops.EPI_BF16, True, False),
    ("tp1_o", 8192, 8192, ops.EPI_BF16, False, True),
    ("tp1_gate_up", 28672, 8192, ops.EPI_SWIGLU, True, False),
    ("tp1_down", 8192, 28672, ops.EPI_BF16, False, True),
    ("tp8_qkv", 1280, 8192, ops.EPI_BF16, True, False),
    ("tp8_o", 8192, 1024, ops.EPI_BF16, False, False),
    ("tp8_gate_up", 3584, 8192, ops.EPI_SWIGLU, True, False),
    ("tp8_down", 8192, 3584, ops.EPI_BF16, False, False),
]
scrub = torch.empty(512 << 20, dtype=torch.uint8, device=dev)


def timed(fn):
    scrub.add_(1)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3


for fp8 in (False, True):
    for name, N, K, epi, norm, res in SHAPES:
        rows = 2 * N if epi == ops.EPI_SWIGLU else N
        w = (torch.rand(rows, K, device=dev) * 2 - 1).to(torch.bfloat16)
        if fp8:
            w = ops.quantize_fp8(w)
        wbytes = rows * K * (1 if fp8 else 2)
        for M in (4, 8, 16):
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            r = torch.zeros(M, N, dtype=torch.bfloat16, device=dev) if res else None
            eps = 1e-5 if norm else None
            arms = {
                "sgemv": lambda: ops._sgemv(x, w, epi, res=r, rms_eps=eps, out=r),
                "mgemm": lambda: ops.mgemm(x, w, epi, res=r, rms_eps=eps, out=r) if not (fp8 and norm)
                else ops.mgemm(ops.rmsnorm(x, ops._ones(K, x.device), 1e-5), w, epi),
            }
            t = {k: [] for k in arms}
            for fn in arms.values():
                fn()
            for _ in range(rounds):
                for k, fn in arms.items():
                    t[k].append(timed(fn))
            s = " ".join(f"{k} {statistics.median(v):7.1f} us ({wbytes / statistics.median(v) / 1e6:5.2f} TB/s)"
                         for k, v in t.items())
            print(f"{'fp8 ' if fp8 else 'bf16'} {name:12s} M={M}: {s}", flush=True)
        del w
