"""Microbench of the paged prefill attention (attn_prefill.hip) at the 256-node prompt's chunk shapes, 70B TP=1
heads (64 q / 8 kv, head_dim 128): µs per launch (graph-replayed) and PFLOP/s of the causal attention work.
    python tools/prefill_attn_bench.py"""

import json
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402

D, BS, NQ, NKV = 128, 16, 64, 8


def graph_us(fn, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(3):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1000 / (3 * reps)


def case(T, ctx):
    nblk = (ctx + BS - 1) // BS
    kc = torch.randn(nblk * BS, NKV, D, device="cuda").to(torch.bfloat16)
    vc = torch.randn(nblk * BS, NKV, D, device="cuda").to(torch.bfloat16)
    bt = torch.randperm(nblk, device="cuda").int().view(1, nblk)
    q = torch.randn(T, NQ, D, device="cuda").to(torch.bfloat16)
    cu = torch.tensor([0, T], dtype=torch.int32, device="cuda")
    cl = torch.tensor([ctx], dtype=torch.int32, device="cuda")
    us = graph_us(lambda: ops.paged_prefill_attention(q, kc, vc, cu, cl, bt, 1 / math.sqrt(D), BS, T))
    keys = sum(ctx - T + i + 1 for i in range(T))          # causal key count over the chunk's queries
    flop = 4.0 * NQ * D * keys
    return dict(T=T, ctx=ctx, us=round(us, 1), pflops=round(flop / us / 1e9, 3))


def main():
    for T, ctx in ((8192, 8192), (8192, 16384), (317, 16701), (2048, 2048), (256, 464)):
        print(json.dumps(case(T, ctx)), flush=True)


if __name__ == "__main__":
    main()
