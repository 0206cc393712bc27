#!/usr/bin/env python3
"""Per-kernel microbenchmarks on one MI355X (isolated, hipGraph-replayed to strip host overhead).

    python tools/kbench.py [--tp 8] [--ctx 564] [--iters 200]

Reports us/call and effective HBM bandwidth (weight bytes / time) for the decode-path kernels at the per-GPU shapes
of Llama-3.3-70B at a given TP degree.
"""

import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402
from k8s_llm_scheduler_amd.ops import reference as ref  # noqa: E402


def timeit(fn, iters):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=564)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--M", type=int, default=1)
    a = ap.parse_args()
    dev = "cuda"
    H, I, V, nq, nkv, D = 8192, 28672 // a.tp, 128256 // a.tp, 64 // a.tp, max(1, 8 // a.tp), 128
    M = a.M
    bf = torch.bfloat16
    res = []

    def gemv_case(name, N, K, epi=0, norm=False):
        x = torch.randn(M, K, device=dev).to(bf)
        w = (torch.randn(N * (2 if epi == 2 else 1), K, device=dev) * 0.02).to(bf)
        nw = torch.ones(K, device=dev, dtype=bf)
        ri, ro = torch.randn(M, K, device=dev).to(bf), torch.empty(M, K, device=dev, dtype=bf)
        if norm and M > ops.GEMV_KERNEL_MAX_M:
            return
        if norm:  # the model's layout: norm weight folded into W, 1/rms in the epilogue
            fn = lambda: ops.linear_norm(x, w, None, 1e-5, ri, ro, epi=epi)
        elif epi == 2:
            fn = lambda: ops.linear_swiglu(x, w)
        else:
            fn = lambda: ops.linear(x, w, out_dtype=torch.float32 if epi == 1 else None)
        us = timeit(fn, a.iters)
        res.append((name, us, w.numel() * 2 / us / 1e6))
        if M > ops.GEMV_MAX_M:  # library GEMM (hipBLASLt) at the same shape, for comparison
            lib = (lambda: ops.silu_mul(torch.nn.functional.linear(x, w))) if epi == 2 else \
                (lambda: torch.nn.functional.linear(x, w))
            us = timeit(lib, a.iters)
            res.append((name + " [hipBLASLt]", us, w.numel() * 2 / us / 1e6))

    gemv_case("qkv (norm)", (nq + 2 * nkv) * D, H, norm=True)
    gemv_case("qkv", (nq + 2 * nkv) * D, H)
    gemv_case("o_proj", H, nq * D)
    gemv_case("gate_up+swiglu (norm)", I, H, epi=2, norm=True)
    gemv_case("gate_up+swiglu", I, H, epi=2)
    gemv_case("down", H, I)
    gemv_case("lm_head f32 (norm)", V, H, epi=1, norm=True)

    bs = 16
    ctx = a.ctx
    maxb = math.ceil(4096 / bs)
    kc = torch.randn(M * maxb * bs, nkv, D, device=dev).to(bf)
    vc = torch.randn_like(kc)
    bt = torch.arange(M * maxb, device=dev, dtype=torch.int32).view(M, maxb)
    cl = torch.full((M,), ctx, device=dev, dtype=torch.int32)
    qkv = torch.randn(M, (nq + 2 * nkv) * D, device=dev).to(bf)
    cs = ref.rope_table(D, 4096, 500000.0, None).to(dev)
    default_pairs = ops.SPLIT_MAX_PAIRS
    for pairs, tag in ((0, "one-wg"), (default_pairs, "split"), (1 << 20, "split-any")):
        ops.SPLIT_MAX_PAIRS = pairs
        for mc in (1024, 4096):
            us = timeit(lambda: ops.decode_attention_fused(qkv, cs, kc, vc, bt, cl, 0.088, bs, mc, nq, nkv, D), a.iters)
            res.append((f"decode_attn[{tag}] ctx={ctx} maxctx={mc}", us, 2 * ctx * nkv * D * 2 * M / us / 1e6))
        for c2 in (1, 64, 256, 1000):
            cl2 = torch.full((M,), c2, device=dev, dtype=torch.int32)
            us = timeit(lambda: ops.decode_attention_fused(qkv, cs, kc, vc, bt, cl2, 0.088, bs, 1024, nq, nkv, D),
                        a.iters)
            res.append((f"decode_attn[{tag}] ctx={c2}", us, 0))
    ops.SPLIT_MAX_PAIRS = default_pairs
    q = torch.randn(M, nq, D, device=dev).to(bf)
    us = timeit(lambda: ops.paged_decode_attention(q, kc, vc, bt, cl, 0.088, bs, 1024), a.iters)
    res.append((f"paged_decode_attention(split64) ctx={ctx}", us, 2 * ctx * nkv * D * 2 * M / us / 1e6))
    x = torch.randn(M, H, device=dev).to(bf)
    r = torch.randn(M, H, device=dev).to(bf)
    w = torch.ones(H, device=dev, dtype=bf)
    res.append(("rmsnorm fused add", timeit(lambda: ops.rmsnorm(x, w, 1e-5, residual=r), a.iters), 0))
    ids = torch.zeros(M, dtype=torch.int32, device=dev)
    emb = torch.randn(1000, H, device=dev).to(bf)
    res.append(("embedding", timeit(lambda: ops.embedding(ids, emb), a.iters), 0))
    logits = torch.randn(a.tp, M, V, device=dev)
    t = torch.full((M,), 0.3, device=dev)
    p = torch.ones(M, device=dev)
    sd = torch.zeros(M, dtype=torch.int32, device=dev)
    res.append(("sampler (gumbel, full vocab)", timeit(lambda: ops.sample(logits, t, p, sd, sd, shards=a.tp, nucleus=False), a.iters), 0))
    p09 = torch.full((M,), 0.9, device=dev)
    res.append(("sampler (nucleus top_p=0.9, T=0.3)",
                timeit(lambda: ops.sample(logits, t, p09, sd, sd, shards=a.tp, nucleus=True), a.iters), 0))
    t0 = torch.zeros(M, device=dev)
    res.append(("sampler (greedy)", timeit(lambda: ops.sample(logits, t0, p, sd, sd, shards=a.tp, nucleus=False), a.iters), 0))
    empty = torch.zeros(1, device=dev)
    res.append(("trivial torch kernel (launch floor)", timeit(lambda: empty.add_(1), a.iters), 0))
    print(f"# tp={a.tp} M={M} ctx={ctx}")
    for name, us, gbs in res:
        print(f"{name:45s} {us:8.2f} us  {gbs:8.2f} TB/s")


if __name__ == "__main__":
    main()
