"""Microbench of the cascade decode attention (70B layer shapes per TP rank): the prefix kernel at several group
counts, the per-row kernel over the suffix with the prefix partials merged, and the plain per-row kernel over the
whole context -- each as a replayed graph of 20 launches (µs per launch).
    python tools/cascade_kbench.py [--B 16] [--prefix 4416] [--suffix 64] [--nkv 8]"""

import argparse
import json
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402
from k8s_llm_scheduler_amd.ops import reference as ref  # noqa: E402

D, BS = 128, 16


def graph_us(fn, reps=20):
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
    for _ in range(5):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1000 / (5 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--prefix", type=int, default=4416)
    ap.add_argument("--suffix", type=int, default=64)
    ap.add_argument("--nkv", type=int, default=8)
    ap.add_argument("--G", type=int, default=8)
    a = ap.parse_args()
    B, nkv = a.B, a.nkv
    nq = nkv * a.G
    pb = a.prefix // BS
    own = (a.suffix + BS - 1) // BS + 1
    nblocks = pb + B * own + 2
    kc = torch.randn(nblocks * BS, nkv, D, device="cuda").to(torch.bfloat16)
    vc = torch.randn(nblocks * BS, nkv, D, device="cuda").to(torch.bfloat16)
    bt = torch.zeros(B, pb + own, dtype=torch.int32)
    for b in range(B):
        bt[b, :pb] = torch.arange(pb)
        bt[b, pb:] = pb + b * own + torch.arange(own)
    bt = bt.cuda()
    ctx = torch.full((B,), a.prefix + a.suffix, dtype=torch.int32, device="cuda")
    qkv = torch.randn(B, (nq + 2 * nkv) * D, device="cuda").to(torch.bfloat16)
    cs = ref.rope_table(D, 16384, 500000.0, None).cuda()
    cas = torch.tensor([a.prefix // 64, 0], dtype=torch.int32, device="cuda")
    sc = 1 / math.sqrt(D)
    full_mc = 1024 * math.ceil((a.prefix + a.suffix) / 1024)
    suf_mc = 1024 * math.ceil((a.prefix + a.suffix - 64 * (a.prefix // 64)) / 1024)
    out = dict(B=B, nq=nq, nkv=nkv, prefix=a.prefix, suffix=a.suffix)
    out["per_row_us"] = round(graph_us(lambda: ops.decode_attention_fused(qkv, cs, kc, vc, bt, ctx, sc, BS, full_mc, nq,
                                                                          nkv, D)), 2)
    ps = a.G * D + 2 * a.G
    for ngm in sorted({4, 8, 16, 32, ops.cascade_groups_max(B, nq, nkv)}):
        pre = torch.empty(B * nkv * ngm * ps, device="cuda")

        def prefix_only():
            ops.native().decode_prefix(pre.data_ptr(), ngm, qkv.data_ptr(), cs.data_ptr(), kc.data_ptr(),
                                       vc.data_ptr(), bt.data_ptr(), ctx.data_ptr(), cas.data_ptr(), sc, B, nq, nkv, D,
                                       BS, bt.shape[1], ngm, -1)

        out[f"prefix_ngm{ngm}_us"] = round(graph_us(prefix_only), 2)
        out[f"cascade_ngm{ngm}_us"] = round(graph_us(lambda: ops.decode_attention_fused(
            qkv, cs, kc, vc, bt, ctx, sc, BS, suf_mc, nq, nkv, D, cascade=(cas, ngm))), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
