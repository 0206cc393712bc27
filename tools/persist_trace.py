#!/usr/bin/env python3
"""Where the layer-persistent decode (decode_persist.hip) spends a layer: chain-wave stamps at every hand-off.

    python tools/persist_trace.py [--tp 8] [--layers 80] [--ctx 528] [--rows 1]

Builds the 70B architecture at one simulated TP rank (random weights), runs the persistent decode and the four-launch
decode (graph-free, GPU-event timed), then one traced persistent launch, and prints per-segment times (median and max
over workgroups, median over layers) next to the layer's weight-streaming floor.
"""

from __future__ import annotations

import argparse
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from k8s_llm_scheduler_amd import ops  # noqa: E402
from k8s_llm_scheduler_amd.models.config import PRESETS, LlamaConfig  # noqa: E402
from k8s_llm_scheduler_amd.models.llama import LlamaModel  # noqa: E402
from k8s_llm_scheduler_amd.parallel import TPGroup  # noqa: E402

SEGS = [("qkv", 8, 0), ("attn+gather_a", 0, 2), ("o_proj", 2, 3), ("gather_o", 3, 4), ("gate_up", 4, 5),
        ("gather_g", 5, 6), ("down", 6, 7), ("gather_x", 7, 8)]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--layers", type=int, default=80)
    ap.add_argument("--ctx", type=int, default=528)
    ap.add_argument("--rows", type=int, default=1)
    ap.add_argument("--preset", default="llama-3.3-70b")
    args = ap.parse_args()
    base = PRESETS[args.preset]
    cfg = LlamaConfig(base.name, args.layers, base.hidden, base.num_heads, base.num_kv_heads, base.head_dim,
                      base.intermediate, base.vocab, rope_scaling=base.rope_scaling, max_position=base.max_position)
    tp = TPGroup(0, args.tp, None, "none", simulate=True) if args.tp > 1 else None
    m = LlamaModel(cfg, tp=tp, device="cuda", seed=1, max_model_len=4096)
    nblk = 64 * args.rows + 8
    m.allocate_kv(nblk, 16)
    B = args.rows
    bt = torch.arange(B * 64, dtype=torch.int32, device="cuda").view(B, 64)
    ctx = torch.full((B,), args.ctx, dtype=torch.int32, device="cuda")
    tok = torch.arange(B, dtype=torch.int32, device="cuda") + 17
    mc = 1024

    def timed(persist: bool, n: int = 10) -> float:
        m.persist_decode = persist
        for _ in range(3):
            m.forward_decode(tok, ctx, bt, mc)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            m.forward_decode(tok, ctx, bt, mc)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    t4 = timed(False)
    tp_ = timed(True)
    assert m._persist is not None and m._persist.ok, "persistent decode not planned for this shape"
    wbytes = sum(sum(t.numel() * t.element_size() for t in (w.wqkv, w.wo, w.wgu, w.wdown)) for w in m.layers)
    print(f"decode step (GPU events, eager launches): four-launch {t4:.3f} ms, persistent {tp_:.3f} ms; "
          f"layer weights {wbytes / args.layers / 1e6:.1f} MB -> floor {wbytes / args.layers / 6.3e6:.1f} us/layer "
          f"at 6.3 TB/s")
    m._persist.set_trace(True)
    m.persist_decode = True
    m.forward_decode(tok, ctx, bt, mc)
    torch.cuda.synchronize()
    tr = m._persist.trace.cpu().double() / 100.0      # us (100 MHz)
    m._persist.set_trace(False)
    G, L, _ = tr.shape
    t0 = tr[:, 0, 0].min().item()
    print(f"grid {G}, layers {L}; traced launch: first QKV done at +{tr[:, 0, 0].median().item() - t0:.1f} us, "
          f"last down done at +{tr[:, L - 1, 7].max().item() - t0:.1f} us")
    per_layer = []
    for l in range(1, L):
        per_layer.append((tr[:, l, 8 if l < L - 1 else 7] - tr[:, l - 1, 8]).median().item() if l < L - 1 else None)
    lay = [(tr[:, l, 0] - tr[:, l - 1, 0]).median().item() for l in range(1, L)]
    print(f"layer period (QKV done -> next QKV done): median {statistics.median(lay):.2f} us, "
          f"min {min(lay):.2f}, max {max(lay):.2f}")
    print(f"{'segment':>16} {'median us':>10} {'max-over-WG us':>15}")
    for name, a, b in SEGS:
        med, mx = [], []
        for l in range(1 if a == 8 else 0, L - (1 if b == 8 else 0)):
            la = l - 1 if a == 8 else l
            d = tr[:, l, b] - tr[:, la, a]
            med.append(d.median().item())
            mx.append(d.max().item())
        print(f"{name:>16} {statistics.median(med):10.2f} {statistics.median(mx):15.2f}")
    # hand-off latency: the LAST workgroup's publish -> the median workgroup has gathered the whole vector
    for name, pub, got, shift in (("qkv->attention", 9, 2, 0), ("o", 10, 4, 0), ("g", 11, 6, 0), ("x", 12, 8, 0)):
        vals = [(tr[:, l, got].median() - tr[:, l, pub].max()).item() for l in range(L - 1)]
        own = [(tr[:, l, got] - tr[:, l, pub]).median().item() for l in range(L - 1)]
        print(f"hand-off {name:>15}: last publish -> median gathered {statistics.median(vals):6.2f} us; "
              f"own publish -> gathered {statistics.median(own):6.2f} us")
    attn = (tr[:, :, 1] - tr[:, :, 0])
    print(f"attention items (their workgroups): max {attn.max(0).values.median().item():.2f} us per layer")
    return 0


if __name__ == "__main__":
    sys.exit(main())
