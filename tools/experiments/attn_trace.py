#!/usr/bin/env python3
"""Timeline of the split decode-attention kernel (attn_decode_split.hip built with -DK8S_ATTN_TRACE).

Every workgroup (one wave = one 64-token chunk) stamps s_memrealtime (10 ns ticks) after draining its memory
traffic at: 0 entry, 1 context length + block ids, 2 q loads + RoPE, 3 K loads + scores + softmax,
4 V loads + P.V, 5 partial record stored, 6 arrival atomic returned, 7 output written (single chunk or the
merging chunk), 8 merge: statistics + first accumulator batch loaded, 9 merge: all chunks combined.  The waits the probe inserts serialise some loads, so stage times are upper bounds; the
point is where the chain spends its microseconds.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -DK8S_ATTN_TRACE \\
        -I k8s_llm_scheduler_amd/csrc/kernels k8s_llm_scheduler_amd/csrc/kernels/attn_decode_split.hip \\
        -o tools/experiments/attn_trace.so
    python tools/attn_trace.py
"""

import ctypes
import math
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from k8s_llm_scheduler_amd.ops import reference as ref  # noqa: E402

STAGES = ("ctx+bt", "q+rope", "K+softmax", "V+PV", "store", "atomic", "out", "merge:stats+batch0", "merge:rest",
          "merge:store")


def main() -> int:
    lib = ctypes.CDLL(str(ROOT / "tools" / "experiments" / (sys.argv[1] if len(sys.argv) > 1 else "attn_trace.so")))
    lib.k8s_attn_trace_set.argtypes = [ctypes.c_void_p]
    lib.k8s_decode_split_workspace.restype = ctypes.c_longlong
    lib.k8s_decode_split_workspace.argtypes = [ctypes.c_int] * 4
    lib.k8s_decode_attention_split.argtypes = [ctypes.c_void_p] * 9 + [ctypes.c_float] + [ctypes.c_int] * 7 + \
        [ctypes.c_void_p]
    dev, bf, D, bs = "cuda", torch.bfloat16, 128, 16
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    # (nq, nkv, tag, batch, contexts, graph-class max context or None = the context itself)
    cases = [(8, 1, "TP=8", 1, (64, 256, 564, 1024), None), (64, 8, "TP=1", 1, (64, 256, 564, 1024), None),
             (64, 8, "TP=1 B=4", 4, (564,), 1024), (64, 8, "TP=1 B=8", 8, (564,), 1024),
             (64, 8, "TP=1 B=8", 8, (564,), None)]
    for (nq, nkv, tag, B, ctxs, maxctx) in cases:
        for ctx in ctxs:
            maxb = 4096 // bs
            pmax = math.ceil((maxctx or ctx) / 64)
            kc = torch.randn(B * maxb * bs, nkv, D, device=dev).to(bf)
            vc = torch.randn_like(kc)
            bt = torch.arange(B * maxb, device=dev, dtype=torch.int32).view(B, maxb)
            cl = torch.full((B,), ctx, device=dev, dtype=torch.int32)
            qkv = torch.randn(B, (nq + 2 * nkv) * D, device=dev).to(bf)
            cs = ref.rope_table(D, 4096, 500000.0, None).to(dev)
            out = torch.empty(B, nq * D, device=dev, dtype=bf)
            part = torch.empty(max(1, lib.k8s_decode_split_workspace(B, nq, nkv, pmax)), device=dev)
            cnt = torch.zeros(B * nkv, dtype=torch.int32, device=dev)
            nwg = pmax * nkv * B
            tr = torch.zeros(nwg * 12, dtype=torch.int64, device=dev)
            assert lib.k8s_attn_trace_set(ctypes.c_void_p(tr.data_ptr())) == 0
            stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

            def run():
                rc = lib.k8s_decode_attention_split(out.data_ptr(), part.data_ptr(), cnt.data_ptr(), qkv.data_ptr(),
                                                    cs.data_ptr(), kc.data_ptr(), vc.data_ptr(), bt.data_ptr(),
                                                    cl.data_ptr(), 0.088, B, nq, nkv, D, bs, maxb, pmax, stream)
                assert rc == 0, rc

            for cold in (False, True):
                for _ in range(3):
                    run()
                if cold:
                    flush.fill_(1)
                tr.zero_()
                run()
                torch.cuda.synchronize()
                t = tr.view(nwg, 12).cpu().double()
                t0 = t[:, 0][t[:, 0] > 0].min()
                rel = torch.where(t > 0, (t - t0) * 0.01, torch.full_like(t, float("nan")))  # us
                end = torch.nan_to_num(rel[:, 7], nan=-1).max().item()
                starts = rel[:, 0]
                live = ~torch.isnan(rel[:, 1])
                ends = torch.nan_to_num(rel[:, 5], nan=-1)[live]
                temp = 'cold' if cold else 'hot '
                print(f"{tag} ctx={ctx:5d} pmax={pmax:2d} wgs={nwg:4d} {temp}: total {end:5.2f} us; "
                      f"entry spread {torch.nan_to_num(starts, nan=0).max().item():4.2f} us (live "
                      f"{torch.nan_to_num(starts[live], nan=0).max().item():4.2f}); partial stored p50/max "
                      f"{ends.median().item():4.2f}/{ends.max().item():4.2f} us")
                # stage i ends at stamp i; the single-chunk output (7) follows 4, the merge runs 6 -> 8 -> 9 -> 7
                prev = {1: 0, 2: 1, 3: 2, 4: 3, 5: 4, 6: 5, 7: 4, 8: 6, 9: 8, 10: 9}
                end_of = {i: i for i in range(1, 10)}
                end_of[10] = 7
                med = []
                for i in range(1, 11):
                    a_, b_ = rel[:, end_of[i]], rel[:, prev[i]]
                    if i == 7:  # single-chunk output only (no stamp 5)
                        a_ = torch.where(torch.isnan(rel[:, 5]), a_, torch.full_like(a_, float("nan")))
                    med.append(torch.nanmedian(a_ - b_).item())
                print("    median stage us: " + "  ".join(f"{s}={v:4.2f}" for s, v in zip(STAGES, med)
                                                         if not math.isnan(v)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
