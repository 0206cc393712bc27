#!/usr/bin/env python3
"""Persistent GEMV chain vs separate launches (tools/experiments/chain.hip): the measured cost of a kernel boundary in the
decode layer, the quantity behind VERDICT r3 item 2 (one launch per decode layer).

Runs 8 layers x 4 projections (QKV, O, gate/up, down shapes of one TP rank of Llama-3.3-70B, distinct weights per
layer: > 256 MiB, so the Infinity Cache never holds the next layer) as a dependent chain, x of each projection = the
previous projection's output, both ways:
  separate   -- 32 graph-captured launches (the engine's structure)
  persistent -- 1 graph-captured launch, grid barriers between the projections, the next projection's first weights
                requested before each barrier wait
and checks that both give identical outputs and that no barrier wait timed out.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I k8s_llm_scheduler_amd/csrc/kernels \\
        tools/experiments/chain.hip -o tools/experiments/chain.so
    python tools/experiments/chain_probe.py [chain_pre2.so]   (built with -DCH_PRE2=1: two rows per wave in flight
                                                          across each barrier instead of one)
"""

import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent


def shapes(tp: int):
    # (name, N, K); K of O / down are the attention / SwiGLU widths
    return [("qkv", 10240 // tp, 8192), ("o", 8192, 8192 // tp), ("gate_up", 57344 // tp, 8192),
            ("down", 8192, 28672 // tp)]


def main() -> int:
    lib = ctypes.CDLL(str(ROOT / "tools" / "experiments" / (sys.argv[1] if len(sys.argv) > 1 else "chain.so")))
    lib.chain_run.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
    ncu = lib.chain_cus()
    dev = "cuda"
    layers = 8
    for tp in (8, 4):
        sh = shapes(tp)
        if any(k % 512 or k > 8192 for _, _, k in sh):
            continue
        Ws, outs, xs, Ns, Ks = [], [], [], [], []
        x0 = torch.randn(8192, device=dev, dtype=torch.float32)
        prev = x0
        for _ in range(layers):
            for name, n, k in sh:
                Ws.append(torch.empty(n, k, device=dev, dtype=torch.bfloat16).uniform_(-0.02, 0.02))
                o = torch.zeros(max(n, 8192), device=dev, dtype=torch.float32)
                xs.append(prev)
                outs.append(o)
                Ns.append(n)
                Ks.append(k)
                prev = o
        nph = len(Ws)
        wbytes = sum(w.numel() * 2 for w in Ws)
        P = ctypes.c_void_p * nph
        I = ctypes.c_int * nph
        argW = P(*[w.data_ptr() for w in Ws])
        argX = P(*[x.data_ptr() for x in xs])
        argO = P(*[o.data_ptr() for o in outs])
        argN, argK = I(*Ns), I(*Ks)
        cnt = torch.zeros(1, device=dev, dtype=torch.int32)
        err = torch.zeros(1, device=dev, dtype=torch.int32)

        def run(persistent: int):
            rc = lib.chain_run(argW, argX, argO, argN, argK, nph, persistent, ncu, cnt.data_ptr(), err.data_ptr(),
                               ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, rc

        results = {}
        for mode in (0, 1, 0, 1):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                run(mode)
                run(mode)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                run(mode)
            ts = []
            for _ in range(10):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000)
            ts.sort()
            final = outs[-1][:Ns[-1]].clone()
            results.setdefault(mode, []).append((ts[len(ts) // 2], ts[0], final))
            del g
        assert int(err.item()) == 0, "a barrier wait timed out (grid not co-resident?)"
        same = torch.equal(results[0][-1][2], results[1][-1][2])
        sep = min(r[0] for r in results[0])
        per = min(r[0] for r in results[1])
        print(f"TP={tp}: {layers} layers x 4 projections, {wbytes / 2**20:.0f} MiB of weights, grid {ncu}")
        print(f"  separate launches  : {sep:8.1f} us per chain ({sep / layers:6.2f} us per layer, "
              f"{wbytes / sep / 1e6:5.2f} TB/s)")
        print(f"  persistent launch  : {per:8.1f} us per chain ({per / layers:6.2f} us per layer, "
              f"{wbytes / per / 1e6:5.2f} TB/s)  -> {per / sep:5.3f}x; outputs identical: {same}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
