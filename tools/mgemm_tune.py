#!/usr/bin/env python3
"""Tune the hand-written MFMA GEMM (csrc/kernels/mgemm.hip) per Llama projection shape and compare it with the
library GEMM path it replaces (hipBLASLt / rocBLAS through F.linear with the engine's TunableOp table, + the
separate silu_mul kernel for gate/up; fp8: per-token quantization + torch._scaled_mm).

Every candidate (tile config x split-K) is timed as a captured hipGraph of REPS launches that cycle over enough
copies of the weight to exceed the 256 MiB Infinity Cache (weights are cold in the real decode / prefill loop).

    python tools/mgemm_tune.py --tp 1 8 --m 16 64 256 [--fp8 | --mx] [--write]

--mx tunes the K16 MX modes (fp8 weights) as the decode layer runs them: QKV with MX activations and the RMS
prologue, O / down with MX activations and the residual epilogue writing the stream's MX copy (table key fp8 = 3),
gate/up with MX activations, the RMS prologue and MX SwiGLU output (key fp8 = 4); each compared with the per-token
path it replaces (quantize_act_fp8 + the tuned fp8 plan).

--write merges the winners into engine/assets/mgemm_gfx950.json (the table ops.mgemm_plan reads).
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_llm_scheduler_amd import ops  # noqa: E402
from k8s_llm_scheduler_amd.engine import _load_gemm_table  # noqa: E402

REPS = 12
ACT = [None]   # MX tuning: the activations every candidate takes (MxAct, or the per-token pair for --mx gate/up)
COLD_BYTES = 600 << 20


def shapes(tp: int, hidden=8192, inter=28672, nq=64, nkv=8, D=128, vocab=128256):
    return [
        ("qkv", (nq + 2 * nkv) * D // tp, hidden, ops.EPI_BF16),
        ("o_proj", hidden, nq * D // tp, ops.EPI_BF16),
        ("gate_up", inter // tp, hidden, ops.EPI_SWIGLU),
        ("down", hidden, inter // tp, ops.EPI_BF16),
        ("lm_head", vocab // tp, hidden, ops.EPI_F32),
    ]


def time_graph(fn, copies: int) -> float:
    """us per launch: REPS launches (cycling over `copies` weight copies) in one graph, best of 3 replays."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(2):
            fn(i % copies)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(REPS):
            fn(i % copies)
    best = float("inf")
    for _ in range(3):
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        g.replay()
        t1.record()
        t1.synchronize()
        best = min(best, t0.elapsed_time(t1) * 1000 / REPS)
    del g
    return best


def candidates(M, N, K, epi, fp8, mx_out=False):
    cfgs = ops.mgemm_configs()
    out = []
    mx_out = mx_out or fp8 == 4
    mode = 3 if fp8 == 4 else fp8
    for c, (bm, bn, _th, _lds, _sw, rb) in enumerate(cfgs):
        steps = K * (1 if fp8 else 2) // rb
        if fp8 in (3, 4) and not ops.mgemm_valid(c, M, N, K, epi, mode, 1, mx_out):
            continue
        if bm > max(16, 2 * M) or (M > 64 and bm < 64) or (M > 256 and bm < 128):
            continue
        tiles = ops._mg_tiles(c, M, N, epi)
        seen = set()
        for gr in ops.MG_GRIDS:
            if not ops.mgemm_valid(c, M, N, K, epi, mode, gr, mx_out):
                continue
            nwg = ops.mgemm_nwg(c, M, N, K, epi, fp8, gr)
            if nwg in seen or (gr > 1 and steps // gr < 4) or nwg > 4096:
                continue
            seen.add(nwg)
            out.append((c, gr))
    return out


def lib_fn(x, Ws, epi, fp8):
    def f(i):
        w = Ws[i]
        if fp8 in (3, 4):   # MX tuning: the per-token e4m3 path it replaces (quantize + the tuned fp8 plan)
            return ops.mgemm(x, w, epi)
        if fp8:
            y = ops._fp8_gemm(x, w)
            if epi == ops.EPI_F32:
                y = y.float()
        else:
            y = ops._lib_linear(x, w)
            if epi == ops.EPI_F32:
                y = y.float()
        if epi == ops.EPI_SWIGLU:
            y = ops.silu_mul(y)
        return y
    return f


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--m", type=int, nargs="+", default=[16, 32, 64, 128, 256, 512])
    ap.add_argument("--all-buckets", action="store_true", help="every row bucket of ops.GEMM_M_BUCKETS + 2048..8192")
    ap.add_argument("--only", nargs="*", default=None, help="projection names")
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--mx", action="store_true", help="tune the MX modes (MX activations; MX SwiGLU output)")
    ap.add_argument("--insitu", action="store_true",
                    help="bf16: time O / down with the residual epilogue and gate/up with the RMS prologue, as the "
                         "17-64-row decode layer runs them (QKV stays plain: norm + GEMM)")
    ap.add_argument("--qkv-rms", action="store_true", help="--insitu: time QKV with the RMS prologue too")
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--verbose", action="store_true", help="print every candidate's time")
    a = ap.parse_args()

    if a.all_buckets:
        a.m = list(ops.GEMM_M_BUCKETS) + [2048, 4096, 8192]
    torch.manual_seed(0)
    lib_table = _load_gemm_table()
    print(f"# library GEMM table loaded: {lib_table}; reps {REPS}; weights cycled over >= {COLD_BYTES >> 20} MiB",
          flush=True)
    print(f"{'tp':>3} {'proj':8} {'M':>5} {'N':>6} {'K':>6} {'lib us':>8} {'mgemm us':>9} {'cfg':>4} {'grid':>5} "
          f"{'heur us':>8} {'speedup':>7} {'TB/s':>6}", flush=True)
    plans, rows = {}, []
    t_start = time.time()
    for tp in a.tp:
        for name, N, K, epi in shapes(tp):
            if a.only and name not in a.only:
                continue
            if a.mx:
                if name == "lm_head":   # bf16 residual stream + the final norm: no MX input
                    continue
                a.fp8 = 4 if epi == ops.EPI_SWIGLU else 3
            wrows = 2 * N if epi == ops.EPI_SWIGLU else N
            wbytes = wrows * K * (1 if a.fp8 else 2)
            copies = max(1, min(16, math.ceil(COLD_BYTES / wbytes)))
            Ws = []
            for _ in range(copies):
                w = torch.empty(wrows, K, dtype=torch.bfloat16, device="cuda").uniform_(-0.05, 0.05)
                Ws.append(ops.quantize_fp8(w) if a.fp8 else w)
                del w
            for M in a.m:
                x = torch.empty(M, K, dtype=torch.bfloat16, device="cuda").uniform_(-1, 1)
                ACT[0] = ops.quantize_act_mx(x) if a.fp8 in (3, 4) else None
                res_mx = (a.mx or a.insitu) and name in ("o_proj", "down")   # residual epilogue (+ MX copy)
                rms_mx = (a.mx and name in ("qkv", "gate_up")) or (a.insitu and (name == "gate_up" or (a.qkv_rms and name == "qkv")))   # RMS prologue
                RES = torch.empty(M, N, dtype=torch.bfloat16, device="cuda").uniform_(-1, 1) if res_mx else None
                lib_us = time_graph(lib_fn(x, Ws, epi, a.fp8), copies)
                best = (float("inf"), None)

                def run(i, c, gr):
                    return ops.mgemm(x, Ws[i], epi, cfg=c, grid=gr, act=ACT[0],
                                     mx_out=a.fp8 == 4 or (res_mx and a.mx), res=RES,
                                     rms_eps=1e-5 if rms_mx else None)

                for c, gr in candidates(M, N, K, epi, a.fp8, res_mx and a.mx):
                    us = time_graph(lambda i, c=c, gr=gr: run(i, c, gr), copies)
                    if a.verbose:
                        bm, bn = ops.mgemm_configs()[c][:2]
                        print(f"    cand tp{tp} {name} M={M} cfg {c:2d} ({bm}x{bn}) grid {gr:5d} "
                              f"nwg {ops.mgemm_nwg(c, M, N, K, epi, a.fp8, gr):5d}: {us:8.2f} us", flush=True)
                    if us < best[0]:
                        best = (us, (c, gr))
                gemv_us = None
                if M <= ops.GEMV_MAX_M:   # the decode GEMV path these rows take today
                    if epi == ops.EPI_SWIGLU:
                        gfn = lambda i: ops.linear_swiglu(x, Ws[i])
                    else:
                        gfn = lambda i: ops.linear(x, Ws[i], out_dtype=torch.float32 if epi == ops.EPI_F32 else None)
                    gemv_us = round(time_graph(gfn, copies), 2)
                hc = (ops.mgemm_heuristic(M, N, K, epi, a.fp8) if a.fp8 in (0, 1, 2) else
                      ops.mgemm_mx_plan(M, N, K, epi, True, a.fp8 == 4 or res_mx))
                h_us = time_graph(lambda i: run(i, hc[0], hc[1]), copies)
                us, (c, ks) = best
                plans[f"{ops._mg_bucket(M)},{N},{K},{epi},{int(a.fp8)}"] = [c, ks, round(us, 2), round(lib_us, 2)]
                row = dict(tp=tp, proj=name, M=M, N=N, K=K, epi=epi, fp8=a.fp8, lib_us=round(lib_us, 2),
                           mgemm_us=round(us, 2), cfg=c, grid=ks, heur_us=round(h_us, 2),
                           speedup=round(lib_us / us, 3), tbps=round(wbytes / us / 1e6, 2), gemv_us=gemv_us)
                rows.append(row)
                print(f"{tp:>3} {name:8} {M:>5} {N:>6} {K:>6} {lib_us:8.2f} {us:9.2f} {c:>4} {ks:>5} {h_us:8.2f} "
                      f"{lib_us / us:7.2f} {wbytes / us / 1e6:6.2f}" + (f" gemv {gemv_us:8.2f}" if gemv_us else ""),
                      flush=True)
                del x
            del Ws
            torch.cuda.empty_cache()
            if a.write:
                write_table(plans)
    n_win = sum(r["speedup"] >= 1.0 for r in rows)
    print(f"# mgemm >= library on {n_win}/{len(rows)} shapes; tuning took {time.time() - t_start:.0f}s", flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(rows, f, indent=1)
    if a.write:
        write_table(plans)
        print(f"# wrote {len(plans)} plans to {ops.MG_TABLE_PATH}")
    return 0


def write_table(plans) -> None:
    path = ops.MG_TABLE_PATH
    table = {"arch": "gfx950", "plans": {}}
    if os.path.isfile(path):
        with open(path) as f:
            table = json.load(f)
    table["plans"].update(plans)
    with open(path, "w") as f:
        json.dump(table, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    sys.exit(main())
