#!/usr/bin/env python3
"""Tune the big-tile MFMA GEMM (csrc/kernels/pgemm.hip) per Llama projection shape at prefill row counts and
compare it with the library GEMM (hipBLASLt through F.linear + silu_mul; fp8: per-token quantization +
torch._scaled_mm) and with mgemm.hip's tuned plan.

Every candidate (tile config x split-K x group_m) is timed as a captured hipGraph of REPS launches cycling over
enough weight copies to exceed the 256 MiB Infinity Cache (prefill weights are cold).

    python tools/pgemm_tune.py --tp 1 8 --m 256 512 2048 8192 [--fp8] [--model 8b] [--write] [--json-out f.json]

--write merges the winners into engine/assets/pgemm_gfx950.json (the table ops.gemm_route reads; a shape where
mgemm's own tuned plan was faster is recorded as "mgemm").
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
from tools.mgemm_tune import COLD_BYTES, lib_fn, shapes, time_graph  # noqa: E402

SPLITS = (1, 2, 3, 4, 6, 8, 12, 16)


def candidates(M, N, K, epi, fp8, num_cus=256, kernels=("pgemm", "pgemm4")):
    """(kernel, cfg, splits, group_m) plans worth timing."""
    out = []
    kt = K * (1 if fp8 else 2) // 128
    for kern in kernels:
        if kern == "pgemm4" and fp8:
            continue
        cfgs = ops.pgemm_configs() if kern == "pgemm" else ops.pgemm4_configs()
        tiles_fn = ops.pgemm_tiles if kern == "pgemm" else ops.pgemm4_tiles
        for c, (bp, bq, _lds) in enumerate(cfgs):
            if bq > 2 * max(M, 128):
                continue
            tiles = tiles_fn(c, M, N, epi)
            for s in SPLITS:
                if s > 1 and (tiles * s > 2 * num_cus or kt // s < 4):
                    continue
                for gm in ((1,) if M <= bq else (4, 8)):
                    out.append((kern, c, s, gm))
    return out


def run_plan(kern, x, w, epi, c, s, gm):
    if kern == "pgemm4":
        return ops.pgemm4(x, w, epi, cfg=c, splits=s, group_m=gm)
    return ops.pgemm(x, w, epi, cfg=c, splits=s, group_m=gm)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--m", type=int, nargs="+", default=[256, 512, 2048, 8192])
    ap.add_argument("--only", nargs="*", default=None, help="projection names")
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--no-mgemm", action="store_true")
    ap.add_argument("--kernels", nargs="+", default=["pgemm", "pgemm4"])
    ap.add_argument("--write", action="store_true")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--model", choices=["70b", "8b"], default="70b", help="projection shapes of Llama-3.3-70B / 3-8B")
    ap.add_argument("--merge-json", default=None, help="merge the plans of an earlier --json-out run into the table "
                                                        "(no GPU needed) and exit")
    a = ap.parse_args()
    if a.merge_json:
        with open(a.merge_json) as f:
            rows = json.load(f)
        plans = {}
        for r in rows:
            key = f"{r['M']},{r['N']},{r['K']},{r['epi']},{int(r['fp8'])}"
            if r["mgemm_us"] == r["mgemm_us"] and r["mgemm_us"] < r["pgemm_us"]:   # (NaN: mgemm not timed)
                plans[key] = ["mgemm", 0, 0, 0, r["mgemm_us"], r["lib_us"]]
            else:
                plans[key] = [r["kernel"], r["cfg"], r["splits"], r["group_m"], r["pgemm_us"], r["lib_us"]]
        _write_plans(plans)
        return 0
    dims = {} if a.model == "70b" else dict(hidden=4096, inter=14336, nq=32, nkv=8)

    torch.manual_seed(0)
    lib_table = _load_gemm_table()
    print(f"# library GEMM table loaded: {lib_table}; weights cycled over >= {COLD_BYTES >> 20} MiB", flush=True)
    print(f"{'tp':>3} {'proj':8} {'M':>5} {'N':>6} {'K':>6} {'lib us':>8} {'mgemm':>8} {'pgemm':>8} {'cfg':>3} "
          f"{'spl':>3} {'gm':>2} {'vs lib':>6} {'TF/s':>6} {'TB/s':>5}", flush=True)
    rows, plans = [], {}
    t0 = time.time()
    for tp in a.tp:
        for name, N, K, epi in shapes(tp, **dims):
            if a.only and name not in a.only:
                continue
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
                lib_us = time_graph(lib_fn(x, Ws, epi, a.fp8), copies)
                mg_us = float("nan")
                if not a.no_mgemm:
                    mg_us = time_graph(lambda i: ops.mgemm(x, Ws[i], epi), copies)
                best = (float("inf"), None)
                for kern, c, s, gm in candidates(M, N, K, epi, a.fp8, kernels=a.kernels):
                    us = time_graph(lambda i, k=kern, c=c, s=s, gm=gm: run_plan(k, x, Ws[i], epi, c, s, gm), copies)
                    if a.verbose:
                        print(f"    cand tp{tp} {name} M={M} {kern} cfg {c} splits {s} gm {gm}: {us:8.2f} us",
                              flush=True)
                    if us < best[0]:
                        best = (us, (kern, c, s, gm))
                us, (kern, c, s, gm) = best
                flop = 2.0 * M * wrows * K
                if mg_us < us:   # mgemm's own tuned plan wins: the router keeps this shape on mgemm
                    plans[f"{M},{N},{K},{epi},{int(a.fp8)}"] = ["mgemm", 0, 0, 0, round(mg_us, 2), round(lib_us, 2)]
                else:
                    plans[f"{M},{N},{K},{epi},{int(a.fp8)}"] = [kern, c, s, gm, round(us, 2), round(lib_us, 2)]
                hand = min(us, mg_us)
                row = dict(tp=tp, proj=name, M=M, N=N, K=K, epi=epi, fp8=a.fp8, lib_us=round(lib_us, 2), hand_us=round(hand, 2),
                           hand_vs_lib=round(lib_us / hand, 3),
                           mgemm_us=round(mg_us, 2), pgemm_us=round(us, 2), kernel=kern, cfg=c, splits=s, group_m=gm,
                           vs_lib=round(lib_us / us, 3), tflops=round(flop / us / 1e6, 1),
                           tbps=round(wbytes / us / 1e6, 2))
                rows.append(row)
                print(f"{tp:>3} {name:8} {M:>5} {N:>6} {K:>6} {lib_us:8.2f} {mg_us:8.2f} {us:8.2f} {kern[-1]}{c:>2} {s:>3} "
                      f"{gm:>2} {lib_us / us:6.2f} {flop / us / 1e6:6.0f} {wbytes / us / 1e6:5.2f}", flush=True)
                del x
            del Ws
            torch.cuda.empty_cache()
    n_win = sum(r["vs_lib"] >= 1.0 for r in rows)
    n_hand = sum(r["hand_vs_lib"] >= 1.0 for r in rows)
    print(f"# pgemm >= library on {n_win}/{len(rows)} shapes, best hand-written (pgemm/pgemm4/mgemm) on {n_hand}; "
          f"{time.time() - t0:.0f}s", flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(rows, f, indent=1)
    if a.write:
        _write_plans(plans)
    return 0


def _write_plans(plans: dict) -> None:
    path = ops.PG_TABLE_PATH
    table = {"arch": "gfx950", "plans": {}}
    if os.path.isfile(path):
        with open(path) as f:
            table = json.load(f)
    table["plans"].update(plans)
    with open(path, "w") as f:
        json.dump(table, f, indent=0, sort_keys=True)
    print(f"# wrote {len(plans)} plans to {path}")


if __name__ == "__main__":
    sys.exit(main())
