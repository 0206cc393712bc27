#!/usr/bin/env python3
"""Select the best hipBLASLt / rocBLAS solution for every library GEMM of batched decode and prefill
(PyTorch TunableOp), for Llama-3.3-70B at TP = 1, 2, 4, 8: the engine's batch buckets above the GEMV
range and the prefill row buckets that ops.linear pads prompt chunks to (ops.GEMM_M_BUCKETS).

    python tools/tune_gemms.py --out /tmp/tuned.csv                      # tune (GPU, minutes)
    python tools/tune_gemms.py --validate /tmp/tuned.csv --out table.csv  # keep only measured wins

Validation times every row of the tuned table against the library default (TunableOp off) in a
graph-replayed loop and keeps a row only when the tuned solution is at least 2 % faster, so the
table never makes a shape slower than the default.  The engine reads the result with tuning OFF
(engine/__init__.py::_load_gemm_table), so captured decode graphs replay the selected kernels.
"""

import argparse
import re
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd.ops import GEMM_M_BUCKETS  # noqa: E402

DECODE_BUCKETS = tuple(m for m in GEMM_M_BUCKETS if m <= 128)
PREFILL_BUCKETS = tuple(m for m in GEMM_M_BUCKETS if m > 128)


def shapes(tp: int):
    H, I, V, nq, nkv, D = 8192, 28672 // tp, 128256 // tp, 64 // tp, max(1, 8 // tp), 128
    return [((nq + 2 * nkv) * D, H), (H, nq * D), (2 * I, H), (H, I), (V, H)]


def _timeit(fn, iters: int = 20) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
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


def tune(out: str) -> int:
    t = torch.cuda.tunable
    t.set_filename(out)
    t.enable(True)
    t.tuning_enable(True)
    t.set_max_tuning_duration(40)
    done = set()
    for tp in (1, 2, 4, 8):
        for i, (N, K) in enumerate(shapes(tp)):
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            # the LM head only ever sees one row per sequence (decode batch / last prompt token)
            for M in DECODE_BUCKETS + (PREFILL_BUCKETS if i < 4 else ()):
                if (M, N, K) in done:
                    continue
                done.add((M, N, K))
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                torch.nn.functional.linear(x, w)
                torch.cuda.synchronize()
            print(f"tp={tp} N={N} K={K} tuned", flush=True)
    print(f"{len(done)} shapes tuned; TunableOp writes {t.get_filename()} at exit")
    return 0


def validate(table: str, out: str) -> int:
    lines = Path(table).read_text().splitlines()
    t = torch.cuda.tunable
    t.set_filename(str(Path(out).with_suffix(".scratch.csv")))
    t.tuning_enable(False)
    if not t.read_file(table):
        print("table rejected by its validators")
        return 1
    keep, kept, dropped = [], 0, 0
    for ln in lines:
        m = re.match(r"GemmTunableOp_BFloat16_TN,tn_(\d+)_(\d+)_(\d+)_ld_\d+_\d+_\d+,([^,]+),", ln)
        if m is None:
            keep.append(ln)     # validators
            continue
        N, M, K, sol = int(m.group(1)), int(m.group(2)), int(m.group(3)), m.group(4)
        if sol == "Default":
            continue            # the library default needs no row
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        f = lambda: torch.nn.functional.linear(x, w)
        t.enable(False)
        d = _timeit(f)
        t.enable(True)
        u = _timeit(f)
        ok = u < 0.98 * d
        print(f"M={M:5d} N={N:6d} K={K:6d} default {d:8.1f} us  tuned {u:8.1f} us  {'keep' if ok else 'drop'}",
              flush=True)
        if ok:
            keep.append(ln)
            kept += 1
        else:
            dropped += 1
    Path(out).write_text("\n".join(keep) + "\n")
    print(f"{kept} rows kept, {dropped} dropped -> {out}")
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--validate", default=None, help="tuned table to filter against the library default")
    a = ap.parse_args()
    if not torch.cuda.is_available():
        print("needs a GPU")
        return 1
    return validate(a.validate, a.out) if a.validate else tune(a.out)


if __name__ == "__main__":
    sys.exit(main())
