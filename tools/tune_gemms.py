#!/usr/bin/env python3
"""Select the best hipBLASLt / rocBLAS solution for every library GEMM of batched decode (PyTorch
TunableOp), for Llama-3.3-70B at TP = 1, 2, 4, 8 and the engine's batch buckets above the GEMV range.

    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \\
    PYTORCH_TUNABLEOP_FILENAME=k8s_llm_scheduler_amd/engine/assets/tunableop_gfx950%d.csv \\
        python tools/tune_gemms.py

The engine reads the resulting table with tuning OFF (engine/__init__.py::_load_gemm_table), so
captured decode graphs replay the selected kernels; shapes not in the table keep the library default.
"""

import sys

import torch

BUCKETS = (16, 32, 48, 64, 96, 128)


def shapes(tp: int):
    H, I, V, nq, nkv, D = 8192, 28672 // tp, 128256 // tp, 64 // tp, max(1, 8 // tp), 128
    return [((nq + 2 * nkv) * D, H), (H, nq * D), (2 * I, H), (H, I), (V, H)]


def main() -> int:
    if not torch.cuda.is_available():
        print("needs a GPU")
        return 1
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_max_tuning_duration(40)
    done = set()
    for tp in (1, 2, 4, 8):
        for (N, K) in shapes(tp):
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            for M in BUCKETS:
                if (M, N, K) in done:
                    continue
                done.add((M, N, K))
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                torch.nn.functional.linear(x, w)
                torch.cuda.synchronize()
            print(f"tp={tp} N={N} K={K} tuned", flush=True)
    print(f"{len(done)} shapes tuned; TunableOp writes {torch.cuda.tunable.get_filename()} at exit")
    return 0


if __name__ == "__main__":
    sys.exit(main())
