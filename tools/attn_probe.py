#!/usr/bin/env python3
"""Run only the fused decode attention (TP=8 shapes) N times -- a target for rocprofv3 --pmc."""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from k8s_llm_scheduler_amd import ops  # noqa: E402
from k8s_llm_scheduler_amd.ops import reference as ref  # noqa: E402

ctx = int(sys.argv[1]) if len(sys.argv) > 1 else 564
n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
nq, nkv, D, bs, dev, bf = 8, 1, 128, 16, "cuda", torch.bfloat16
maxb = 256
kc = torch.randn(maxb * bs, nkv, D, device=dev).to(bf)
vc = torch.randn_like(kc)
bt = torch.arange(maxb, device=dev, dtype=torch.int32).view(1, maxb)
cl = torch.full((1,), ctx, device=dev, dtype=torch.int32)
qkv = torch.randn(1, (nq + 2 * nkv) * D, device=dev).to(bf)
cs = ref.rope_table(D, 4096, 500000.0, None).to(dev)
for _ in range(n):
    ops.decode_attention_fused(qkv, cs, kc, vc, bt, cl, 0.088, bs, 1024, nq, nkv, D)
torch.cuda.synchronize()
print("ok")
