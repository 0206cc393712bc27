#!/usr/bin/env python3
"""Probe: the engine part of the 8-rank one-GPU TP rehearsal (tests/test_multigpu.py) with Python stack dumps of
every rank after DUMP seconds, to see where a straggler rank waits.  Env: K8S_SGEMV, K8S_XGMI_TIMEOUT_S."""
import faulthandler
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def rank_fn(rank, world):
    import torch
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine
    from k8s_llm_scheduler_amd.parallel import init_from_env

    faulthandler.dump_traceback_later(float(os.environ.get("DUMP", "40")), exit=False)
    tp = init_from_env("cuda", backend="gloo", comm="xgmi")
    t0 = time.time()
    eng = build_engine("tiny-tp8", tp=tp, device="cuda", max_batch=4, max_model_len=512, num_blocks=128, seed=1,
                       capture_nucleus=True)
    print(f"rank {rank}: engine built {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    outs = eng.generate(["tensor parallel over xgmi", "second request", "third"],
                        [SamplingParams(max_tokens=12, temperature=0.8, seed=9, ignore_eos=True),
                         SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True),
                         SamplingParams(max_tokens=12, temperature=0.3, top_p=0.9, seed=4, ignore_eos=True)])
    torch.cuda.synchronize()
    print(f"rank {rank}: generate done {time.time() - t0:.1f}s stats {eng.stats['graph_replays']}", file=sys.stderr,
          flush=True)
    faulthandler.cancel_dump_traceback_later()
    dist.barrier()
    dist.destroy_process_group()
    return [o.token_ids for o in outs]


if __name__ == "__main__":
    from mp_harness import run_ranks

    world = int(os.environ.get("WORLD", "8"))
    res = run_ranks(rank_fn, world, env={"K8S_TP_BACKEND": "gloo", "K8S_TP_COMM": "xgmi"},
                    timeout_s=float(os.environ.get("T", "150")))
    print("ok", res[0])
