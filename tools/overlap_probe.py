#!/usr/bin/env python3
"""TP > 1 prefill with and without the two-micro-batch all-reduce overlap (LlamaModel._layers_folded_overlap).

Spawns ``--world`` rank processes (gloo process group + the xGMI peer-memory collectives, so several ranks
may share one GPU), builds the Llama-3.3-70B architecture with ``--layers`` decoder layers at TP = world,
and times one ``--tokens``-token prefill chunk unsplit and split (max over ranks, median of ``--reps``).
Under ``rocprofv3 --kernel-trace`` the trace shows whether the xg_allreduce kernels of a rank run
concurrently with its GEMMs (tools/overlap_timeline.py).  Ranks sharing one GPU time-share its CUs, so the
timings here are a rehearsal of the schedule, not the 8-GPU numbers."""

import argparse
import dataclasses
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def _rank(rank, world):
    import torch
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.engine.engine import split_prefill_meta
    from k8s_llm_scheduler_amd.models.config import PRESETS
    from k8s_llm_scheduler_amd.models.llama import LlamaModel
    from k8s_llm_scheduler_amd.parallel import init_from_env

    a = json.loads(os.environ["OVERLAP_PROBE_ARGS"])
    tp = init_from_env("cuda", backend="gloo", comm="xgmi")
    assert tp.xgmi is not None
    cfg = dataclasses.replace(PRESETS["llama-3.3-70b"], num_layers=a["layers"])
    m = LlamaModel(cfg, tp, device="cuda", seed=1, max_model_len=4096)
    T, bs = a["tokens"], 16
    m.allocate_kv(T // bs + 2, bs)
    i32 = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")   # noqa: E731
    ids, pos, slots = i32([(7 * i) % 120000 + 5 for i in range(T)]), i32(list(range(T))), i32(list(range(T)))
    bt = i32([list(range(T // bs + 1))])
    cu, ctx = [0, T], [T]
    T0 = T // 2
    halves = [(i32(c), i32(x), bt, max(q - p for p, q in zip(c, c[1:]))) for c, x, _ in split_prefill_meta(cu, ctx, T0)]
    split = (T0, halves[0], halves[1])
    out = {}
    modes = {"unsplit": None, "split": split}
    for name in a["modes"].split(",") * 2:
        sp = modes[name]
        ts = []
        for it in range(a["reps"] + 1):
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.forward_prefill(ids, pos, slots, i32(cu), i32(ctx), bt, T, i32([T - 1]), split=sp)
            torch.cuda.synchronize()
            if it:
                ts.append((time.perf_counter() - t0) * 1e3)
        out.setdefault(name, []).append(statistics.median(ts))
    dist.barrier()
    dist.destroy_process_group()
    return {k: min(v) for k, v in out.items()}


def simulated(a):
    """One TP rank's shapes in this process, collectives skipped: what splitting a chunk costs by itself
    (two half-size passes over every weight, the comm-stream fork / join), per chunk length."""
    import torch

    from k8s_llm_scheduler_amd.engine.engine import split_prefill_meta
    from k8s_llm_scheduler_amd.models.config import PRESETS
    from k8s_llm_scheduler_amd.models.llama import LlamaModel
    from k8s_llm_scheduler_amd.parallel import TPGroup

    os.environ["K8S_PREFILL_OVERLAP"] = "sim"
    cfg = dataclasses.replace(PRESETS["llama-3.3-70b"], num_layers=a.layers)
    tmax = max(a.sweep)
    m = LlamaModel(cfg, TPGroup(0, a.simulate_tp, None, "none", simulate=True), device="cuda", seed=1,
                   max_model_len=max(4096, tmax))
    bs = 16
    m.allocate_kv(tmax // bs + 2, bs)
    i32 = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")   # noqa: E731
    rows = []
    for T in a.sweep:
        ids, pos, slots = i32([(7 * i) % 120000 + 5 for i in range(T)]), i32(list(range(T))), i32(list(range(T)))
        bt = i32([list(range(T // bs + 1))])
        halves = [(i32(c), i32(x), bt, max(q - p for p, q in zip(c, c[1:])))
                  for c, x, _ in split_prefill_meta([0, T], [T], T // 2)]
        res = {}
        for name, sp in (("unsplit", None), ("split", (T // 2, halves[0], halves[1]))) * 2:
            ts = []
            for it in range(a.reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                m.forward_prefill(ids, pos, slots, i32([0, T]), i32([T]), bt, T, i32([T - 1]), split=sp)
                torch.cuda.synchronize()
                if it:
                    ts.append((time.perf_counter() - t0) * 1e3)
            res[name] = min(res.get(name, 1e9), statistics.median(ts))
        rows.append({"tokens": T, "ms_unsplit": round(res["unsplit"], 3), "ms_split": round(res["split"], 3),
                     "split_cost_us_per_layer": round((res["split"] - res["unsplit"]) * 1e3 / a.layers, 1)})
        print(json.dumps({"probe": "prefill_split_cost_simulated", "tp": a.simulate_tp, "layers": a.layers, **rows[-1]}),
              flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--tokens", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="unsplit,split", help="comma list of unsplit / split")
    ap.add_argument("--simulate-tp", type=int, default=0, help="one rank of this TP degree, no collectives")
    ap.add_argument("--sweep", type=int, nargs="+", default=[256, 1024, 2048, 4096, 8192])
    a = ap.parse_args()
    if a.simulate_tp:
        return simulated(a)
    from mp_harness import run_ranks

    res = run_ranks(_rank, a.world, env={"K8S_TP_BACKEND": "gloo", "K8S_TP_COMM": "xgmi", "K8S_XGMI_MAX_BYTES": str(4 << 20),
                                         "K8S_PREFILL_OVERLAP_MIN": "0",
                                         "OVERLAP_PROBE_ARGS": json.dumps(vars(a))}, timeout_s=600)
    worst = {k: round(max(res[r][k] for r in res), 3) for k in res[0]}
    print(json.dumps({"probe": "prefill_allreduce_overlap", "world": a.world, "layers": a.layers, "tokens": a.tokens,
                      "ms_max_over_ranks": worst, "per_rank": res}))


if __name__ == "__main__":
    main()
