#!/usr/bin/env python3
"""Headline benchmark: scheduling decisions/s + p50 decision latency, Llama-3.3-70B, TP = N.

BASELINE.json metric: "scheduling decisions/sec + p50 decision latency, Llama-3.3-70B local TP=8".
One *step* is one complete scheduling decision of the reference's per-pod pipeline
(scheduler.py:690-729) minus the apiserver round trips: pod spec -> prompt (exact reference
template, 3-node kind cluster as in ai-test-pods.yaml) -> decision service (cache disabled,
breaker, retries) -> Llama-3 chat template + tokenize -> prefill (paged KV, prefix cache) ->
decode of a FIXED number of tokens (default 64 ~ one JSON answer; EOS ignored because the
weights are random) -> detokenize -> JSON extraction -> validation/fallback.

Weights: Llama-3.3-70B architecture, deterministic random init, bf16 (no checkpoint offline).
Data: synthetic cluster snapshots and pods.  Parallelism: one process per GPU (torchrun),
tensor parallel over RCCL; decisions are made by all ranks together, so the job value is the
decision rate itself.  Scaling is "strong" (fixed work per decision, more GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--preset llama-3.3-70b] [--gen-tokens 64]
    python bench.py --gpus 8                        # launches the 8 ranks itself (torch.distributed.run child)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8   # the same, launched from outside
    python bench.py --gpus 8 --tp 4 --dtype fp8     # 2 half-node replicas (config 5)

--gpus N must equal the launcher's WORLD_SIZE (the run refuses otherwise); without a launcher, N > 1 ranks are
started here before anything touches the GPU.

Default: one TP=N engine (strong scaling).  With --tp T < N, N/T replicas each decide their own
pods (data parallelism, weak scaling) and the value is the sum over replicas.
"""

from __future__ import annotations

import argparse
import json
import logging
import os
import random
import statistics
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

BASELINE_DECISIONS_PER_S = 0.3   # implied by test_e2e.py:68-75 (3 pods within 10 s); BASELINE.md


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--preset", default="llama-3.3-70b")
    ap.add_argument("--nodes", type=int, default=3, help="cluster size in the prompt (reference: 3-node kind)")
    ap.add_argument("--gen-tokens", type=int, default=64)
    ap.add_argument("--batch", type=int, default=1, help="pods decided per step (1 = reference single-pod loop)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16",
                    help="projection weight dtype (fp8 = BASELINE config 5: row-scaled e4m3 weights, bf16 activations)")
    ap.add_argument("--tp", type=int, default=0,
                    help="TP degree of one engine replica (0 = all GPUs); WORLD_SIZE / tp replicas decide in "
                         "parallel (data parallelism, e.g. --tp 4 on 8 GPUs = two half-node engines)")
    ap.add_argument("--prompt-layout", choices=["reference", "cluster_first"], default="reference",
                    help="cluster_first (opt-in compat.prompt_layout): node block before the pod block, so a batch "
                         "decided against one snapshot prefills the cluster state once")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--simulate-tp", type=int, default=0,
                    help="PROFILING ONLY: run one TP rank's shapes on one GPU with collectives skipped")
    ap.add_argument("--arrival-rate", type=float, default=0.0,
                    help="serving mode: pods arrive as a Poisson process at this rate (pods/s) into the scheduler "
                         "in continuous mode on an in-memory apiserver; reports detect->bind latency "
                         "(--steps pods after --warmup pods; single rank)")
    ap.add_argument("--speculative", type=int, default=0,
                    help="prompt-lookup speculative decoding: drafted tokens per step (engine.speculative_tokens)")
    ap.add_argument("--top-p", type=float, default=1.0,
                    help="nucleus sampling (the reference sends no top_p: provider default 1.0); < 1 captures the "
                         "decode graphs with the top-p passes")
    ap.add_argument("--verbose", action="store_true", help="engine INFO logs (init, autotune, graph capture)")
    args = ap.parse_args()
    t_start = time.perf_counter()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and args.simulate_tp <= 1:
        # `python bench.py --gpus N` without a launcher: start the N rank processes ourselves (one per GPU) before
        # anything in this process touches the GPU, and exit with the launcher's code; rank 0 prints the JSON line
        return self_launch(args.gpus)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.simulate_tp <= 1 and world_env != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world_env}: refusing to report a {world_env}-rank run as "
              f"{args.gpus} GPUs", file=sys.stderr)
        return 2

    def progress(msg: str) -> None:
        # stage lines on stderr (stdout carries only the JSON line): shows where a slow start is spent
        print(f"[bench rank {os.environ.get('RANK', '0')} +{time.perf_counter() - t_start:.1f}s] {msg}",
              file=sys.stderr, flush=True)

    from k8s_llm_scheduler_amd.utils import stages

    # every start-up stage is timed and bounded: one that outlives its bound exits with code 3 naming the stage
    # (a rank parked in a collective cannot be interrupted otherwise; utils/stages.py, K8S_STAGE_TIMEOUT_*)
    stages.install(int(os.environ.get("RANK", "0")))
    import torch
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.control import DecisionService, LocalEngineBackend
    from k8s_llm_scheduler_amd.control.breaker import CircuitBreaker
    from k8s_llm_scheduler_amd.control.prompt import PromptEngine
    from k8s_llm_scheduler_amd.engine import build_engine
    from k8s_llm_scheduler_amd.engine.synthetic import random_nodes, random_pod, reference_cluster
    from k8s_llm_scheduler_amd.parallel import init_from_env, make_control_channel
    from k8s_llm_scheduler_amd.parallel.replicas import ReplicaRouterBackend, make_replica_links, serve_replica

    logging.basicConfig(level=logging.WARNING, format="%(asctime)s %(levelname)s %(message)s")
    if args.verbose:
        logging.getLogger("k8s_llm_scheduler_amd").setLevel(logging.INFO)
    progress("imports done")
    world = world_env
    local = int(os.environ.get("LOCAL_RANK", "0"))
    on_gpu = torch.cuda.is_available()   # CPU: reference ops, for trying the harness without a GPU
    if on_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    tp = init_from_env("cuda" if on_gpu else "cpu", tp_size=args.tp)
    if args.simulate_tp > 1:
        from k8s_llm_scheduler_amd.parallel import TPGroup
        tp = TPGroup(0, args.simulate_tp, None, "none", simulate=True)
    rank = tp.global_rank
    dp = tp.replicas
    progress(f"process group ready (tp {tp.world}, comm {tp.comm_info.get('selected', '-')})")

    # --arrival-rate on several ranks: rank 0 runs the scheduler, the other TP ranks of its replica follow its
    # schedule (control channel), every other replica serves rank 0's requests over a link (least-loaded routing)
    serving = args.arrival_rate > 0 and world > 1 and not tp.simulate
    control = make_control_channel(tp) if serving else None
    links = make_replica_links(tp) if serving else []

    t_init = time.perf_counter()
    bs = 16
    per_seq = max(2048, args.max_model_len) + args.gen_tokens + bs   # KV blocks reserved per decision
    # serving (--arrival-rate): the engine's decode batch must hold the pods in flight, not --batch (pods per step)
    slots = max(1, args.batch, 16 if args.arrival_rate > 0 else 1)
    with stages.stage("engine_build"):
        eng = build_engine(args.preset, tp=tp, max_batch=slots, block_size=bs,
                           num_blocks=max(slots, 2) * (per_seq // bs + 2) + 64,
                           max_model_len=args.max_model_len, cuda_graphs=not args.no_graphs,
                           prefix_caching=not args.no_prefix_cache, capture=False, decode_chunk=8,
                           weight_dtype=args.dtype, speculative_tokens=args.speculative, control=control)
    progress("engine built")
    with stages.stage("graph_capture"):
        if eng.use_graphs:
            eng.capture_graphs([b for b in (1, 2, 4, 6, 8, 16, 32, 48, 64) if b <= slots] or [1],
                               nucleus=args.top_p < 1)
        if on_gpu:
            torch.cuda.synchronize()
    init_s = time.perf_counter() - t_init
    progress(f"graphs captured, init {init_s:.1f}s")

    backend = LocalEngineBackend(eng, ignore_eos=True)
    if serving and tp.global_rank != 0:
        if tp.rank == 0:
            serve_replica(backend, links[0], eng)     # a remote replica's leader
        else:
            eng.serve_worker()                        # a TP follower of its replica's leader
        dist.barrier()
        dist.destroy_process_group()
        return 0
    router = ReplicaRouterBackend(backend, links) if links else None
    svc = DecisionService(router or backend, max_retries=3, max_tokens=args.gen_tokens, temperature=0.3, top_p=args.top_p,
                          timeout=None, cache=None, breaker=CircuitBreaker())
    pe = PromptEngine(layout=args.prompt_layout)
    rng = random.Random(1234)
    base_nodes, base_pods = reference_cluster(args.nodes)

    def make_items():
        # one cluster snapshot per step, as the batched scheduler takes one snapshot per round
        # (scheduler.py schedule_batch); utilisation varies from step to step (cache is off anyway)
        nodes = base_nodes if args.nodes == 3 else random_nodes(rng, args.nodes)
        for n in nodes:
            n.pod_count = rng.randint(2, 12)
            n.cpu_usage_percent = n.memory_usage_percent = n.pod_count / n.max_pods * 50
        items = []
        for _ in range(args.batch):
            pod = rng.choice(base_pods) if rng.random() < 0.5 else random_pod(rng)
            items.append((pe.construct_scheduling_prompt(pod, nodes), pod, list(nodes)))
        return items

    # size check on a sample drawn from a COPY of the generator: the timed steps see exactly the snapshots they would
    # without it (the reported prompt sizes below are those of the timed decisions themselves)
    state = rng.getstate()
    prompt_tokens = max(len(eng.render_chat(svc.system_message, p)) for p, _, _ in make_items())
    rng.setstate(state)
    if prompt_tokens + args.gen_tokens > args.max_model_len:
        # the engine would reject every request and the bench would time the fallback path instead
        raise SystemExit(f"prompt ({prompt_tokens} tokens) + --gen-tokens {args.gen_tokens} exceeds --max-model-len "
                         f"{args.max_model_len}: raise --max-model-len")
    if args.arrival_rate > 0:
        rc = run_arrivals(args, eng, svc, prompt_tokens, init_s, tp, router)
        if serving:
            if router is not None:
                router.shutdown()
            eng.shutdown_workers()
            dist.barrier()
            dist.destroy_process_group()
        return rc

    distributed = world > 1 and not tp.simulate

    def barrier():
        if distributed:
            dist.barrier()
        if on_gpu:
            torch.cuda.synchronize()

    with stages.stage("warmup"):
        for _ in range(args.warmup):
            svc.decide_many(make_items())
        if on_gpu:
            torch.cuda.synchronize()
    progress("warmup done")
    # per-stage start-up times of every rank (rank 0's and, per stage, the slowest rank's)
    init_stages = {"rank0": stages.timings()}
    if distributed:
        every = [None] * dist.get_world_size()
        dist.all_gather_object(every, stages.timings())
        init_stages["rank0"] = every[0]
        slowest = {}
        for r, t in enumerate(every):
            for k, v in t.items():
                if k not in slowest or v > slowest[k][0]:
                    slowest[k] = (v, r)
        init_stages["slowest"] = {k: {"s": v, "rank": r} for k, (v, r) in slowest.items()}
    eng.stats.update({k: 0 if isinstance(v, int) else 0.0 for k, v in eng.stats.items()})
    tp.rccl_calls = 0
    lat = []
    log_mark = len(eng.finished_log)
    barrier()
    t0 = time.perf_counter()
    fallbacks = 0
    for _ in range(args.steps):
        s0 = time.perf_counter()
        ds = svc.decide_many(make_items())
        lat.append(time.perf_counter() - s0)
        fallbacks += sum(d.fallback_needed for d in ds)
    barrier()
    elapsed = time.perf_counter() - t0
    # the workload the timed region ran, per engine request (retries included): prompt tokens, tokens prefilled
    # (prompt minus the prefix-cache hit) and tokens generated
    timed = list(eng.finished_log)[log_mark:]

    def dist_of(vals):
        return {"mean": round(statistics.mean(vals), 1), "min": min(vals), "max": max(vals)} if vals else None

    workload = {"engine_requests": len(timed),
                "prompt_tokens": dist_of([e[4] for e in timed]),
                "prefilled_tokens": dist_of([e[4] - e[5] for e in timed]),
                "generated_tokens": dist_of([e[3] for e in timed])}
    if os.environ.get("K8S_ENGINE_TRACE") == "1" and rank == 0:   # host timeline of the last prefill (diagnostics)
        pf = [(t, m) for t, m in getattr(eng, "recovery_trace", []) if m.startswith("prefill")]
        last = max((i for i, (_, m) in enumerate(pf) if m.startswith("prefill: ") and "requests" in m), default=None)
        if last is not None:
            t_0 = pf[last][0]
            progress("last prefill host timeline: " + " | ".join(f"{m.split(': ', 1)[1]} +{(t - t_0) * 1e3:.1f} ms"
                                                                   for t, m in pf[last + 1:last + 9]))
    if distributed:
        t = torch.tensor([elapsed], device="cuda" if on_gpu and tp.backend == "nccl" else "cpu",
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    decisions = args.steps * args.batch * dp   # every replica decides its own pods
    value = decisions / elapsed
    st = eng.stats
    dec_tok_ms = 1000 * st["decode_time"] / max(1, st["decode_steps"])
    res = {
        "metric": "scheduling_decisions_per_sec",
        "value": round(value, 4),
        "unit": "decisions/s",
        # --simulate-tp: ONE GPU ran one TP rank's shapes (collectives skipped) -- n_gpus stays the GPUs used
        "n_gpus": tp.world * dp if not tp.simulate else 1,
        "simulated_tp": tp.world if tp.simulate else None,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak" if dp > 1 else "strong",
        "vs_baseline": round(value / BASELINE_DECISIONS_PER_S, 3),
        "dtype": "bf16" if args.dtype == "bf16" else "fp8-e4m3 weights, bf16 activations",
        "data": "synthetic cluster-state prompts, random-init weights",
        "config": {
            "model": f"{args.preset} (Llama-3.3-70B-Instruct architecture)" if "70b" in args.preset else args.preset,
            "global_batch": args.batch * dp,
            "seq_len": round(workload["prompt_tokens"]["mean"] + args.gen_tokens) if timed else None,
            "prompt_tokens": workload["prompt_tokens"]["mean"] if timed else None,
            "gen_tokens": args.gen_tokens,
            "cluster_nodes": args.nodes,
            "parallelism": (f"dp{dp}-" if dp > 1 else "") + f"tp{tp.world}" + ("-SIMULATED-no-comm" if tp.simulate else ""),
            "cuda_graphs": eng.use_graphs,
            "prefix_cache": not args.no_prefix_cache,
            "prompt_layout": args.prompt_layout,
            "temperature": 0.3,
            "top_p": args.top_p,
        },
        "p50_decision_latency_ms": round(1000 * statistics.median(lat), 2),
        "p99_decision_latency_ms": round(1000 * sorted(lat)[min(len(lat) - 1, int(0.99 * len(lat)))], 2),
        "decode_ms_per_step": round(dec_tok_ms, 3),
        "prefill_ms_per_step": round(1000 * st["prefill_time"] / max(1, args.steps), 2),
        "prefill_ms_per_decision": round(1000 * st["prefill_time"] / max(1, args.steps * args.batch), 2),
        "prefill_tokens_per_decision": round(st["prefill_tokens"] / max(1, args.steps * args.batch), 1),
        "prefill_graph_replays": st.get("prefill_graph_replays", 0),
        "timed_workload": workload,
        "rccl_calls_timed": tp.rccl_calls,
        "prefill_overlap_chunks": st.get("prefill_overlap_chunks", 0),
        "speculative": {"tokens": args.speculative, "steps": st.get("spec_steps", 0),
                        "drafted": st.get("spec_drafted", 0), "accepted": st.get("spec_accepted", 0)},
        "fallback_rate": round(fallbacks / (args.steps * args.batch), 3),
        "init_s": round(init_s, 1),
        "physical_gpus": torch.cuda.device_count() if on_gpu else 0,
        "tp_comm": tp.comm_info,
        "init_stages": init_stages,
        "allreduce_transports": dict(sorted(tp.ar_log.items())),
        "baseline_note": "BASELINE.md publishes no numbers; vs_baseline uses the implied 0.3 decisions/s of test_e2e.py",
    }
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def self_launch(n: int) -> int:
    """Run this same command line as an N-rank job: ``torch.distributed.run`` as a CHILD process (one rank per GPU,
    rendezvous on 127.0.0.1), this process never initialises the GPU and exits with the launcher's code.  Ranks
    r >= device_count share GPU r % device_count (the one-GPU rehearsal)."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    print(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    rc = subprocess.call(cmd, env=env)
    if rc != 0:
        print(f"[bench] the {n}-rank job failed (exit {rc})", file=sys.stderr, flush=True)
    return rc


def run_arrivals(args, eng, svc, prompt_tokens: int, init_s: float, tp, router=None) -> int:
    """Continuous-mode serving under Poisson arrivals: the reference's watch -> decide -> bind loop
    (scheduler.py:662-729) with pods created at exponential inter-arrival times on an in-memory
    apiserver (3-node kind cluster); latency = pod creation -> successful binding."""
    import asyncio

    from k8s_llm_scheduler_amd.control import CustomScheduler
    from k8s_llm_scheduler_amd.kube import FakeKubeAPI, make_node, make_pod

    logging.getLogger("k8s_llm_scheduler_amd").setLevel(logging.ERROR)   # one fallback warning per pod otherwise
    api = FakeKubeAPI([make_node(n, cpu="4", memory="8Gi", pods="110") for n in
                       ("kind-worker", "kind-worker2", "kind-worker3")])
    sched = CustomScheduler("ai-llama-scheduler", api, svc, mode="continuous", max_batch=max(8, args.batch),
                            watch_timeout=3600)
    rng = random.Random(7)
    n_total = args.warmup + args.steps
    created, detected = {}, {}
    claim = sched._claim

    def traced_claim(pod):   # detection time of every pod (the scheduler claims it on its first event)
        key = f"{pod['metadata'].get('namespace', 'default')}/{pod['metadata']['name']}"
        detected.setdefault(key, time.perf_counter())
        return claim(pod)

    sched._claim = traced_claim
    # per-pod phase stamps inside the worker thread: start, decision call, decision return
    phases = {}
    run_claimed, decide = sched._schedule_claimed, sched.llm_client.get_scheduling_decision

    def traced_run(pod, t0, revalidate):
        key = f"{pod['metadata'].get('namespace', 'default')}/{pod['metadata']['name']}"
        phases.setdefault(key, {})["start"] = time.perf_counter()
        tls.key = key
        return run_claimed(pod, t0, revalidate)

    def traced_decide(prompt, spec, nodes):
        ph = phases.setdefault(getattr(tls, "key", ""), {})
        ph["call"] = time.perf_counter()
        d = decide(prompt, spec, nodes)
        ph["ret"] = time.perf_counter()
        return d

    import threading
    tls = threading.local()
    sched._schedule_claimed = traced_run
    sched.llm_client.get_scheduling_decision = traced_decide

    async def main():
        task = asyncio.create_task(sched.start())
        await asyncio.sleep(0.1)
        for i in range(n_total):
            await asyncio.sleep(rng.expovariate(args.arrival_rate))
            name = f"arrival-{i}"
            created[f"default/{name}"] = time.perf_counter()
            api.create_pod(make_pod(name, cpu=f"{rng.choice([100, 250, 500])}m",
                                    memory=f"{rng.choice([128, 256, 512])}Mi"))
        deadline = time.perf_counter() + 600
        while len(api.binding_times) < n_total and time.perf_counter() < deadline:
            await asyncio.sleep(0.01)
        sched.stop()
        await asyncio.wait_for(task, 30)

    t0 = time.perf_counter()
    asyncio.run(main())
    eng.stop_background()
    keys = [f"default/arrival-{i}" for i in range(args.warmup, n_total)]
    lat = sorted(api.binding_times[k] - created[k] for k in keys if k in api.binding_times)
    if not lat:
        raise SystemExit("no pod was bound")
    first = min(created[k] for k in keys)
    span = max(api.binding_times[k] for k in keys if k in api.binding_times) - first
    st = sched.get_stats()
    c2d = sorted(detected[k] - created[k] for k in keys if k in detected) or [0.0]
    d2b = sorted(api.binding_times[k] - detected[k] for k in keys if k in detected and k in api.binding_times) or [0.0]
    def p50(vals):
        vals = sorted(vals) or [0.0]
        return round(1000 * vals[len(vals) // 2], 1)

    ph = [(detected[k], phases[k], api.binding_times[k]) for k in keys
          if k in detected and k in api.binding_times and {"start", "call", "ret"} <= set(phases.get(k, {}))]
    phase_ms = {"detect_to_thread": p50([p["start"] - d for d, p, _ in ph]),
                "thread_to_engine_call": p50([p["call"] - p["start"] for d, p, _ in ph]),
                "decision_call": p50([p["ret"] - p["call"] for d, p, _ in ph]),
                "decision_to_bind": p50([b - p["ret"] for d, p, b in ph])}
    fl = list(eng.finished_log)[args.warmup:]
    ttft = sorted(e[1] - e[0] for e in fl) or [0.0]
    e2e = sorted(e[2] - e[0] for e in fl) or [0.0]
    res = {
        "metric": "scheduling_decisions_per_sec",
        "value": round(len(lat) / span, 4),
        "unit": "decisions/s",
        "n_gpus": tp.world * tp.replicas,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * span / max(1, len(lat)), 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": round(len(lat) / span / BASELINE_DECISIONS_PER_S, 3),
        "dtype": "bf16" if args.dtype == "bf16" else "fp8-e4m3 weights, bf16 activations",
        "data": "synthetic Poisson pod arrivals on an in-memory apiserver, random-init weights",
        "config": {"model": args.preset, "arrival_rate_pods_per_s": args.arrival_rate, "prompt_tokens": prompt_tokens,
                   "gen_tokens": args.gen_tokens, "scheduler_mode": "continuous",
                   "parallelism": (f"dp{tp.replicas}-" if tp.replicas > 1 else "") + f"tp{tp.world}"
                   + ("-SIMULATED-no-comm" if tp.simulate else ""),
                   "replica_dispatch": list(router.dispatched) if router is not None else None},
        "p50_detect_to_bind_ms": round(1000 * statistics.median(lat), 2),
        "p99_detect_to_bind_ms": round(1000 * lat[min(len(lat) - 1, int(0.99 * len(lat)))], 2),
        "max_detect_to_bind_ms": round(1000 * lat[-1], 2),
        "bound": len(lat),
        "total_scheduled": st["total_scheduled"],
        "fallback_decisions": st["fallback_decisions"],
        "wall_s": round(time.perf_counter() - t0, 2),
        "init_s": round(init_s, 1),
        "p50_phase_ms": phase_ms,
        "p50_create_to_detect_ms": round(1000 * c2d[len(c2d) // 2], 1),
        "p50_detect_to_bind_ms_scheduler": round(1000 * d2b[len(d2b) // 2], 1),
        "engine_p50_queue_to_first_token_ms": round(1000 * ttft[len(ttft) // 2], 1),
        "engine_p50_request_ms": round(1000 * e2e[len(e2e) // 2], 1),
        "engine_decode_steps": eng.stats["decode_steps"],
        "engine_graph_replays": eng.stats["graph_replays"],
        "engine_prefill_graph_replays": eng.stats.get("prefill_graph_replays", 0),
        "mean_decode_batch": round(eng.stats["decode_tokens"] / max(1, eng.stats["decode_steps"]), 2),
        "engine_prefill_s": round(eng.stats["prefill_time"], 2),
        "engine_decode_s": round(eng.stats["decode_time"], 2),
        "engine_prefill_tokens": eng.stats["prefill_tokens"],
        "engine_cached_tokens": eng.stats["cached_tokens"],
        "engine_prefill_steps": eng.stats.get("prefill_steps", 0),
        "engine_mixed_steps": eng.stats["mixed_steps"],
        "engine_mixed_decode_rows": eng.stats["mixed_decode_rows"],
    }
    line = json.dumps(res)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
