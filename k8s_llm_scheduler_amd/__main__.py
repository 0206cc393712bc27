"""Command line: ``python -m k8s_llm_scheduler_amd [run|verify|smoke]``.

``run`` is the reference's ``python scheduler.py`` (``scheduler.py:775-823``): banner, build the
scheduler, watch pods until Ctrl+C, print final statistics.  Under ``torchrun`` (one process per
GPU) rank 0 runs the control plane and the decision engine's rank-0 shard; every other rank
follows rank 0's engine schedule (tensor parallel over RCCL).

``verify`` replaces ``verify_setup.py`` (files, env, packages, GPU + native extension, cluster).
``smoke`` replaces ``test_runner.py``: apply the three ai-test-pods, wait, count bound pods --
against a real cluster, or fully in-process with ``--fake`` (no cluster needed).
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import os
import sys
import time
from pathlib import Path
from typing import Optional

from .config import Config, load_config, load_dotenv

log = logging.getLogger("k8s_llm_scheduler_amd")
ROOT = Path(__file__).resolve().parent.parent
TEST_PODS = ROOT / "examples" / "ai-test-pods.yaml"


def _fake_cluster(n: int):
    from .kube import FakeKubeAPI, make_node

    names = [f"kind-worker{i + 1 if i else ''}" for i in range(n)]
    return FakeKubeAPI([make_node(nm, cpu="8", memory="16281924Ki") for nm in names], run_bound_pods=True)


class Runtime:
    """What build_backend made for this process: the decision backend (rank 0), the engine, the
    parallel layout and the links to the other engine replicas (data parallelism)."""

    def __init__(self, backend=None, engine=None, tp=None, links=(), local=None):
        self.backend, self.engine, self.tp, self.links, self.local = backend, engine, tp, list(links), local

    @property
    def is_control_rank(self) -> bool:
        return self.tp is None or self.tp.global_rank == 0

    def serve(self) -> None:
        """Non-control ranks: a remote replica's leader answers rank 0's batches, every other
        rank follows its replica leader's engine schedule."""
        from .parallel.replicas import serve_replica

        if self.tp.rank == 0 and self.links:
            serve_replica(self.local, self.links[0], self.engine)
        else:
            self.engine.serve_worker()

    def shutdown(self) -> None:
        if self.is_control_rank:
            if hasattr(self.router, "shutdown"):
                self.router.shutdown()
            if self.engine is not None:
                self.engine.shutdown_workers()

    router = None


def build_backend(cfg: Config, metrics=None) -> Runtime:
    from .control.backends import LocalEngineBackend, ScriptedBackend, first_node_answer

    if not cfg.engine.enabled or cfg.engine.backend == "fallback":
        return Runtime()
    from .control.backends import FaultInjectingBackend

    if cfg.engine.backend == "scripted":
        return Runtime(FaultInjectingBackend.from_spec(ScriptedBackend(default=first_node_answer),
                                                       cfg.engine.fault_injection, cfg.engine.seed))
    from .engine import engine_from_config
    from .parallel import init_from_env, make_control_channel
    from .parallel.replicas import ReplicaRouterBackend, make_replica_links

    tp = init_from_env(tp_size=cfg.engine.tp)
    control = make_control_channel(tp)
    links = make_replica_links(tp)
    engine = engine_from_config(cfg, tp, metrics, control=control)
    local = LocalEngineBackend(engine, ignore_eos=cfg.engine.ignore_eos)
    rt = Runtime(None, engine, tp, links, local)
    backend = local
    if tp.global_rank == 0 and links:
        backend = rt.router = ReplicaRouterBackend(local, links)
    rt.backend = FaultInjectingBackend.from_spec(backend, cfg.engine.fault_injection, cfg.engine.seed)
    return rt


def build_scheduler(cfg: Config, api, backend, metrics=None):
    from .control.decision import DecisionService
    from .control.scheduler import CustomScheduler

    svc = DecisionService.from_config(cfg, backend, metrics=metrics)
    return CustomScheduler.from_config(cfg, api, svc, metrics=metrics)


def print_final_stats(stats: dict) -> None:
    """Same lines as scheduler.py:803-819, plus the two counters the reference never printed."""
    print("\n" + "=" * 60)
    print(" Final Statistics:")
    print("=" * 60)
    print(f"Total Scheduled: {stats['total_scheduled']}")
    print(f"LLM Decisions: {stats['llm_decisions']}")
    print(f"Fallback Decisions: {stats['fallback_decisions']}")
    print(f"Failed Bindings: {stats['failed_bindings']}")
    llm = stats.get("llm_client", {})
    print("\nLLM Client Stats:")
    print(f"  Total Requests: {llm.get('total_requests', 0)}")
    print(f"  Successful: {llm.get('successful_requests', 0)}")
    print(f"  Failed: {llm.get('failed_requests', 0)}")
    print(f"  Cached: {llm.get('cached_requests', 0)}")
    print(f"  Circuit Breaker Trips: {llm.get('circuit_breaker_trips', 0)}")
    print(f"  Avg Response Time: {llm.get('avg_response_time', 0):.2f}s")
    print("=" * 60)


def cmd_run(args, cfg: Config) -> int:
    from .control.metrics import SchedulerMetrics

    metrics = SchedulerMetrics(cfg.metrics.enabled, cfg.metrics.port)
    rt = build_backend(cfg, metrics)
    backend, engine, tp = rt.backend, rt.engine, rt.tp
    if not rt.is_control_rank:
        rt.serve()   # follow rank 0 until it shuts down
        return 0
    metrics.start()
    print(f" AI-Powered Kubernetes Scheduler with {cfg.llm.model.split('/')[-1]}")
    print("=" * 60)
    if engine is not None:
        print(f"Local decision engine: {cfg.engine.preset} on MI355X, TP={tp.world if tp else 1}"
              + (f" x {tp.replicas} replicas" if tp is not None and tp.replicas > 1 else ""))
    else:
        print(f"Decision backend: {cfg.engine.backend if cfg.engine.enabled else 'disabled (fallback only)'}")
    print(f"Model: {cfg.llm.model}")
    print("=" * 60)
    if args.fake_cluster:
        api = _fake_cluster(args.fake_cluster)
    else:
        from .kube.rest import KubeConnection, RestKubeAPI

        api = RestKubeAPI(KubeConnection.auto(args.kubeconfig))
    sched = build_scheduler(cfg, api, backend, metrics)

    async def main():
        task = asyncio.create_task(sched.start())
        if args.fake_cluster and args.demo_pods:
            await asyncio.sleep(0.2)
            api.apply_manifest(TEST_PODS.read_text())
        if args.duration:
            await asyncio.sleep(args.duration)
            sched.stop()
        await task

    try:
        print("\n Scheduler initialized successfully!")
        print(f" Watching for pods with schedulerName={cfg.scheduler.name}")
        print("\nPress Ctrl+C to stop...\n")
        asyncio.run(main())
    except KeyboardInterrupt:
        print("\n\n⏹  Scheduler stopped by user")
    finally:
        sched.stop()
        rt.shutdown()
        print_final_stats(sched.get_stats())
    return 0


def cmd_verify(args, cfg: Config) -> int:
    ok = True

    def check(label: str, good: bool, detail: str = "", required: bool = True) -> None:
        nonlocal ok
        mark = "ok " if good else ("FAIL" if required else "warn")
        print(f"[{mark}] {label}{(': ' + detail) if detail else ''}")
        if required and not good:
            ok = False

    print(" MI355X LLM scheduler - setup verification\n" + "=" * 60)
    check("config", True, cfg.source or "built-in defaults")
    check("examples/ai-test-pods.yaml", TEST_PODS.is_file())
    for mod in ("torch", "yaml", "tokenizers", "safetensors", "requests", "prometheus_client"):
        try:
            __import__(mod)
            check(f"python package {mod}", True)
        except Exception as e:  # noqa: BLE001
            check(f"python package {mod}", False, str(e))
    try:
        import torch

        from . import ops

        n = torch.cuda.device_count()
        check("GPUs visible", n > 0, f"{n}", required=cfg.engine.enabled and cfg.engine.backend == "local")
        ops.native()
        check("native HIP extension (_C, gfx950)", True)
        if n and torch.cuda.is_available():
            p = torch.cuda.get_device_properties(0)
            check("device", "gfx950" in getattr(p, "gcnArchName", ""), f"{p.name} {getattr(p, 'gcnArchName', '')}",
                  required=False)
    except Exception as e:  # noqa: BLE001
        check("native HIP extension (_C, gfx950)", False, f"{e}  (run: python -m k8s_llm_scheduler_amd._build)")
    if args.fake_cluster:
        check("cluster", True, f"in-memory fake with {args.fake_cluster} nodes")
    else:
        try:
            from .kube.rest import KubeConnection, RestKubeAPI

            nodes = RestKubeAPI(KubeConnection.auto(args.kubeconfig)).list_nodes()
            check("Kubernetes connection", True, f"{len(nodes)} nodes")
        except Exception as e:  # noqa: BLE001
            check("Kubernetes connection", False, f"{e}  (e.g. kind create cluster --config 3-nodes.yaml)")
    print("=" * 60 + ("\n All checks passed." if ok else "\n Some checks failed."))
    return 0 if ok else 1


def cmd_smoke(args, cfg: Config) -> int:
    """test_runner.py semantics: (re)create the 3 test pods, wait, report how many got a node."""
    import yaml

    docs = [d for d in yaml.safe_load_all(TEST_PODS.read_text()) if d]
    pods = [it for d in docs for it in (d.get("items", []) if d.get("kind") == "List" else [d])]
    if args.fake_cluster:
        api = _fake_cluster(args.fake_cluster)
        backend = build_backend(cfg).backend if cfg.engine.backend != "local" or args.with_engine else None
        sched = build_scheduler(cfg, api, backend)

        async def run():
            task = asyncio.create_task(sched.start())
            await asyncio.sleep(0.1)
            for p in pods:
                api.create_pod(p)
            t0 = time.time()
            while time.time() - t0 < args.wait:
                if all(api.get_pod("default", p["metadata"]["name"])["spec"].get("nodeName") for p in pods):
                    break
                await asyncio.sleep(0.05)
            sched.stop()
            await asyncio.wait_for(task, 10)

        asyncio.run(run())
        get = lambda n: api.get_pod("default", n)
    else:
        from .kube.rest import KubeConnection, RestKubeAPI

        api = RestKubeAPI(KubeConnection.auto(args.kubeconfig))
        for p in pods:
            api.delete_pod("default", p["metadata"]["name"])
        time.sleep(2)
        for p in pods:
            api.create_pod(p)
        print(f"\n Waiting for pods to be scheduled ({args.wait:.0f} seconds)...")
        time.sleep(args.wait)
        get = lambda n: api.get_pod("default", n)
    print("\n Pod Status:\n" + "-" * 60)
    bound = 0
    for p in pods:
        name = p["metadata"]["name"]
        cur = get(name) or {}
        node = (cur.get("spec") or {}).get("nodeName")
        bound += bool(node)
        print(f"{name:20} | Status: {(cur.get('status') or {}).get('phase', '?'):10} | Node: {node or 'Not scheduled'}")
    print("-" * 60 + f"\n Results: {bound}/{len(pods)} pods scheduled")
    return 0 if bound == len(pods) else 1


def main(argv: Optional[list] = None) -> int:
    ap = argparse.ArgumentParser(prog="k8s_llm_scheduler_amd", description=__doc__.splitlines()[0])
    ap.add_argument("command", nargs="?", default="run", choices=["run", "verify", "smoke"])
    ap.add_argument("--config", default=None, help="config.yaml (default: $SCHEDULER_CONFIG or ./config.yaml)")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--fake-cluster", type=int, default=0, metavar="N",
                    help="use an in-memory cluster of N kind-worker nodes instead of an apiserver")
    ap.add_argument("--demo-pods", action="store_true", help="(run --fake-cluster) submit ai-test-pods.yaml")
    ap.add_argument("--duration", type=float, default=0.0, help="(run) stop after N seconds")
    ap.add_argument("--backend", choices=["local", "fallback", "scripted"], default=None)
    ap.add_argument("--preset", default=None)
    ap.add_argument("--wait", type=float, default=30.0, help="(smoke) seconds to wait (test_runner.py: 30)")
    ap.add_argument("--with-engine", action="store_true", help="(smoke --fake-cluster) build the GPU engine")
    args = ap.parse_args(argv)
    load_dotenv()
    cfg = load_config(args.config)
    if args.backend:
        cfg.engine.backend = args.backend
    if args.preset:
        cfg.engine.preset = args.preset
    from .utils.logging import setup_logging

    setup_logging(cfg.logging.level, cfg.logging.format, cfg.logging.file)
    return {"run": cmd_run, "verify": cmd_verify, "smoke": cmd_smoke}[args.command](args, cfg)


if __name__ == "__main__":
    sys.exit(main())
