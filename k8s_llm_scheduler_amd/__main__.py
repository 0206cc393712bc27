"""Command line: ``python -m k8s_llm_scheduler_amd [run|verify|smoke|e2e]``.

``run`` is the reference's ``python scheduler.py`` (``scheduler.py:775-823``): banner, build the
scheduler, watch pods until Ctrl+C, print final statistics.  Under ``torchrun`` (one process per
GPU) rank 0 runs the control plane and the decision engine's rank-0 shard; every other rank
follows rank 0's engine schedule (tensor parallel over RCCL).

``verify`` replaces ``verify_setup.py`` (files, env, packages, GPU + native extension, cluster).
``smoke`` replaces ``test_runner.py``: apply the three ai-test-pods, wait, count bound pods --
against a real cluster, or fully in-process with ``--fake`` (no cluster needed).
``e2e`` replaces ``test_e2e.py``: verify, clean up, list nodes, start the scheduler, apply the
test pods, wait 10 s, then require every pod scheduled AND Running.
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
    if engine is not None:
        metrics.add_health_source("engine", engine.health_probe)
    metrics.add_health_source("scheduler", lambda: (True, bool(sched.running), {"stats": sched.get_stats()}))

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


def _test_pods() -> list:
    import yaml

    docs = [d for d in yaml.safe_load_all(TEST_PODS.read_text()) if d]
    return [it for d in docs for it in (d.get("items", []) if d.get("kind") == "List" else [d])]


def cmd_smoke(args, cfg: Config) -> int:
    """test_runner.py semantics: (re)create the 3 test pods, wait, report how many got a node."""
    pods = _test_pods()
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


def cmd_e2e(args, cfg: Config) -> int:
    """test_e2e.py semantics (reference ``test_e2e.py:26-152``) without the human in the loop.

    Steps: 1 verify (exit 1 on failure), 2 delete old test pods, 3 list the cluster's nodes,
    4 start the scheduler -- in this process by default; ``--external-scheduler`` keeps the
    reference's "start it in another terminal, press ENTER" step --, 5 apply the test pods and wait
    ``--wait`` seconds (reference: 10), 6 report phase / node / schedulerName per pod.  Success
    requires every test pod scheduled AND Running, as the reference's final verdict does."""
    bar = "=" * 70
    print(bar + "\n AI Kubernetes Scheduler - End-to-End Test (MI355X decision engine)\n" + bar)
    print("\n Step 1: Verifying setup...")
    if cmd_verify(args, cfg) != 0:
        print(" Setup verification failed. Please fix issues first.")
        return 1
    pods = _test_pods()
    names = [p["metadata"]["name"] for p in pods]
    if args.fake_cluster:
        api = _fake_cluster(args.fake_cluster)
    else:
        from .kube.rest import KubeConnection, RestKubeAPI

        api = RestKubeAPI(KubeConnection.auto(args.kubeconfig))
    print("\n Step 2: Cleaning up existing test pods...")
    for n in names:
        try:
            api.delete_pod("default", n)
        except Exception:  # noqa: BLE001 -- --ignore-not-found
            pass
    print("\n Step 3: Checking Kubernetes cluster...")
    try:
        nodes = api.list_nodes()
    except Exception as e:  # noqa: BLE001
        print(f" Cannot connect to Kubernetes: {e}")
        return 1
    print(f" Cluster has {len(nodes)} nodes:")
    for nd in nodes:
        print(f"   - {nd['metadata']['name']}")

    print("\n" + bar + "\n Step 4: Start the Scheduler\n" + bar)
    wait = args.wait if args.wait_set else 10.0

    def apply_and_wait():
        print("\n Step 5: Creating test pods...")
        for p in pods:
            api.create_pod(p)
        print(f"\n Waiting {wait:.0f} seconds for scheduling...")

    if args.external_scheduler:
        print("\n Start the scheduler in another terminal: python scheduler.py (wait for 'Watching for pods')")
        input("\n Press ENTER when the scheduler is running...")
        apply_and_wait()
        time.sleep(wait)
    else:
        rt = build_backend(cfg) if cfg.engine.backend != "local" or args.with_engine else None
        sched = build_scheduler(cfg, api, rt.backend if rt else None)
        print(" scheduler started in-process (schedulerName "
              f"{cfg.scheduler.name}, backend {cfg.engine.backend if rt else 'fallback'})")

        async def run():
            task = asyncio.create_task(sched.start())
            await asyncio.sleep(0.1)
            apply_and_wait()
            t0 = time.time()
            while time.time() - t0 < wait:
                cur = [api.get_pod("default", n) or {} for n in names]
                if all((c.get("status") or {}).get("phase") == "Running" for c in cur):
                    break
                await asyncio.sleep(0.05)
            sched.stop()
            await asyncio.wait_for(task, 10)

        try:
            asyncio.run(run())
        finally:
            if rt is not None:
                rt.shutdown()

    print("\n Step 6: Checking pod status...\n" + "-" * 70)
    print(f"{'POD NAME':<20} {'STATUS':<12} {'NODE':<20} SCHEDULER")
    print("-" * 70)
    scheduled = running = 0
    for n in names:
        cur = api.get_pod("default", n) or {}
        spec, phase = cur.get("spec") or {}, (cur.get("status") or {}).get("phase", "?")
        scheduled += bool(spec.get("nodeName"))
        running += phase == "Running"
        print(f"{n:<20} {phase:<12} {spec.get('nodeName') or 'Not scheduled':<20} {spec.get('schedulerName', '')}")
    print("-" * 70 + f"\n Results:\n   - Scheduled: {scheduled}/{len(names)} pods\n"
          f"   - Running:   {running}/{len(names)} pods")
    ok = scheduled == running == len(names)
    print("\n" + bar + ("\n SUCCESS! All pods scheduled and running!" if ok else
                        "\n FAILED: not every test pod was scheduled and running.") + "\n" + bar)
    return 0 if ok else 1


def main(argv: Optional[list] = None) -> int:
    ap = argparse.ArgumentParser(prog="k8s_llm_scheduler_amd", description=__doc__.splitlines()[0])
    ap.add_argument("command", nargs="?", default="run", choices=["run", "verify", "smoke", "e2e"])
    ap.add_argument("--config", default=None, help="config.yaml (default: $SCHEDULER_CONFIG or ./config.yaml)")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--fake-cluster", type=int, default=0, metavar="N",
                    help="use an in-memory cluster of N kind-worker nodes instead of an apiserver")
    ap.add_argument("--demo-pods", action="store_true", help="(run --fake-cluster) submit ai-test-pods.yaml")
    ap.add_argument("--duration", type=float, default=0.0, help="(run) stop after N seconds")
    ap.add_argument("--backend", choices=["local", "fallback", "scripted"], default=None)
    ap.add_argument("--preset", default=None)
    ap.add_argument("--wait", type=float, default=None,
                    help="seconds to wait for scheduling (smoke: 30 as test_runner.py, e2e: 10 as test_e2e.py)")
    ap.add_argument("--external-scheduler", action="store_true",
                    help="(e2e) the scheduler runs elsewhere: wait for ENTER like test_e2e.py instead of starting it")
    ap.add_argument("--with-engine", action="store_true", help="(smoke --fake-cluster) build the GPU engine")
    args = ap.parse_args(argv)
    args.wait_set = args.wait is not None
    if args.wait is None:
        args.wait = 30.0
    load_dotenv()
    cfg = load_config(args.config)
    if args.backend:
        cfg.engine.backend = args.backend
    if args.preset:
        cfg.engine.preset = args.preset
    from .utils.logging import setup_logging

    setup_logging(cfg.logging.level, cfg.logging.format, cfg.logging.file)
    return {"run": cmd_run, "verify": cmd_verify, "smoke": cmd_smoke, "e2e": cmd_e2e}[args.command](args, cfg)


if __name__ == "__main__":
    sys.exit(main())
