"""Scheduler orchestration: watch -> snapshot -> prompt -> decide -> bind.

Reference: ``CustomScheduler`` (``scheduler.py:625-770``).  Kept: the pending-pod filter
(``phase == Pending`` and ``schedulerName`` matches and no ``nodeName``, ``:674-676``), the
per-pod pipeline and its log lines (``:690-729``), the four stats keys plus the nested decision
stats (``:635-640``, ``:766-770``), the 5 s back-off after a watch error (``:683-685``) and the
re-list on every re-stream, which is the only requeue mechanism for pods that failed to bind
(``:662-667``, quirk 9).

Changed (docs/COMPAT.md):

* The watch stream runs in a thread and the decision pipeline in an executor, so nothing blocks
  the event loop (the reference's awaits never yield, quirk 10).
* DELETED events are ignored and pods are de-duplicated by UID while in flight and after a
  successful bind (quirk 8: duplicate events double-bind and get 409).  Set
  ``compat.watch_all_event_types`` to restore the reference filter.
* ``scheduler.mode: continuous`` hands every detected pod to a worker at once (up to ``max_batch``
  in flight); the engine runs in its background loop, so each decision joins the running decode
  batch at the next engine step and is bound as soon as it is done (re-validated against the
  current node counts).
* ``scheduler.mode: batched`` drains up to ``max_batch`` pending pods and decides them in ONE
  engine call (continuous batching on the GPU).  All pods of a round see the same snapshot;
  bindings are applied in order and each is re-validated against the snapshot updated with
  the previous bindings of the round (a node at its pod limit falls back per pod).
"""

from __future__ import annotations

import asyncio
import collections
import concurrent.futures
import logging
import threading
import time
from typing import Deque, Dict, List, Optional, Sequence, Set

from ..kube.api import KubeAPI, Obj, pod_key, pod_uid
from .binder import IntegrationLayer
from .cluster import ClusterSnapshotter, apply_assumed_binding, find_node, pod_to_spec
from .decision import DecisionService
from .models import NodeMetrics, SchedulingDecision
from .prompt import PromptEngine

log = logging.getLogger(__name__)


def start_backend_loop(backend) -> bool:
    """Put the decision engine behind ``backend`` (possibly wrapped, e.g. by FaultInjectingBackend) in
    background-loop mode, so concurrent decisions share engine steps.  False if there is none."""
    while backend is not None:
        eng = getattr(backend, "engine", None)
        if eng is not None and hasattr(eng, "start_background"):
            eng.start_background()
            return True
        backend = getattr(backend, "inner", None)
    return False


class CustomScheduler:
    def __init__(self, name: str, api: KubeAPI, decision_service: DecisionService, *,
                 snapshot_mode: str = "informer", quantity_mode: str = "full",
                 status_always_ready: bool = True, watch_all_event_types: bool = False,
                 mode: str = "sequential", max_batch: int = 64, batch_window_ms: float = 20.0,
                 watch_timeout: int = 60, error_backoff_s: float = 5.0,
                 engine_label: str = "local Llama-3.3-70B", metrics=None, prompt_layout: str = "reference"):
        self.scheduler_name = name
        self.api = api
        self.context_manager = ClusterSnapshotter(api, snapshot_mode, quantity_mode)
        self.prompt_engine = PromptEngine(status_always_ready, layout=prompt_layout)
        self.llm_client = decision_service
        self.integration_layer = IntegrationLayer(api)
        self.qmode = quantity_mode
        self.watch_all = watch_all_event_types
        self.mode = mode
        self.max_batch = max(1, int(max_batch))
        self.batch_window = batch_window_ms / 1000.0
        self.watch_timeout = watch_timeout
        self.error_backoff_s = error_backoff_s
        self.engine_label = engine_label
        self.metrics = metrics
        self.running = False
        self._lock = threading.Lock()
        self._inflight: Set[str] = set()
        self._bound: "collections.OrderedDict[str, None]" = collections.OrderedDict()
        self._bind_lock = threading.Lock()
        self._pool: Optional[concurrent.futures.ThreadPoolExecutor] = None
        self.decision_latencies: Deque[float] = collections.deque(maxlen=100000)
        self.stats = {"total_scheduled": 0, "llm_decisions": 0, "fallback_decisions": 0, "failed_bindings": 0}

    @classmethod
    def from_config(cls, cfg, api: KubeAPI, decision_service: DecisionService, metrics=None,
                    engine_label: Optional[str] = None) -> "CustomScheduler":
        label = f"local {cfg.llm.model.split('/')[-1].replace('-Instruct', '')}"
        eng = getattr(cfg, "engine", None)
        if eng is not None and eng.backend == "local" and "70b" not in eng.preset.lower():
            label = f"local {eng.preset}"  # the served model, not the config's llm.model
        label = engine_label or label
        return cls(cfg.scheduler.name, api, decision_service,
                   snapshot_mode=cfg.compat.snapshot_mode, quantity_mode=cfg.compat.quantity_parsing,
                   status_always_ready=cfg.compat.prompt_status_always_ready,
                   watch_all_event_types=cfg.compat.watch_all_event_types,
                   mode=cfg.scheduler.mode, max_batch=cfg.scheduler.max_batch,
                   batch_window_ms=cfg.scheduler.batch_window_ms,
                   watch_timeout=cfg.scheduler.watch_interval, error_backoff_s=cfg.scheduler.error_backoff_s,
                   engine_label=label, metrics=metrics, prompt_layout=cfg.compat.prompt_layout)

    # ------------------------------------------------------------------ lifecycle
    async def start(self) -> None:
        self.running = True
        if self.mode == "continuous":
            start_backend_loop(self.llm_client.backend)
        log.info(f" Starting {self.scheduler_name}...")
        log.info(f" Watching for pods with schedulerName={self.scheduler_name}")
        await self._watch_pods()

    def stop(self) -> None:
        self.running = False
        if self._pool is not None:
            self._pool.shutdown(wait=False)
        stopper = getattr(self.api, "stop_watches", None)
        if stopper:
            stopper()
        log.info("⏹  Scheduler stopped")

    def get_stats(self) -> Dict:
        with self._lock:
            stats = dict(self.stats)
        stats["llm_client"] = self.llm_client.get_stats()
        return stats

    # ------------------------------------------------------------------ filtering
    def wants(self, event_type: str, pod: Obj) -> bool:
        spec, status = pod.get("spec") or {}, pod.get("status") or {}
        if not (status.get("phase") == "Pending" and spec.get("schedulerName") == self.scheduler_name
                and not spec.get("nodeName")):
            return False
        if self.watch_all:
            return True
        if event_type == "DELETED":
            return False
        uid = pod_uid(pod)
        with self._lock:
            return uid not in self._inflight and uid not in self._bound

    def _claim(self, pod: Obj) -> bool:
        uid = pod_uid(pod)
        with self._lock:
            if not self.watch_all and (uid in self._inflight or uid in self._bound):
                return False
            self._inflight.add(uid)
            return True

    def _release(self, pod: Obj, bound: bool) -> None:
        uid = pod_uid(pod)
        with self._lock:
            self._inflight.discard(uid)
            if bound:
                self._bound[uid] = None
                while len(self._bound) > 100000:
                    self._bound.popitem(last=False)

    # ------------------------------------------------------------------ watch loop
    def _watch_thread(self, loop: asyncio.AbstractEventLoop, q: "asyncio.Queue") -> None:
        """LIST + WATCH: every (re)stream starts with one LIST, handed to the consumer as a SYNC
        event (informer counts are rebuilt from it and every listed pod is considered as the
        reference's re-stream would, quirk 9), then watches from that LIST's resourceVersion."""
        while self.running:
            try:
                pods, rv = self.api.list_pods()
                loop.call_soon_threadsafe(q.put_nowait, ("SYNC", pods))
                for ev in self.api.watch_pods(rv or None, timeout_seconds=self.watch_timeout):
                    if not self.running:
                        break
                    loop.call_soon_threadsafe(q.put_nowait, ev)
            except Exception as e:  # noqa: BLE001
                log.error(f"Watch error: {e}")
                deadline = time.monotonic() + self.error_backoff_s
                while self.running and time.monotonic() < deadline:
                    time.sleep(0.05)
        loop.call_soon_threadsafe(q.put_nowait, None)

    async def _watch_pods(self) -> None:
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        t = threading.Thread(target=self._watch_thread, args=(loop, q), name="pod-watch", daemon=True)
        t.start()
        log.info(" Watching for unscheduled pods...")
        pending: Deque = collections.deque()

        async def next_event(timeout: Optional[float] = None):
            """Next pod event in stream order (SYNC lists expand to ADDED events); "TIMEOUT" or None
            (stream closed)."""
            while not pending:
                try:
                    ev = await (asyncio.wait_for(q.get(), timeout) if timeout is not None else q.get())
                except asyncio.TimeoutError:
                    return "TIMEOUT"
                if ev is None:
                    return None
                typ, obj = ev
                if typ == "SYNC":
                    self.context_manager.resync(obj)
                    pending.extend(("ADDED", p) for p in obj)
                else:
                    self.context_manager.observe(typ, obj)
                    pending.append(ev)
            return pending.popleft()

        inflight: Set["asyncio.Future"] = set()
        slots = asyncio.Semaphore(self.max_batch)
        try:
            while self.running:
                ev = await next_event()
                if ev is None:
                    break
                typ, pod = ev
                if not self.wants(typ, pod):
                    continue
                if self.mode == "continuous":
                    await self._dispatch(loop, pod, inflight, slots)
                elif self.mode == "batched":
                    batch = [pod]
                    deadline = loop.time() + self.batch_window
                    while len(batch) < self.max_batch:
                        left = deadline - loop.time()
                        if left <= 0:
                            break
                        nxt = await next_event(left)
                        if nxt == "TIMEOUT":
                            break
                        if nxt is None:
                            self.running = False
                            break
                        if self.wants(*nxt) and all(pod_uid(nxt[1]) != pod_uid(b) for b in batch):
                            batch.append(nxt[1])
                    await loop.run_in_executor(None, self.schedule_batch, batch)
                else:
                    log.info(f"\n{'=' * 60}")
                    log.info(f" Detected pod: {pod['metadata'].get('namespace')}/{pod['metadata'].get('name')}")
                    await loop.run_in_executor(None, self.schedule_pod, pod)
                    log.info(f"{'=' * 60}\n")
        finally:
            self.running = False
            if inflight:
                await asyncio.gather(*inflight, return_exceptions=True)

    async def _dispatch(self, loop, pod: Obj, inflight: Set["asyncio.Future"], slots: asyncio.Semaphore) -> None:
        """Continuous mode: claim the pod now (duplicates of it are dropped from here on) and run its
        pipeline on a worker thread; up to ``max_batch`` decisions are in the engine at once and the
        engine's background loop batches them step by step."""
        if not self._claim(pod):
            return
        t_detect = time.perf_counter()
        log.info(f" Detected pod: {pod['metadata'].get('namespace')}/{pod['metadata'].get('name')}")
        await slots.acquire()
        if self._pool is None:
            self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=self.max_batch,
                                                               thread_name_prefix="decide")
        fut = loop.run_in_executor(self._pool, self._schedule_claimed, pod, t_detect, True)
        inflight.add(fut)

        def _done(f):
            inflight.discard(f)
            slots.release()

        fut.add_done_callback(_done)

    # ------------------------------------------------------------------ pipelines
    def _record(self, decision: SchedulingDecision, t0: float) -> None:
        dt = time.perf_counter() - t0
        self.decision_latencies.append(dt)
        with self._lock:
            key = "fallback_decisions" if decision.fallback_needed else "llm_decisions"
            self.stats[key] += 1
        if decision.fallback_needed:
            log.warning(f"  Using fallback: {decision.reasoning}")
        else:
            log.info(f" LLM decision: {decision.selected_node} (confidence: {decision.confidence:.2f})")
        log.info(f" Reasoning: {decision.reasoning}")
        if self.metrics is not None:
            self.metrics.decision("fallback" if decision.fallback_needed else "llm", dt)

    def _bind(self, pod: Obj, decision: SchedulingDecision) -> bool:
        md = pod["metadata"]
        ok = False
        if decision.selected_node:
            ok = self.integration_layer.bind_pod_to_node(md["name"], md.get("namespace", "default"),
                                                         decision.selected_node)
            if ok:
                self.context_manager.assume(pod_key(pod), decision.selected_node)
        else:
            log.error(" No node selected")
        with self._lock:
            self.stats["total_scheduled" if ok else "failed_bindings"] += 1
        if self.metrics is not None:
            self.metrics.bound(ok)
        return ok

    def schedule_pod(self, pod: Obj) -> Optional[SchedulingDecision]:
        """The reference's per-pod pipeline (scheduler.py:690-729), synchronous."""
        if not self._claim(pod):
            return None
        return self._schedule_claimed(pod, time.perf_counter(), False)

    def _schedule_claimed(self, pod: Obj, t0: float, revalidate: bool) -> Optional[SchedulingDecision]:
        bound = False
        try:
            spec = pod_to_spec(pod, self.qmode)
            nodes = self.context_manager.get_node_metrics()
            if not nodes:
                log.error(" No available nodes")
                return None
            prompt = self.prompt_engine.construct_scheduling_prompt(spec, nodes)
            log.info(f" Calling {self.engine_label} for scheduling decision...")
            decision = self.llm_client.get_scheduling_decision(prompt, spec, nodes)
            if revalidate and decision.selected_node:
                # concurrent decisions saw snapshots taken before each other's bindings: re-check the
                # chosen node against the current counts (which include our own assumed bindings)
                with self._bind_lock:
                    decision = self._revalidate(decision)
                    self._record(decision, t0)
                    bound = self._bind(pod, decision)
                return decision
            self._record(decision, t0)
            bound = self._bind(pod, decision)
            return decision
        finally:
            self._release(pod, bound)

    def _revalidate(self, d: SchedulingDecision) -> SchedulingDecision:
        current = self.context_manager.get_node_metrics()
        target = find_node(current, d.selected_node)
        if target is not None and target.max_pods > 0 and target.pod_count >= target.max_pods:
            return self.llm_client.fallback.decide(
                [n for n in current if n.max_pods == 0 or n.pod_count < n.max_pods],
                f"Node {d.selected_node} full after concurrent bindings")
        return d

    def schedule_batch(self, pods: Sequence[Obj]) -> List[Optional[SchedulingDecision]]:
        """Batched round: one snapshot, one engine call, in-order validated bindings."""
        claimed = [p for p in pods if self._claim(p)]
        results: List[Optional[SchedulingDecision]] = []
        if not claimed:
            return results
        t0 = time.perf_counter()
        bound_flags = [False] * len(claimed)
        try:
            for p in claimed:
                log.info(f" Detected pod: {p['metadata'].get('namespace')}/{p['metadata'].get('name')}")
            nodes = self.context_manager.get_node_metrics()
            if not nodes:
                log.error(" No available nodes")
                return [None] * len(claimed)
            specs = [pod_to_spec(p, self.qmode) for p in claimed]
            items = [(self.prompt_engine.construct_scheduling_prompt(s, nodes), s, nodes) for s in specs]
            log.info(f" Calling {self.engine_label} for {len(items)} scheduling decisions...")
            decisions = self.llm_client.decide_many(items)
            current: List[NodeMetrics] = list(nodes)
            for i, (p, d) in enumerate(zip(claimed, decisions)):
                target = find_node(current, d.selected_node) if d.selected_node else None
                if target is not None and target.max_pods > 0 and target.pod_count >= target.max_pods:
                    d = self.llm_client.fallback.decide(
                        [n for n in current if n.max_pods == 0 or n.pod_count < n.max_pods],
                        f"Node {d.selected_node} full after earlier bindings in this batch")
                self._record(d, t0)
                if self._bind(p, d):
                    bound_flags[i] = True
                    current = apply_assumed_binding(current, d.selected_node)
                results.append(d)
            return results
        finally:
            for p, b in zip(claimed, bound_flags):
                self._release(p, b)
