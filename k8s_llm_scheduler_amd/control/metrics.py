"""Prometheus metrics (``metrics.enabled`` / ``metrics.port``, ``config.yaml:29-31``).

The reference advertises metrics (``README.md:173-184``) but never starts a server.  Here the
same counters as the reference's stats dicts (``scheduler.py:344-351``, ``:635-640``) are exported,
plus engine gauges: decision latency histogram, engine-call latency, tokens generated, batch size
and KV-cache utilisation.  Each instance owns a private registry so tests can build many.
"""

from __future__ import annotations

import logging
from typing import Optional

log = logging.getLogger(__name__)

try:
    from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, start_http_server
    _HAVE_PROM = True
except Exception:  # pragma: no cover - prometheus_client is installed in this image
    _HAVE_PROM = False

_LAT_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0, 60.0)


class SchedulerMetrics:
    def __init__(self, enabled: bool = True, port: Optional[int] = None):
        self.enabled = enabled and _HAVE_PROM
        self.port = port
        self.server_started = False
        if not self.enabled:
            return
        r = self.registry = CollectorRegistry()
        self.scheduled = Counter("scheduler_pods_scheduled_total", "Pods bound", registry=r)
        self.decisions = Counter("scheduler_decisions_total", "Decisions by source", ["source"], registry=r)
        self.failed_bindings = Counter("scheduler_failed_bindings_total", "Failed bindings", registry=r)
        self.llm = Counter("scheduler_llm_events_total", "Decision-service events", ["event"], registry=r)
        self.decision_latency = Histogram("scheduler_decision_latency_seconds",
                                          "Per-pod detect->decision latency", buckets=_LAT_BUCKETS, registry=r)
        self.engine_latency = Histogram("scheduler_engine_call_seconds", "Engine call latency",
                                        buckets=_LAT_BUCKETS, registry=r)
        self.batch_size = Gauge("scheduler_engine_batch_size", "Pods per engine call", registry=r)
        self.tokens = Counter("engine_generated_tokens_total", "Tokens generated", registry=r)
        self.kv_util = Gauge("engine_kv_cache_utilization", "Fraction of KV blocks in use", registry=r)

    def start(self) -> None:
        if self.enabled and self.port and not self.server_started:
            try:
                start_http_server(int(self.port), registry=self.registry)
                self.server_started = True
                log.info(f" Metrics on :{self.port}/metrics")
            except OSError as e:
                log.warning(f"metrics server not started: {e}")

    # hooks used by the control plane
    def llm_event(self, key: str, n: int = 1) -> None:
        if self.enabled:
            self.llm.labels(event=key).inc(n)

    def observe_engine_latency(self, seconds: float, batch: int) -> None:
        if self.enabled:
            self.engine_latency.observe(seconds)
            self.batch_size.set(batch)

    def decision(self, source: str, seconds: float) -> None:
        if self.enabled:
            self.decisions.labels(source=source).inc()
            self.decision_latency.observe(seconds)

    def bound(self, ok: bool) -> None:
        if self.enabled:
            (self.scheduled if ok else self.failed_bindings).inc()

    def engine_tokens(self, n: int, kv_utilization: Optional[float] = None) -> None:
        if self.enabled:
            self.tokens.inc(n)
            if kv_utilization is not None:
                self.kv_util.set(kv_utilization)
