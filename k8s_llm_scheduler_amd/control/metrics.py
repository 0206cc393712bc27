"""Prometheus metrics (``metrics.enabled`` / ``metrics.port``, ``config.yaml:29-31``).

The reference advertises metrics (``README.md:173-184``) but never starts a server.  Here the
same counters as the reference's stats dicts (``scheduler.py:344-351``, ``:635-640``) are exported,
plus engine gauges: decision latency histogram, engine-call latency, tokens generated, batch size
and KV-cache utilisation.  Each instance owns a private registry so tests can build many.

The same port serves the Kubernetes probes (the reference has none):
``/healthz`` (liveness: 200 while the process serves; 503 once a health source reports it dead, e.g. the
engine loop thread died) and ``/readyz`` (readiness: 200 only while the decision engine is ready -- a stalled
or failed collective turns it 503 until the engine recovers; the body says why).
"""

from __future__ import annotations

import json
import logging
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, Optional, Tuple

log = logging.getLogger(__name__)

try:
    from prometheus_client import CONTENT_TYPE_LATEST, CollectorRegistry, Counter, Gauge, Histogram, generate_latest
    _HAVE_PROM = True
except Exception:  # pragma: no cover - prometheus_client is installed in this image
    _HAVE_PROM = False

_LAT_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0, 60.0)


HealthFn = Callable[[], Tuple[bool, bool, dict]]   # -> (live, ready, detail)


class SchedulerMetrics:
    def __init__(self, enabled: bool = True, port: Optional[int] = None):
        self.enabled = enabled and _HAVE_PROM
        self.port = port
        self.server_started = False
        self._health: Dict[str, HealthFn] = {}
        self._server: Optional[ThreadingHTTPServer] = None
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
        self.ready_gauge = Gauge("engine_ready", "1 while the decision engine is ready", registry=r)
        self.ready_gauge.set(1)

    # ---- probes
    def add_health_source(self, name: str, fn: HealthFn) -> None:
        """Register a component whose (live, ready, detail) feeds /healthz and /readyz."""
        self._health[name] = fn

    def health(self) -> Tuple[bool, bool, dict]:
        live, ready, detail = True, True, {}
        for name, fn in list(self._health.items()):
            try:
                lv, rd, d = fn()
            except Exception as e:  # noqa: BLE001 -- a broken source is reported, not raised
                lv, rd, d = True, False, {"error": repr(e)}
            live, ready = live and lv, ready and rd
            detail[name] = dict(d, live=lv, ready=rd)
        return live, ready, detail

    def engine_health(self, ready: bool) -> None:
        if self.enabled:
            self.ready_gauge.set(1 if ready else 0)

    def start(self) -> None:
        if self.port and not self.server_started:
            try:
                self._server = ThreadingHTTPServer(("", int(self.port)), _handler(self))
            except OSError as e:
                log.warning(f"metrics / probe server not started: {e}")
                return
            self._server.daemon_threads = True
            threading.Thread(target=self._server.serve_forever, name="metrics-http", daemon=True).start()
            self.server_started = True
            log.info(f" Metrics on :{self.port}/metrics, probes on /healthz and /readyz")

    def stop(self) -> None:
        if self._server is not None:
            self._server.shutdown()
            self._server.server_close()
            self._server = None
            self.server_started = False

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


def _handler(m: "SchedulerMetrics"):
    class H(BaseHTTPRequestHandler):
        def _send(self, code: int, body: bytes, ctype: str) -> None:
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_GET(self):  # noqa: N802 -- http.server API
            path = self.path.split("?", 1)[0]
            if path in ("/healthz", "/readyz"):
                live, ready, detail = m.health()
                ok = live if path == "/healthz" else (live and ready)
                body = json.dumps({"status": "ok" if ok else "unavailable", "live": live, "ready": ready,
                                   "components": detail}).encode()
                self._send(200 if ok else 503, body, "application/json")
            elif path == "/metrics" and m.enabled:
                self._send(200, generate_latest(m.registry), CONTENT_TYPE_LATEST)
            else:
                self._send(404, b"not found\n", "text/plain")

        def log_message(self, *args):  # keep probes out of the scheduler log
            pass

    return H
