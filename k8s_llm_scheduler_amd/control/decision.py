"""Decision service: cache -> circuit breaker -> retries -> engine -> JSON -> validation -> fallback.

Reference: ``HuggingFaceClient`` (``scheduler.py:337-563``).  Behaviour kept:

* cache lookup first; a hit increments ``cached_requests`` and returns (``:380-385``),
* ``total_requests`` counts cache misses (``:387``),
* up to ``llm.max_retries`` attempts, each through the breaker (``:390-395``); between attempts
  the caller sleeps ``retry_delay ** attempt`` seconds (reference: ``2 ** attempt`` with the
  default ``retry_delay`` of 2, ``:409-412``),
* an OPEN breaker returns the fallback immediately and counts ``circuit_breaker_trips``
  (``:404-407``); the last failed attempt counts ``failed_requests`` and falls back (``:413-416``),
* only non-fallback decisions are cached (``:398-399``),
* the model output goes through :func:`extract_json`; a valid ``selected_node`` yields an LLM
  decision (confidence default 0.8, reasoning default "LLM decision", ``:456-462``); an
  unknown node -> fallback "Invalid node selected"; no JSON -> fallback "JSON parsing failed"
  (``:463-468``).  Both of those *return* (the breaker counts them as successes, quirk 6).

Fixed (documented in docs/COMPAT.md): ``max_retries <= 0`` falls back instead of returning
``None`` (quirk 13); a non-numeric ``confidence`` is replaced by 0.8 instead of crashing the log
line (quirk 14); ``avg_response_time`` is the mean over completed engine calls (quirk 7); the
engine call has a real deadline (``llm.timeout``); decisions can be made for a *batch* of pods in
one engine call (continuous batching), with the same per-pod semantics.
"""

from __future__ import annotations

import logging
import threading
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Protocol, Sequence, Tuple

from .breaker import CircuitBreaker, CircuitOpenError
from .cache import DecisionCache
from .fallback import FallbackPolicy
from .jsonextract import extract_json
from .models import NodeMetrics, PodSpec, SchedulingDecision

log = logging.getLogger(__name__)

DEFAULT_LLM_CONFIDENCE = 0.8


@dataclass
class GenerationRequest:
    system: str
    user: str
    max_tokens: int = 200
    temperature: float = 0.3
    top_p: float = 1.0
    deadline_s: Optional[float] = None


class DecisionBackend(Protocol):
    """Anything that turns chat requests into completion texts (raises on failure)."""

    name: str

    def complete(self, requests: Sequence[GenerationRequest]) -> List[str]:
        ...


Item = Tuple[str, PodSpec, Sequence[NodeMetrics]]   # (prompt, pod, node snapshot)


class DecisionService:
    def __init__(self, backend: Optional[DecisionBackend], *, max_retries: int = 3,
                 retry_delay: float = 2.0, max_tokens: int = 200, temperature: float = 0.3,
                 top_p: float = 1.0, timeout: Optional[float] = 60.0,
                 system_message: str = "You are an intelligent Kubernetes scheduler. Respond only with valid JSON.",
                 cache: Optional[DecisionCache] = None, breaker: Optional[CircuitBreaker] = None,
                 fallback: Optional[FallbackPolicy] = None,
                 sleep: Callable[[float], None] = time.sleep,
                 clock: Callable[[], float] = time.perf_counter,
                 metrics=None):
        self.backend = backend
        self.max_retries = int(max_retries)
        self.retry_delay = float(retry_delay)
        self.max_tokens = int(max_tokens)
        self.temperature = float(temperature)
        self.top_p = float(top_p)
        self.timeout = timeout
        self.system_message = system_message
        self.cache = cache
        self.circuit_breaker = breaker
        self.fallback = fallback or FallbackPolicy()
        self._sleep = sleep
        self._clock = clock
        self.metrics = metrics
        self._lock = threading.Lock()
        self._calls = 0
        # Same six keys as scheduler.py:344-351.
        self.stats = {
            "total_requests": 0,
            "successful_requests": 0,
            "failed_requests": 0,
            "cached_requests": 0,
            "avg_response_time": 0.0,
            "circuit_breaker_trips": 0,
        }

    @classmethod
    def from_config(cls, cfg, backend: Optional[DecisionBackend], metrics=None, **kw) -> "DecisionService":
        cache = (DecisionCache(cfg.cache.ttl, cfg.cache.max_size) if cfg.cache.enabled else None)
        breaker = (CircuitBreaker(cfg.circuit_breaker.failure_threshold, cfg.circuit_breaker.timeout,
                                  cfg.circuit_breaker.half_open_max_calls,
                                  cumulative_failures=cfg.compat.breaker_cumulative_failures)
                   if cfg.circuit_breaker.enabled else None)
        fb = FallbackPolicy(cfg.fallback.strategy, cfg.compat.round_robin_picks_most_pods)
        return cls(backend, max_retries=cfg.llm.max_retries, retry_delay=cfg.llm.retry_delay,
                   max_tokens=cfg.llm.max_tokens, temperature=cfg.llm.temperature, top_p=cfg.llm.top_p,
                   timeout=cfg.llm.timeout, system_message=cfg.llm.system_message,
                   cache=cache, breaker=breaker, fallback=fb, metrics=metrics, **kw)

    # ------------------------------------------------------------------ public API
    def get_scheduling_decision(self, prompt: str, pod: PodSpec,
                                nodes: Sequence[NodeMetrics]) -> SchedulingDecision:
        return self.decide_many([(prompt, pod, nodes)])[0]

    decide = get_scheduling_decision

    def get_stats(self) -> dict:
        with self._lock:
            return dict(self.stats)

    def decide_many(self, items: Sequence[Item]) -> List[SchedulingDecision]:
        results: List[Optional[SchedulingDecision]] = [None] * len(items)
        misses: List[int] = []
        for i, (_, pod, nodes) in enumerate(items):
            hit = self.cache.get(pod, nodes) if self.cache is not None else None
            if hit is not None:
                self._bump("cached_requests")
                log.info(" Using cached decision")
                results[i] = hit
            else:
                misses.append(i)
        if not misses:
            return results  # type: ignore[return-value]
        self._bump("total_requests", len(misses))

        if self.backend is None:
            for i in misses:
                results[i] = self.fallback.decide(items[i][2], "LLM disabled")
            return results  # type: ignore[return-value]
        if self.max_retries <= 0:
            for i in misses:
                results[i] = self.fallback.decide(items[i][2], "LLM disabled (max_retries=0)")
            return results  # type: ignore[return-value]

        batch = [items[i] for i in misses]
        for attempt in range(self.max_retries):
            try:
                if self.circuit_breaker is not None:
                    decided = self.circuit_breaker.call(self._call_engine, batch)
                else:
                    decided = self._call_engine(batch)
                for i, d in zip(misses, decided):
                    if self.cache is not None and not d.fallback_needed:
                        self.cache.set(items[i][1], items[i][2], d)
                    results[i] = d
                return results  # type: ignore[return-value]
            except CircuitOpenError:
                self._bump("circuit_breaker_trips", len(misses))
                log.warning(" Circuit breaker is OPEN, using fallback")
                for i in misses:
                    results[i] = self.fallback.decide(items[i][2], "Circuit breaker open")
                return results  # type: ignore[return-value]
            except Exception as e:  # engine/transport failure
                if attempt < self.max_retries - 1:
                    wait = self.retry_delay ** attempt
                    log.warning(f"Attempt {attempt + 1} failed, retrying in {wait:g}s: {e}")
                    self._sleep(wait)
                else:
                    log.error(f"All {self.max_retries} attempts failed: {e}")
                    self._bump("failed_requests", len(misses))
                    for i in misses:
                        results[i] = self.fallback.decide(items[i][2], f"All retries failed: {e}")
                    return results  # type: ignore[return-value]
        raise AssertionError("unreachable")

    # ------------------------------------------------------------------ internals
    def _bump(self, key: str, n: int = 1) -> None:
        with self._lock:
            self.stats[key] += n
        if self.metrics is not None:
            self.metrics.llm_event(key, n)

    def _call_engine(self, batch: Sequence[Item]) -> List[SchedulingDecision]:
        """One engine call for a batch (the reference's _make_api_call, scheduler.py:418-472)."""
        reqs = [GenerationRequest(self.system_message, prompt, self.max_tokens, self.temperature,
                                  self.top_p, self.timeout) for prompt, _, _ in batch]
        t0 = self._clock()
        try:
            texts = self.backend.complete(reqs)
        except Exception as e:
            log.error(f"Error calling local decision engine: {e}")
            raise
        dt = self._clock() - t0
        with self._lock:
            self._calls += 1
            avg = self.stats["avg_response_time"]
            self.stats["avg_response_time"] = avg + (dt - avg) / self._calls
        if self.metrics is not None:
            self.metrics.observe_engine_latency(dt, len(batch))
        if len(texts) != len(batch):
            raise RuntimeError(f"backend returned {len(texts)} completions for {len(batch)} requests")
        return [self._validate(text, nodes) for text, (_, _, nodes) in zip(texts, batch)]

    def _validate(self, text: str, nodes: Sequence[NodeMetrics]) -> SchedulingDecision:
        log.debug(f"LLM Response: {text}")
        data = extract_json(text)
        if not isinstance(data, dict) or not data:
            log.error("Could not parse JSON from LLM response")
            return self.fallback.decide(nodes, "JSON parsing failed")
        selected = data.get("selected_node", "")
        if isinstance(selected, str) and selected in [n.name for n in nodes]:
            self._bump("successful_requests")
            conf = data.get("confidence", DEFAULT_LLM_CONFIDENCE)
            try:
                conf = float(conf)
            except (TypeError, ValueError):
                conf = DEFAULT_LLM_CONFIDENCE
            reasoning = data.get("reasoning", "LLM decision")
            return SchedulingDecision(selected, conf, str(reasoning), False)
        log.warning(f"LLM selected invalid node: {selected}")
        return self.fallback.decide(nodes, "Invalid node selected")
