"""Heuristic fallback when the LLM cannot decide.

Reference: ``_fallback_decision`` (``scheduler.py:521-559``).

* no nodes -> ``("", 0.0, "No nodes available", True)``
* nodes whose conditions lack ``Ready=True`` are skipped
* ``resource_balanced``: 0.35*(100-cpu%)/100 + 0.35*(100-mem%)/100 + 0.30*(max-pods)/max
* ``least_loaded``: (100-cpu%) + (100-mem%)
* anything else (``round_robin`` included): score = pod_count, i.e. the node with the MOST pods
  wins (quirk 1, preserved by default via ``compat.round_robin_picks_most_pods``).  With the
  quirk disabled ``round_robin`` rotates over the Ready nodes in list order.
* ties keep the first node in list order (strict ``>``); the initial best score is -1, so a
  node with score exactly -1 can never win (reachable only with negative usage numbers).
* result: confidence 0.4, reasoning ``"Fallback ({strategy}): {reason}"``, ``fallback_needed``;
  no eligible node -> ``("", 0.0, "Fallback failed: {reason}", True)``.
"""

from __future__ import annotations

import itertools
import threading
from typing import Callable, Dict, Optional, Sequence

from .models import NodeMetrics, SchedulingDecision

FALLBACK_CONFIDENCE = 0.4


def _resource_balanced(n: NodeMetrics) -> float:
    cpu = (100 - n.cpu_usage_percent) / 100.0
    mem = (100 - n.memory_usage_percent) / 100.0
    pods = (n.max_pods - n.pod_count) / n.max_pods if n.max_pods > 0 else 0
    return cpu * 0.35 + mem * 0.35 + pods * 0.30


def _least_loaded(n: NodeMetrics) -> float:
    return (100 - n.cpu_usage_percent) + (100 - n.memory_usage_percent)


def _pod_count(n: NodeMetrics) -> float:
    return n.pod_count


SCORERS: Dict[str, Callable[[NodeMetrics], float]] = {
    "resource_balanced": _resource_balanced,
    "least_loaded": _least_loaded,
}


class FallbackPolicy:
    def __init__(self, strategy: str = "resource_balanced", round_robin_picks_most_pods: bool = True):
        self.strategy = strategy
        self.quirk_rr = round_robin_picks_most_pods
        self._rr = itertools.count()
        self._rr_lock = threading.Lock()

    def decide(self, nodes: Sequence[NodeMetrics], reason: str) -> SchedulingDecision:
        if not nodes:
            return SchedulingDecision("", 0.0, "No nodes available", True)
        ready = [n for n in nodes if n.is_ready]
        best: Optional[NodeMetrics] = None
        if self.strategy == "round_robin" and not self.quirk_rr:
            if ready:
                with self._rr_lock:
                    best = ready[next(self._rr) % len(ready)]
        else:
            score_fn = SCORERS.get(self.strategy, _pod_count)
            best_score = -1.0
            for n in ready:
                s = score_fn(n)
                if s > best_score:
                    best_score, best = s, n
        if best is None:
            return SchedulingDecision("", 0.0, f"Fallback failed: {reason}", True)
        return SchedulingDecision(best.name, FALLBACK_CONFIDENCE,
                                  f"Fallback ({self.strategy}): {reason}", True)
