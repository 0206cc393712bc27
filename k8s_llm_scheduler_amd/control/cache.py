"""Decision cache.

Semantics of the reference ``RequestCache`` (``scheduler.py:257-294``):

* key = md5 of ``"{cpu}_{mem}_{priority}_" + "_".join(name_cpu%.1f_mem%.1f for nodes sorted by
  name)``; pod name/namespace are NOT part of the key (preserved),
* TTL checked on ``get``; an expired entry is deleted lazily,
* when full, ``set`` evicts the entry with the oldest insertion time before inserting (even when
  the key being set is already present); ``get`` does not refresh, so eviction is FIFO.

Here the FIFO order is kept in an ``OrderedDict`` (O(1) eviction instead of the reference's
O(n) ``min``), the clock is injectable and the cache is thread-safe (the batched scheduler
looks entries up from worker threads).
"""

from __future__ import annotations

import hashlib
import threading
import time
from collections import OrderedDict
from typing import Callable, Optional, Sequence, Tuple

from .models import NodeMetrics, PodSpec, SchedulingDecision


def cache_key(pod: PodSpec, nodes: Sequence[NodeMetrics]) -> str:
    pod_part = f"{pod.cpu_request}_{pod.memory_request}_{pod.priority}"
    node_part = "_".join(f"{n.name}_{n.cpu_usage_percent:.1f}_{n.memory_usage_percent:.1f}"
                         for n in sorted(nodes, key=lambda n: n.name))
    return hashlib.md5(f"{pod_part}_{node_part}".encode()).hexdigest()


class DecisionCache:
    def __init__(self, ttl: float = 300, max_size: int = 100,
                 clock: Callable[[], float] = time.monotonic):
        self.ttl = float(ttl)
        self.max_size = int(max_size)
        self._clock = clock
        self._lock = threading.Lock()
        self._entries: "OrderedDict[str, Tuple[SchedulingDecision, float]]" = OrderedDict()

    def __len__(self) -> int:
        return len(self._entries)

    def get(self, pod: PodSpec, nodes: Sequence[NodeMetrics]) -> Optional[SchedulingDecision]:
        key = cache_key(pod, nodes)
        with self._lock:
            hit = self._entries.get(key)
            if hit is None:
                return None
            decision, stamp = hit
            if self._clock() - stamp < self.ttl:
                return decision
            del self._entries[key]
            return None

    def set(self, pod: PodSpec, nodes: Sequence[NodeMetrics], decision: SchedulingDecision) -> None:
        key = cache_key(pod, nodes)
        with self._lock:
            if self.max_size <= 0:
                return
            if len(self._entries) >= self.max_size:
                self._entries.popitem(last=False)
            self._entries.pop(key, None)
            self._entries[key] = (decision, self._clock())

    def clear(self) -> None:
        with self._lock:
            self._entries.clear()
