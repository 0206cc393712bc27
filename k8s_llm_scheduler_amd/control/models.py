"""Scheduling data model.

Field-for-field compatible with the reference dataclasses ``NodeMetrics``
(``scheduler.py:72-84``), ``PodSpec`` (``:86-96``) and ``SchedulingDecision`` (``:98-104``).
Kubernetes objects themselves are handled as plain JSON dicts (the apiserver's wire form), so
neither the ``kubernetes`` package nor its model classes are needed.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List


@dataclass
class NodeMetrics:
    name: str
    cpu_usage_percent: float
    memory_usage_percent: float
    available_cpu: float          # allocatable cores
    available_memory: float       # allocatable GB (GiB, as the reference computes it)
    pod_count: int
    max_pods: int
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Dict[str, str]] = field(default_factory=list)
    conditions: List[Dict[str, str]] = field(default_factory=list)

    @property
    def is_ready(self) -> bool:
        """The fallback's readiness test (scheduler.py:532-533)."""
        return any(c.get("type") == "Ready" and c.get("status") == "True" for c in self.conditions)


@dataclass
class PodSpec:
    name: str
    namespace: str
    cpu_request: float            # cores
    memory_request: float         # GB
    node_selector: Dict[str, str] = field(default_factory=dict)
    tolerations: List[Any] = field(default_factory=list)
    affinity_rules: Dict[str, Any] = field(default_factory=dict)
    priority: int = 0
    uid: str = ""                 # not in the reference; used for de-duplication


@dataclass
class SchedulingDecision:
    selected_node: str
    confidence: float
    reasoning: str
    fallback_needed: bool = False
