"""Cluster snapshot (the reference's "Context Manager") and pod -> PodSpec conversion.

Reference semantics kept for every derived value (``scheduler.py:121-170``):

* ``available_cpu`` / ``available_memory`` come from **allocatable**, ``max_pods`` from
  allocatable pods; ``capacity`` is ignored,
* ``pod_count`` = every pod whose ``spec.nodeName`` is the node, whatever its phase,
* "usage" is synthetic: ``cpu% = mem% = pod_count / max_pods * 50`` (quirk 4),
* any error while snapshotting yields ``[]``.

Two modes (``compat.snapshot_mode``):

``direct``    the reference's N+1 REST calls per decision (``list_node`` + one field-selected
              pod list per node, ``scheduler.py:124-147``).
``informer``  one ``list_nodes`` per snapshot; pod counts per node are maintained from the pod
              watch stream (``observe``) plus an *assume* step right after our own successful
              bindings, so a snapshot taken immediately after a bind already counts the pod --
              what the apiserver would have answered the reference.  Counts are rebuilt from a
              LIST at the start of every watch stream (LIST + WATCH from its resourceVersion).
"""

from __future__ import annotations

import logging
import threading
from typing import Dict, List, Optional, Sequence

from ..kube.api import KubeAPI, Obj, pod_key
from . import quantity
from .models import NodeMetrics, PodSpec

log = logging.getLogger(__name__)


def node_to_metrics(node: Obj, pod_count: int, qmode: str = "full") -> NodeMetrics:
    md, spec, status = node.get("metadata", {}), node.get("spec", {}) or {}, node.get("status", {}) or {}
    alloc = status.get("allocatable", {}) or {}
    cpu = quantity.node_cpu(alloc.get("cpu", "0"), qmode)
    mem = quantity.node_memory_gb(alloc.get("memory", "0"), qmode)
    max_pods = int(alloc.get("pods", "0"))
    usage = (pod_count / max_pods) * 50 if max_pods > 0 else 0
    return NodeMetrics(
        name=md.get("name", ""),
        cpu_usage_percent=usage,
        memory_usage_percent=usage,
        available_cpu=cpu,
        available_memory=mem,
        pod_count=pod_count,
        max_pods=max_pods,
        labels=dict(md.get("labels") or {}),
        taints=[{"key": t.get("key", ""), "effect": t.get("effect", ""), "value": t.get("value") or ""}
                for t in (spec.get("taints") or [])],
        conditions=[{"type": c.get("type", ""), "status": c.get("status", ""), "reason": c.get("reason") or ""}
                    for c in (status.get("conditions") or [])],
    )


def pod_to_spec(pod: Obj, qmode: str = "full") -> PodSpec:
    """Reference ``_convert_pod_to_spec`` (``scheduler.py:731-764``): requests summed over
    ``spec.containers`` only (init containers, overhead and limits ignored)."""
    md, spec = pod.get("metadata", {}), pod.get("spec", {}) or {}
    cpu = mem = 0.0
    for c in spec.get("containers") or []:
        req = ((c.get("resources") or {}).get("requests")) or {}
        if req:
            cpu += quantity.pod_cpu(req.get("cpu", "0"), qmode)
            mem += quantity.pod_memory_gb(req.get("memory", "0"), qmode)
    return PodSpec(
        name=md.get("name", ""),
        namespace=md.get("namespace", "default"),
        cpu_request=cpu,
        memory_request=mem,
        node_selector=dict(spec.get("nodeSelector") or {}),
        tolerations=list(spec.get("tolerations") or []),
        affinity_rules={},
        priority=spec.get("priority") or 0,
        uid=md.get("uid", "") or pod_key(pod),
    )


class ClusterSnapshotter:
    def __init__(self, api: KubeAPI, mode: str = "informer", quantity_mode: str = "full"):
        self.api = api
        self.mode = mode
        self.qmode = quantity_mode
        self._lock = threading.Lock()
        self._pod_node: Dict[str, str] = {}   # pod key -> node name (bound pods only)
        self._seeded = False

    # ------------------------------------------------------------ informer bookkeeping
    def seed(self) -> None:
        pods, _ = self.api.list_pods()
        self.resync(pods)

    def resync(self, pods: Sequence[Obj]) -> None:
        """Replace the pod -> node map with one LIST result.  Called at the start of every watch
        stream (the watch then continues from that LIST's resourceVersion), so pods deleted while
        no stream was open -- e.g. during the 5 s error back-off -- cannot linger in the counts."""
        with self._lock:
            self._pod_node = {pod_key(p): p["spec"]["nodeName"] for p in pods
                              if (p.get("spec") or {}).get("nodeName")}
            self._seeded = True

    def observe(self, event_type: str, pod: Obj) -> None:
        key = pod_key(pod)
        node = (pod.get("spec") or {}).get("nodeName")
        with self._lock:
            if event_type == "DELETED" or not node:
                self._pod_node.pop(key, None)
            else:
                self._pod_node[key] = node

    def assume(self, pod_key_: str, node: str) -> None:
        with self._lock:
            self._pod_node[pod_key_] = node

    # ------------------------------------------------------------ snapshot
    def get_node_metrics(self) -> List[NodeMetrics]:
        try:
            nodes = self.api.list_nodes()
            if self.mode == "direct":
                out = []
                for n in nodes:
                    name = n["metadata"]["name"]
                    pods, _ = self.api.list_pods(field_selector=f"spec.nodeName={name}")
                    out.append(node_to_metrics(n, len(pods), self.qmode))
                return out
            if not self._seeded:
                self.seed()
            with self._lock:
                counts: Dict[str, int] = {}
                for node in self._pod_node.values():
                    counts[node] = counts.get(node, 0) + 1
            return [node_to_metrics(n, counts.get(n["metadata"]["name"], 0), self.qmode) for n in nodes]
        except Exception as e:
            log.error(f"Error collecting node metrics: {e}")
            return []


def apply_assumed_binding(nodes: Sequence[NodeMetrics], node_name: str) -> List[NodeMetrics]:
    """Snapshot as it would look after one more pod lands on ``node_name`` (batched rounds)."""
    out = []
    for n in nodes:
        if n.name == node_name:
            pc = n.pod_count + 1
            usage = (pc / n.max_pods) * 50 if n.max_pods > 0 else 0
            n = NodeMetrics(n.name, usage, usage, n.available_cpu, n.available_memory, pc, n.max_pods,
                            n.labels, n.taints, n.conditions)
        out.append(n)
    return out


def find_node(nodes: Sequence[NodeMetrics], name: str) -> Optional[NodeMetrics]:
    return next((n for n in nodes if n.name == name), None)
