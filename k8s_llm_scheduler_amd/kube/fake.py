"""In-memory Kubernetes API for tests and the CPU-only plumbing configuration.

Models what the scheduler relies on: nodes with allocatable/conditions/taints, pods with
``schedulerName``/``nodeName``/``phase``, a watch stream of ADDED/MODIFIED/DELETED events with a
resourceVersion, field-selector listing by ``spec.nodeName``, and the binding subresource
(404 for unknown pods, 409 when the pod is already bound -- the double-bind the reference can
trigger).  Fault injection: ``fail_next(op, status)`` makes the next
call of an operation raise :class:`ApiError`; ``duplicate_events`` re-emits events.
"""

from __future__ import annotations

import copy
import itertools
import queue
import threading
import time
import uuid
from typing import Any, Dict, Iterator, List, Optional, Tuple

import yaml

from .api import ApiError, Obj, WatchEvent, pod_key


def make_node(name: str, cpu: str = "4", memory: str = "8Gi", pods: str = "110", ready: bool = True,
              labels: Optional[Dict[str, str]] = None, taints: Optional[List[Dict[str, str]]] = None) -> Obj:
    return {
        "apiVersion": "v1", "kind": "Node",
        "metadata": {"name": name, "labels": labels or {"kubernetes.io/hostname": name}},
        "spec": {"taints": taints or []},
        "status": {
            "capacity": {"cpu": cpu, "memory": memory, "pods": pods},
            "allocatable": {"cpu": cpu, "memory": memory, "pods": pods},
            "conditions": [{"type": "Ready", "status": "True" if ready else "False",
                            "reason": "KubeletReady" if ready else "KubeletNotReady"}],
        },
    }


def make_pod(name: str, namespace: str = "default", cpu: Optional[str] = "100m",
             memory: Optional[str] = "128Mi", scheduler_name: str = "ai-llama-scheduler",
             node_name: Optional[str] = None, phase: str = "Pending", priority: Optional[int] = None,
             containers: int = 1) -> Obj:
    requests = {}
    if cpu is not None:
        requests["cpu"] = cpu
    if memory is not None:
        requests["memory"] = memory
    spec: Dict[str, Any] = {
        "schedulerName": scheduler_name,
        "containers": [{"name": f"c{i}", "image": "nginx:alpine", "resources": {"requests": dict(requests)}}
                       for i in range(containers)],
    }
    if node_name:
        spec["nodeName"] = node_name
    if priority is not None:
        spec["priority"] = priority
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": namespace},
            "spec": spec, "status": {"phase": phase}}


class FakeKubeAPI:
    def __init__(self, nodes: Optional[List[Obj]] = None, duplicate_events: bool = False,
                 run_bound_pods: bool = False):
        self._lock = threading.RLock()
        self._rv = itertools.count(1)
        self._nodes: Dict[str, Obj] = {}
        self._pods: Dict[str, Obj] = {}
        self._watchers: List["queue.Queue[Optional[WatchEvent]]"] = []
        self._faults: Dict[str, List[int]] = {}
        self.duplicate_events = duplicate_events
        self.run_bound_pods = run_bound_pods     # bound pods transition to Running (kubelet stand-in)
        self.bindings: List[Tuple[str, str]] = []  # (ns/name, node)
        self.binding_times: Dict[str, float] = {}   # ns/name -> time.perf_counter() of the successful bind
        self._history: List[Tuple[int, WatchEvent]] = []   # (resourceVersion, event): watch-from-rv replay
        self.calls: Dict[str, int] = {}
        for n in nodes or []:
            self.add_node(n)

    # --------------------------------------------------------------- fixtures
    def add_node(self, node: Obj) -> None:
        with self._lock:
            self._nodes[node["metadata"]["name"]] = copy.deepcopy(node)

    def create_pod(self, pod: Obj) -> Obj:
        with self._lock:
            pod = copy.deepcopy(pod)
            md = pod.setdefault("metadata", {})
            md.setdefault("namespace", "default")
            md.setdefault("uid", str(uuid.uuid4()))
            md["resourceVersion"] = str(next(self._rv))
            pod.setdefault("status", {}).setdefault("phase", "Pending")
            self._pods[pod_key(pod)] = pod
            self._emit("ADDED", pod)
            return copy.deepcopy(pod)

    def delete_pod(self, namespace: str, name: str) -> None:
        with self._lock:
            pod = self._pods.pop(f"{namespace}/{name}", None)
            if pod is not None:
                pod["metadata"]["resourceVersion"] = str(next(self._rv))
                self._emit("DELETED", pod)

    def apply_manifest(self, text: str) -> List[Obj]:
        """kubectl-apply equivalent for Pod manifests (single docs, multi-doc YAML or a List)."""
        out = []
        for doc in yaml.safe_load_all(text):
            if not doc:
                continue
            items = doc.get("items", []) if doc.get("kind") == "List" else [doc]
            for it in items:
                if it.get("kind") == "Pod":
                    out.append(self.create_pod(it))
                elif it.get("kind") == "Node":
                    self.add_node(it)
        return out

    def get_pod(self, namespace: str, name: str) -> Optional[Obj]:
        with self._lock:
            p = self._pods.get(f"{namespace}/{name}")
            return copy.deepcopy(p) if p else None

    def fail_next(self, op: str, status: int = 500, times: int = 1) -> None:
        with self._lock:
            self._faults.setdefault(op, []).extend([status] * times)

    def _maybe_fail(self, op: str) -> None:
        self.calls[op] = self.calls.get(op, 0) + 1
        f = self._faults.get(op)
        if f:
            status = f.pop(0)
            raise ApiError(status, "Injected", '{"message": "injected failure"}')

    def _emit(self, typ: str, obj: Obj) -> None:
        ev = (typ, copy.deepcopy(obj))
        self._history.append((int(obj.get("metadata", {}).get("resourceVersion", "0") or 0), ev))
        if len(self._history) > 100000:
            del self._history[:50000]
        for q in list(self._watchers):
            q.put(ev)
            if self.duplicate_events:
                q.put((typ, copy.deepcopy(obj)))

    # --------------------------------------------------------------- KubeAPI
    def list_nodes(self) -> List[Obj]:
        with self._lock:
            self._maybe_fail("list_nodes")
            return [copy.deepcopy(n) for n in self._nodes.values()]

    def list_pods(self, field_selector: Optional[str] = None) -> Tuple[List[Obj], str]:
        with self._lock:
            self._maybe_fail("list_pods")
            pods = list(self._pods.values())
            if field_selector:
                for clause in field_selector.split(","):
                    key, _, val = clause.partition("=")
                    if key.strip() == "spec.nodeName":
                        pods = [p for p in pods if p.get("spec", {}).get("nodeName", "") == val.strip()]
            return [copy.deepcopy(p) for p in pods], str(next(self._rv))

    def watch_pods(self, resource_version: Optional[str] = None,
                   timeout_seconds: int = 60) -> Iterator[WatchEvent]:
        q: "queue.Queue[Optional[WatchEvent]]" = queue.Queue()
        with self._lock:
            self._maybe_fail("watch_pods")
            if resource_version is None:
                # Like a fresh LIST+WATCH: synthetic ADDED for every existing pod.
                for p in self._pods.values():
                    q.put(("ADDED", copy.deepcopy(p)))
            else:
                # Watch from a LIST's resourceVersion: replay every later change, as the apiserver does.
                rv = int(resource_version)
                for erv, (typ, obj) in self._history:
                    if erv > rv:
                        q.put((typ, copy.deepcopy(obj)))
            self._watchers.append(q)
        deadline = time.monotonic() + timeout_seconds
        try:
            while True:
                left = deadline - time.monotonic()
                if left <= 0:
                    return
                try:
                    ev = q.get(timeout=min(left, 0.05))
                except queue.Empty:
                    continue
                if ev is None:
                    return
                yield ev
        finally:
            with self._lock:
                if q in self._watchers:
                    self._watchers.remove(q)

    def stop_watches(self) -> None:
        with self._lock:
            for q in self._watchers:
                q.put(None)

    def create_binding(self, namespace: str, body: Obj) -> Obj:
        with self._lock:
            self._maybe_fail("create_binding")
            name = body["metadata"]["name"]
            node = body["target"]["name"]
            pod = self._pods.get(f"{namespace}/{name}")
            if pod is None:
                raise ApiError(404, "Not Found", f'{{"message": "pods \\"{name}\\" not found"}}')
            if node not in self._nodes:
                raise ApiError(404, "Not Found", f'{{"message": "nodes \\"{node}\\" not found"}}')
            if pod["spec"].get("nodeName"):
                raise ApiError(409, "Conflict",
                               f'{{"message": "pod {name} is already assigned to node '
                               f'\\"{pod["spec"]["nodeName"]}\\""}}')
            pod["spec"]["nodeName"] = node
            if self.run_bound_pods:
                pod["status"]["phase"] = "Running"
            pod["metadata"]["resourceVersion"] = str(next(self._rv))
            self.bindings.append((f"{namespace}/{name}", node))
            self.binding_times[f"{namespace}/{name}"] = time.perf_counter()
            self._emit("MODIFIED", pod)
            return {"kind": "Status", "status": "Success"}
