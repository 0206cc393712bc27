"""The slice of the Kubernetes API the scheduler uses, as a small protocol over JSON dicts.

The reference calls the ``kubernetes`` python client: ``list_node`` (``scheduler.py:124``),
``list_pod_for_all_namespaces`` with a ``spec.nodeName`` field selector (``:144-146``), a
``Watch().stream`` over all pods (``:664-667``) and ``create_namespaced_binding``
(``:598-602``).  Implementations here: :class:`~.fake.FakeKubeAPI` (in-memory, tests and the
CPU plumbing config) and :class:`~.rest.RestKubeAPI` (plain HTTPS, kubeconfig or in-cluster).
"""

from __future__ import annotations

from typing import Any, Dict, Iterator, List, Optional, Protocol, Tuple

Obj = Dict[str, Any]
WatchEvent = Tuple[str, Obj]   # ("ADDED" | "MODIFIED" | "DELETED" | "BOOKMARK" | "ERROR", object)


class ApiError(Exception):
    """HTTP-level API failure (mirrors kubernetes.client.rest.ApiException's status/body)."""

    def __init__(self, status: int, reason: str = "", body: Optional[str] = None):
        super().__init__(f"({status}) Reason: {reason}")
        self.status = status
        self.reason = reason
        self.body = body


class KubeAPI(Protocol):
    def list_nodes(self) -> List[Obj]:
        ...

    def list_pods(self, field_selector: Optional[str] = None) -> Tuple[List[Obj], str]:
        """Returns (pods, resourceVersion)."""
        ...

    def watch_pods(self, resource_version: Optional[str] = None,
                   timeout_seconds: int = 60) -> Iterator[WatchEvent]:
        ...

    def create_binding(self, namespace: str, body: Obj) -> Obj:
        ...


def binding_body(pod_name: str, namespace: str, node_name: str) -> Obj:
    """The Binding object of scheduler.py:583-595 in wire form."""
    return {
        "apiVersion": "v1",
        "kind": "Binding",
        "metadata": {"name": pod_name, "namespace": namespace},
        "target": {"apiVersion": "v1", "kind": "Node", "name": node_name},
    }


def pod_key(pod: Obj) -> str:
    md = pod.get("metadata", {})
    return f"{md.get('namespace', 'default')}/{md.get('name', '')}"


def pod_uid(pod: Obj) -> str:
    md = pod.get("metadata", {})
    return md.get("uid") or pod_key(pod)
