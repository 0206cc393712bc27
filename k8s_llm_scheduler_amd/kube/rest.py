"""Dependency-free Kubernetes REST client (``requests`` over HTTPS).

Replaces the ``kubernetes`` python package the reference imports (``scheduler.py:17-18``).
Connection sources, in order:

1. an explicit kubeconfig path (or ``$KUBECONFIG``, or ``~/.kube/config``): current context's
   cluster ``server`` + ``certificate-authority(-data)`` / ``insecure-skip-tls-verify`` and the
   user's ``token`` / ``tokenFile`` / ``client-certificate(-data)`` + ``client-key(-data)`` /
   basic auth (exec/auth-provider plugins are not supported),
2. in-cluster service-account credentials (the reference can only use a kubeconfig,
   ``scheduler.py:114``; quirk 11 fixed).

Endpoints: ``GET /api/v1/nodes``, ``GET /api/v1/pods[?fieldSelector=]``, the chunked watch
``GET /api/v1/pods?watch=1&resourceVersion=&timeoutSeconds=`` and
``POST /api/v1/namespaces/{ns}/pods/{name}/binding``.
"""

from __future__ import annotations

import base64
import json
import os
import tempfile
from pathlib import Path
from typing import Any, Dict, Iterator, List, Optional, Tuple

import yaml

from .api import ApiError, Obj, WatchEvent

SA_DIR = Path("/var/run/secrets/kubernetes.io/serviceaccount")


def _materialize(data_b64: Optional[str], path: Optional[str], base: Path, suffix: str) -> Optional[str]:
    if data_b64:
        f = tempfile.NamedTemporaryFile(delete=False, suffix=suffix)
        f.write(base64.b64decode(data_b64))
        f.close()
        return f.name
    if path:
        p = Path(path)
        return str(p if p.is_absolute() else base / p)
    return None


class KubeConnection:
    def __init__(self, server: str, verify: Any = True, token: Optional[str] = None,
                 cert: Optional[Tuple[str, str]] = None, auth: Optional[Tuple[str, str]] = None):
        self.server = server.rstrip("/")
        self.verify = verify
        self.token = token
        self.cert = cert
        self.auth = auth

    @classmethod
    def from_kubeconfig(cls, path: Optional[str] = None, context: Optional[str] = None) -> "KubeConnection":
        p = Path(path or os.environ.get("KUBECONFIG", "").split(os.pathsep)[0] or Path.home() / ".kube" / "config")
        cfg = yaml.safe_load(p.read_text())
        ctx_name = context or cfg.get("current-context")
        ctx = next(c["context"] for c in cfg.get("contexts", []) if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in cfg.get("clusters", []) if c["name"] == ctx["cluster"])
        user = next((u.get("user", {}) for u in cfg.get("users", []) if u["name"] == ctx.get("user")), {})
        base = p.parent
        if cluster.get("insecure-skip-tls-verify"):
            verify: Any = False
        else:
            verify = _materialize(cluster.get("certificate-authority-data"),
                                  cluster.get("certificate-authority"), base, ".crt") or True
        token = user.get("token")
        if not token and user.get("tokenFile"):
            token = Path(user["tokenFile"]).read_text().strip()
        cert_f = _materialize(user.get("client-certificate-data"), user.get("client-certificate"), base, ".crt")
        key_f = _materialize(user.get("client-key-data"), user.get("client-key"), base, ".key")
        auth = (user["username"], user.get("password", "")) if user.get("username") else None
        if "exec" in user or "auth-provider" in user:
            raise RuntimeError("kubeconfig exec/auth-provider plugins are not supported; use a token")
        return cls(cluster["server"], verify, token, (cert_f, key_f) if cert_f and key_f else None, auth)

    @classmethod
    def in_cluster(cls) -> "KubeConnection":
        host, port = os.environ["KUBERNETES_SERVICE_HOST"], os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        token = (SA_DIR / "token").read_text().strip()
        ca = SA_DIR / "ca.crt"
        return cls(f"https://{host}:{port}", str(ca) if ca.exists() else True, token)

    @classmethod
    def auto(cls, kubeconfig: Optional[str] = None) -> "KubeConnection":
        if kubeconfig:
            return cls.from_kubeconfig(kubeconfig)
        if "KUBERNETES_SERVICE_HOST" in os.environ and (SA_DIR / "token").exists():
            return cls.in_cluster()
        return cls.from_kubeconfig()


class RestKubeAPI:
    def __init__(self, conn: KubeConnection, request_timeout: float = 30.0):
        import requests  # local import: only needed when talking to a real apiserver

        self.conn = conn
        self.timeout = request_timeout
        self.session = requests.Session()
        self.session.verify = conn.verify
        if conn.cert:
            self.session.cert = conn.cert
        if conn.auth:
            self.session.auth = conn.auth
        self.session.headers["Accept"] = "application/json"
        if conn.token:
            self.session.headers["Authorization"] = f"Bearer {conn.token}"

    def _check(self, r) -> Any:
        if r.status_code >= 400:
            raise ApiError(r.status_code, r.reason or "", r.text)
        return r.json()

    def list_nodes(self) -> List[Obj]:
        r = self.session.get(f"{self.conn.server}/api/v1/nodes", timeout=self.timeout)
        return self._check(r).get("items", [])

    def list_pods(self, field_selector: Optional[str] = None) -> Tuple[List[Obj], str]:
        params = {"fieldSelector": field_selector} if field_selector else None
        r = self.session.get(f"{self.conn.server}/api/v1/pods", params=params, timeout=self.timeout)
        body = self._check(r)
        return body.get("items", []), body.get("metadata", {}).get("resourceVersion", "")

    def watch_pods(self, resource_version: Optional[str] = None,
                   timeout_seconds: int = 60) -> Iterator[WatchEvent]:
        params: Dict[str, Any] = {"watch": "1", "timeoutSeconds": str(int(timeout_seconds)),
                                  "allowWatchBookmarks": "true"}
        if resource_version:
            params["resourceVersion"] = resource_version
        with self.session.get(f"{self.conn.server}/api/v1/pods", params=params, stream=True,
                              timeout=(self.timeout, timeout_seconds + 30)) as r:
            if r.status_code >= 400:
                raise ApiError(r.status_code, r.reason or "", r.text)
            for line in r.iter_lines():
                if not line:
                    continue
                ev = json.loads(line)
                typ, obj = ev.get("type", ""), ev.get("object") or {}
                if typ == "ERROR":
                    # a Status object, not a pod.  410 Gone (the resourceVersion was compacted away): end the stream
                    # at once -- the watch loop re-LISTs and watches from the new resourceVersion; any other error
                    # goes through the loop's error back-off
                    code = int(obj.get("code") or 0)
                    if code == 410:
                        return
                    raise ApiError(code or 500, obj.get("reason", "") or "watch error", json.dumps(obj))
                rv = (obj.get("metadata") or {}).get("resourceVersion")
                if rv:
                    self.last_resource_version = rv
                if typ == "BOOKMARK":
                    continue        # only advances the resourceVersion (allowWatchBookmarks): no pod in it
                yield typ, obj

    last_resource_version: str = ""   # of the last watch event or bookmark seen

    def create_binding(self, namespace: str, body: Obj) -> Obj:
        name = body["metadata"]["name"]
        r = self.session.post(f"{self.conn.server}/api/v1/namespaces/{namespace}/pods/{name}/binding",
                              data=json.dumps(body), headers={"Content-Type": "application/json"},
                              timeout=self.timeout)
        return self._check(r)

    # ---- used by the smoke tool (kubectl apply/delete equivalents)
    def create_pod(self, pod: Obj) -> Obj:
        ns = pod.get("metadata", {}).get("namespace", "default")
        r = self.session.post(f"{self.conn.server}/api/v1/namespaces/{ns}/pods", data=json.dumps(pod),
                              headers={"Content-Type": "application/json"}, timeout=self.timeout)
        return self._check(r)

    def delete_pod(self, namespace: str, name: str) -> None:
        r = self.session.delete(f"{self.conn.server}/api/v1/namespaces/{namespace}/pods/{name}",
                                timeout=self.timeout)
        if r.status_code not in (200, 202, 404):
            raise ApiError(r.status_code, r.reason or "", r.text)

    def get_pod(self, namespace: str, name: str) -> Optional[Obj]:
        r = self.session.get(f"{self.conn.server}/api/v1/namespaces/{namespace}/pods/{name}", timeout=self.timeout)
        if r.status_code == 404:
            return None
        return self._check(r)
