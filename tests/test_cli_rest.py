"""CLI (run / smoke / verify on the in-memory cluster), JSON logging, metrics, and the
dependency-free REST client against a local fake apiserver (HTTP, kubeconfig auth)."""

import json
import logging
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from k8s_llm_scheduler_amd.__main__ import main as cli
from k8s_llm_scheduler_amd.control.metrics import SchedulerMetrics
from k8s_llm_scheduler_amd.kube import ApiError, FakeKubeAPI, make_node, make_pod
from k8s_llm_scheduler_amd.kube.rest import KubeConnection, RestKubeAPI
from k8s_llm_scheduler_amd.utils.logging import JsonFormatter, setup_logging


def test_cli_smoke_fake_cluster_fallback(capsys):
    assert cli(["smoke", "--fake-cluster", "3", "--backend", "fallback", "--wait", "5"]) == 0
    assert "Results: 3/3 pods scheduled" in capsys.readouterr().out


def test_cli_e2e_fake_cluster_scripted(capsys):
    """test_e2e.py flow: verify, cleanup, node list, in-process scheduler, apply, scheduled AND Running."""
    assert cli(["e2e", "--fake-cluster", "3", "--backend", "scripted", "--wait", "5"]) == 0
    out = capsys.readouterr().out
    for line in ("Cluster has 3 nodes:", "Scheduled: 3/3 pods", "Running:   3/3 pods", "SUCCESS! All pods scheduled"):
        assert line in out, line
    assert out.count("ai-llama-scheduler") >= 3  # schedulerName column


def test_cli_run_scripted_demo(capsys):
    assert cli(["run", "--fake-cluster", "3", "--backend", "scripted", "--demo-pods", "--duration", "1.5"]) == 0
    out = capsys.readouterr().out
    assert "Total Scheduled: 3" in out and "LLM Decisions: 3" in out and "Circuit Breaker Trips: 0" in out


def test_json_logging():
    rec = logging.LogRecord("x", logging.INFO, __file__, 1, " Bound pod default/a to node n", None, None)
    d = json.loads(JsonFormatter().format(rec))
    assert d["level"] == "INFO" and d["message"] == "Bound pod default/a to node n"
    setup_logging("DEBUG", "json")
    assert logging.getLogger().level == logging.DEBUG
    setup_logging("INFO", "text")


def test_metrics_counters():
    m = SchedulerMetrics(True, None)
    m.decision("llm", 0.2)
    m.bound(True)
    m.llm_event("cached_requests", 2)
    from prometheus_client import generate_latest

    text = generate_latest(m.registry).decode()
    assert 'scheduler_decisions_total{source="llm"} 1.0' in text
    assert "scheduler_pods_scheduled_total 1.0" in text


class _Apiserver(BaseHTTPRequestHandler):
    """Minimal apiserver over a FakeKubeAPI: nodes, pods (+fieldSelector), watch, binding."""

    fake: FakeKubeAPI = None
    token = "s3cret"
    script = None        # raw watch events to stream instead of the fake's (ERROR / BOOKMARK tests)

    def log_message(self, *a):
        pass

    def _auth(self):
        if self.headers.get("Authorization") != f"Bearer {self.token}":
            self._send(401, {"message": "Unauthorized"})
            return False
        return True

    def _send(self, code, obj):
        body = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def do_GET(self):
        if not self._auth():
            return
        from urllib.parse import parse_qs, urlparse

        u = urlparse(self.path)
        q = {k: v[0] for k, v in parse_qs(u.query).items()}
        if u.path == "/api/v1/nodes":
            return self._send(200, {"items": self.fake.list_nodes()})
        if u.path == "/api/v1/pods" and q.get("watch"):
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.end_headers()
            evs = self.script if self.script is not None else \
                self.fake.watch_pods(None, timeout_seconds=float(q.get("timeoutSeconds", 1)))
            for typ, obj in evs:
                self.wfile.write((json.dumps({"type": typ, "object": obj}) + "\n").encode())
                self.wfile.flush()
            return
        if u.path == "/api/v1/pods":
            pods, rv = self.fake.list_pods(q.get("fieldSelector"))
            return self._send(200, {"items": pods, "metadata": {"resourceVersion": rv}})
        self._send(404, {"message": "not found"})

    def do_POST(self):
        if not self._auth():
            return
        body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
        parts = self.path.strip("/").split("/")
        if parts[-1] == "binding":
            try:
                self.fake.create_binding(parts[3], body)
                return self._send(201, {"kind": "Status", "status": "Success"})
            except ApiError as e:
                return self._send(e.status, json.loads(e.body))
        self._send(404, {"message": "not found"})


@pytest.fixture
def apiserver(tmp_path):
    fake = FakeKubeAPI([make_node("n1"), make_node("n2", ready=False)])
    _Apiserver.fake = fake
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _Apiserver)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    kc = tmp_path / "kubeconfig"
    kc.write_text(
        "apiVersion: v1\nkind: Config\ncurrent-context: c\n"
        f"clusters: [{{name: k, cluster: {{server: 'http://127.0.0.1:{srv.server_address[1]}'}}}}]\n"
        "contexts: [{name: c, context: {cluster: k, user: u}}]\n"
        f"users: [{{name: u, user: {{token: {_Apiserver.token}}}}}]\n")
    yield fake, str(kc)
    srv.shutdown()


def test_rest_client_against_fake_apiserver(apiserver):
    fake, kc = apiserver
    api = RestKubeAPI(KubeConnection.from_kubeconfig(kc))
    assert [n["metadata"]["name"] for n in api.list_nodes()] == ["n1", "n2"]
    fake.create_pod(make_pod("p1"))
    fake.create_pod(make_pod("p2", node_name="n1", phase="Running"))
    pods, _ = api.list_pods("spec.nodeName=n1")
    assert [p["metadata"]["name"] for p in pods] == ["p2"]
    events = list(api.watch_pods(None, timeout_seconds=1))
    assert {e[1]["metadata"]["name"] for e in events} == {"p1", "p2"}
    from k8s_llm_scheduler_amd.control.binder import IntegrationLayer

    il = IntegrationLayer(api)
    assert il.bind("p1", "default", "n1") is True
    assert il.bind("p1", "default", "n1") is False        # 409 conflict, logged, returns False
    assert fake.get_pod("default", "p1")["spec"]["nodeName"] == "n1"


def test_rest_client_auth_error(apiserver):
    fake, kc = apiserver
    conn = KubeConnection.from_kubeconfig(kc)
    conn.token = "wrong"
    with pytest.raises(ApiError) as ei:
        RestKubeAPI(conn).list_nodes()
    assert ei.value.status == 401


def test_rest_watch_ends_on_410_and_hides_bookmarks(apiserver):
    """ERROR events carry a Status, BOOKMARK events only a resourceVersion.  A 410 Gone ends the
    stream at once (the watch loop then re-LISTs), a bookmark advances the client's resourceVersion and never reaches
    the consumer as a pod, any other ERROR raises (the loop's error back-off)."""
    fake, kc = apiserver
    api = RestKubeAPI(KubeConnection.from_kubeconfig(kc))
    p1, p2 = make_pod("p1"), make_pod("p2")
    p1["metadata"]["resourceVersion"] = "40"
    bookmark = {"kind": "Pod", "metadata": {"resourceVersion": "42"}}
    gone = {"kind": "Status", "status": "Failure", "reason": "Expired", "code": 410,
            "message": "too old resource version: 7 (40)"}
    try:
        _Apiserver.script = [("ADDED", p1), ("BOOKMARK", bookmark), ("ERROR", gone), ("ADDED", p2)]
        events = list(api.watch_pods("7", timeout_seconds=1))
        assert [(t, o["metadata"]["name"]) for t, o in events] == [("ADDED", "p1")]
        assert api.last_resource_version == "42"
        _Apiserver.script = [("ERROR", {"kind": "Status", "code": 500, "reason": "InternalError"})]
        with pytest.raises(ApiError) as ei:
            list(api.watch_pods(None, timeout_seconds=1))
        assert ei.value.status == 500
    finally:
        _Apiserver.script = None
    # the snapshotter never sees a Status / bookmark object as a pod: the informer counts stay the pods' own
    from k8s_llm_scheduler_amd.control.cluster import ClusterSnapshotter

    snap = ClusterSnapshotter(api)
    fake.create_pod(make_pod("p3", node_name="n1", phase="Running"))
    snap.seed()
    for typ, obj in [("ADDED", p1)]:
        snap.observe(typ, obj)
    assert {m.name: m.pod_count for m in snap.get_node_metrics()} == {"n1": 1, "n2": 0}
