"""T2 control-plane integration (CPU): decision service with a scripted engine, and the full
watch -> decide -> bind loop against the in-memory FakeKubeAPI (reproduces test_runner.py /
test_e2e.py semantics of the reference without a cluster)."""

import asyncio
import threading
import time
from pathlib import Path

import pytest

from k8s_llm_scheduler_amd.config import Config
from k8s_llm_scheduler_amd.control import (CustomScheduler, DecisionService, Hang, ScriptedBackend,
                                           first_node_answer)
from k8s_llm_scheduler_amd.control.cluster import ClusterSnapshotter, pod_to_spec
from k8s_llm_scheduler_amd.control.models import SchedulingDecision
from k8s_llm_scheduler_amd.kube import FakeKubeAPI, make_node, make_pod

ROOT = Path(__file__).resolve().parent.parent


def cluster(n=3, **kw):
    return FakeKubeAPI([make_node(f"kind-worker{i + 1 if i else ''}", cpu="8", memory="16281924Ki")
                        for i in range(n)], **kw)


def service(backend, **kw):
    sleeps = []
    cfg = Config()
    for k, v in kw.items():
        sec, key = k.split("__")
        setattr(getattr(cfg, sec), key, v)
    svc = DecisionService.from_config(cfg, backend, sleep=sleeps.append)
    return svc, sleeps


def snapshot(api):
    return ClusterSnapshotter(api).get_node_metrics()


def test_llm_success_and_cache():
    api = cluster()
    nodes = snapshot(api)
    be = ScriptedBackend(default='noise ```json\n{"selected_node": "kind-worker2", "confidence": 0.91, '
                                 '"reasoning": "ok"}\n```')
    svc, _ = service(be)
    pod = pod_to_spec(make_pod("a", cpu="250m", memory="256Mi"))
    d = svc.decide("prompt", pod, nodes)
    assert d == SchedulingDecision("kind-worker2", 0.91, "ok", False)
    d2 = svc.decide("prompt", pod, nodes)
    assert d2 is d and len(be.calls) == 1
    s = svc.get_stats()
    assert (s["total_requests"], s["successful_requests"], s["cached_requests"]) == (1, 1, 1)
    assert s["avg_response_time"] >= 0


def test_invalid_node_and_bad_json_fall_back_without_retry():
    nodes = snapshot(cluster())
    be = ScriptedBackend(['{"selected_node": "nope"}', "garbage"])
    svc, sleeps = service(be)
    pod = pod_to_spec(make_pod("a"))
    d1 = svc.decide("p", pod, nodes)
    assert d1.fallback_needed and d1.reasoning == "Fallback (resource_balanced): Invalid node selected"
    d2 = svc.decide("p", pod, nodes)
    assert d2.fallback_needed and d2.reasoning.endswith("JSON parsing failed")
    assert sleeps == [] and svc.circuit_breaker.failures == 0   # returned, not raised (quirk 6)
    assert svc.get_stats()["total_requests"] == 2                # fallbacks are not cached


def test_retries_backoff_then_fallback():
    nodes = snapshot(cluster())
    be = ScriptedBackend([RuntimeError("e1"), RuntimeError("e2"), RuntimeError("e3")])
    svc, sleeps = service(be)
    d = svc.decide("p", pod_to_spec(make_pod("a")), nodes)
    assert sleeps == [1.0, 2.0]                                  # 2**attempt
    assert d.fallback_needed and d.reasoning == "Fallback (resource_balanced): All retries failed: e3"
    assert svc.get_stats()["failed_requests"] == 1


def test_breaker_opens_and_trips():
    nodes = snapshot(cluster())
    be = ScriptedBackend(default=RuntimeError("down"))
    svc, _ = service(be, circuit_breaker__failure_threshold=3)
    pod = pod_to_spec(make_pod("a"))
    svc.decide("p", pod, nodes)                 # 3 failures -> OPEN
    d = svc.decide("p", pod, nodes)
    assert d.reasoning.endswith("Circuit breaker open")
    assert svc.get_stats()["circuit_breaker_trips"] == 1


def test_timeout_is_enforced_via_backend_deadline():
    nodes = snapshot(cluster())
    be = ScriptedBackend([Hang(10), Hang(10), first_node_answer])
    svc, sleeps = service(be, llm__timeout=0.01)
    t0 = time.time()
    d = svc.decide("VALID NODE NAMES: kind-worker, kind-worker2\n", pod_to_spec(make_pod("a")), nodes)
    assert time.time() - t0 < 2 and not d.fallback_needed and d.selected_node == "kind-worker"


def test_max_retries_zero_falls_back():
    svc, _ = service(ScriptedBackend(), llm__max_retries=0)
    d = svc.decide("p", pod_to_spec(make_pod("a")), snapshot(cluster()))
    assert d.fallback_needed                                    # quirk 13 fixed: no None


def test_non_numeric_confidence():
    be = ScriptedBackend(['{"selected_node": "kind-worker", "confidence": "high"}'])
    svc, _ = service(be)
    d = svc.decide("p", pod_to_spec(make_pod("a")), snapshot(cluster()))
    assert d.confidence == 0.8 and d.reasoning == "LLM decision"


def test_snapshot_direct_equals_informer():
    api = cluster()
    api.create_pod(make_pod("x", node_name="kind-worker2", phase="Running"))
    api.create_pod(make_pod("y", node_name="kind-worker2", phase="Succeeded"))   # counted too
    a = ClusterSnapshotter(api, "direct").get_node_metrics()
    b = ClusterSnapshotter(api, "informer").get_node_metrics()
    assert a == b and a[1].pod_count == 2 and a[1].cpu_usage_percent == pytest.approx(2 / 110 * 50)
    assert api.calls["list_pods"] == 3 + 1                     # N direct + 1 seed


def test_snapshot_error_returns_empty():
    api = cluster()
    api.fail_next("list_nodes", 500)
    assert ClusterSnapshotter(api).get_node_metrics() == []


def test_pod_to_spec_sums_containers():
    s = pod_to_spec(make_pod("p", cpu="250m", memory="256Mi", containers=2, priority=7))
    assert (s.cpu_request, s.memory_request, s.priority) == (0.5, 0.5, 7)


def run_scheduler(api, backend, manifest_pods, mode="sequential", timeout=10.0, **extra):
    svc, _ = service(backend)
    sched = CustomScheduler("ai-llama-scheduler", api, svc, mode=mode, watch_timeout=1, **extra)

    async def main():
        task = asyncio.create_task(sched.start())
        await asyncio.sleep(0.05)
        for p in manifest_pods:
            api.create_pod(p)
        t0 = time.time()
        while time.time() - t0 < timeout:
            if all(api.get_pod("default", p["metadata"]["name"])["spec"].get("nodeName") for p in manifest_pods):
                break
            await asyncio.sleep(0.02)
        sched.stop()
        await asyncio.wait_for(task, 5)

    asyncio.run(main())
    return sched


def ai_test_pods(api):
    text = (ROOT / "examples" / "ai-test-pods.yaml").read_text()
    created = FakeKubeAPI().apply_manifest(text)
    return created


@pytest.mark.parametrize("mode", ["sequential", "batched", "continuous"])
def test_e2e_ai_test_pods_all_bound_llm_path(mode):
    api = cluster(run_bound_pods=True)
    pods = ai_test_pods(api)
    assert len(pods) == 3
    sched = run_scheduler(api, ScriptedBackend(default=first_node_answer), pods, mode=mode)
    for p in pods:
        assert api.get_pod("default", p["metadata"]["name"])["status"]["phase"] == "Running"
    st = sched.get_stats()
    assert st["total_scheduled"] == 3 and st["failed_bindings"] == 0
    assert st["llm_decisions"] + st["fallback_decisions"] == 3


def test_e2e_fallback_only_and_duplicate_events():
    api = cluster(duplicate_events=True)
    pods = ai_test_pods(api)
    sched = run_scheduler(api, None, pods)
    st = sched.get_stats()
    assert st["total_scheduled"] == 3 and st["fallback_decisions"] == 3
    assert st["failed_bindings"] == 0 and len(api.bindings) == 3   # no double bind (quirk 8 fixed)


def test_e2e_bind_failure_is_requeued_by_relist():
    api = cluster()
    api.fail_next("create_binding", 500)
    pods = [make_pod("solo")]
    sched = run_scheduler(api, None, pods, timeout=6)
    assert api.get_pod("default", "solo")["spec"]["nodeName"]
    assert sched.get_stats()["failed_bindings"] == 1 and sched.get_stats()["total_scheduled"] == 1


def test_batched_round_revalidates_capacity():
    api = FakeKubeAPI([make_node("small", pods="1"), make_node("big", pods="110")])
    be = ScriptedBackend(default='{"selected_node": "small"}')
    svc, _ = service(be)
    sched = CustomScheduler("ai-llama-scheduler", api, svc, mode="batched")
    pods = [api.create_pod(make_pod(f"p{i}")) for i in range(3)]
    out = sched.schedule_batch(pods)
    assert out[0].selected_node == "small" and not out[0].fallback_needed
    assert all(d.selected_node == "big" and d.fallback_needed for d in out[1:])
    assert len(be.calls) == 1 and len(be.calls[0]) == 3     # one engine call for the batch


def test_fault_injection_hook_drives_retries_breaker_and_fallback():
    from k8s_llm_scheduler_amd.control.backends import FaultInjectingBackend

    nodes = snapshot(cluster())
    pod = pod_to_spec(make_pod("a"))
    inner = ScriptedBackend(default=first_node_answer)
    assert FaultInjectingBackend.from_spec(inner, "none") is inner
    # every call raises: 3 retries, then the breaker opens and trips
    fi = FaultInjectingBackend.from_spec(inner, "raise:1.0")
    svc, sleeps = service(fi, circuit_breaker__failure_threshold=3)
    d = svc.decide("VALID NODE NAMES: kind-worker\n", pod, nodes)
    assert d.fallback_needed and sleeps == [1.0, 2.0] and fi.injected == 3
    assert svc.decide("VALID NODE NAMES: kind-worker\n", pod, nodes).reasoning.endswith("Circuit breaker open")
    # garbage answers: fallback "JSON parsing failed", not a breaker failure (reference quirk 6)
    svc, _ = service(FaultInjectingBackend.from_spec(inner, "garbage:1"))
    d = svc.decide("VALID NODE NAMES: kind-worker\n", pod, nodes)
    assert d.reasoning.endswith("JSON parsing failed") and svc.circuit_breaker.failures == 0
    # hang past the deadline -> engine failure per attempt
    svc, _ = service(FaultInjectingBackend.from_spec(inner, "hang:1"), llm__timeout=0.01, llm__max_retries=1)
    d = svc.decide("VALID NODE NAMES: kind-worker\n", pod, nodes)
    assert d.fallback_needed and svc.get_stats()["failed_requests"] == 1
    # rate 0: transparent
    svc, _ = service(FaultInjectingBackend.from_spec(inner, "raise:0.0"))
    assert svc.decide("VALID NODE NAMES: kind-worker\n", pod, nodes).selected_node == "kind-worker"


@pytest.mark.parametrize("mode", ["sequential", "batched", "continuous"])
def test_e2e_real_engine_forced_decode_llm_success_path(mode):
    """The whole pipeline through the real (tiny, CPU) engine: chat template -> tokenize ->
    prefill/decode -> detokenize -> JSON extraction -> validation -> bind.  Forced decode makes the
    random-init model emit a valid answer, so every pod is an LLM decision, not a fallback."""
    from k8s_llm_scheduler_amd.control.backends import LocalEngineBackend
    from k8s_llm_scheduler_amd.engine import build_engine

    eng = build_engine("tiny", device="cpu", max_batch=4, max_model_len=1024, num_blocks=256, seed=1)
    api = cluster(run_bound_pods=True)
    pods = ai_test_pods(api)
    sched = run_scheduler(api, LocalEngineBackend(eng, forced_answer=first_node_answer), pods, mode=mode, timeout=60)
    st = sched.get_stats()
    assert st["total_scheduled"] == 3 and st["llm_decisions"] == 3 and st["fallback_decisions"] == 0
    assert st["llm_client"]["successful_requests"] == 3
    assert eng.stats["decode_tokens"] > 0 and eng.stats["prefill_tokens"] > 0


def test_continuous_mode_revalidates_concurrent_bindings():
    """Continuous mode: decisions run concurrently against snapshots taken before each other's
    bindings; the bind step re-checks the node (pod limit 1 here) and falls back per pod."""
    api = FakeKubeAPI([make_node("small", pods="1"), make_node("big", pods="110")])
    pods = [make_pod(f"c{i}") for i in range(4)]
    sched = run_scheduler(api, ScriptedBackend(default='{"selected_node": "small"}'), pods, mode="continuous")
    nodes = [api.get_pod("default", p["metadata"]["name"])["spec"]["nodeName"] for p in pods]
    assert nodes.count("small") == 1 and nodes.count("big") == 3
    st = sched.get_stats()
    assert st["total_scheduled"] == 4 and st["llm_decisions"] == 1 and st["fallback_decisions"] == 3


def test_informer_resync_drops_pods_deleted_while_no_stream_was_open():
    """a pod deleted while the watch was down (no DELETED event ever seen) must leave the
    informer counts at the next stream's LIST instead of inflating the node's usage for good."""
    api = cluster()
    api.create_pod(make_pod("ghost", node_name="kind-worker", phase="Running"))
    svc, _ = service(None)
    sched = CustomScheduler("ai-llama-scheduler", api, svc, watch_timeout=1, snapshot_mode="informer")

    def count():
        return {n.name: n.pod_count for n in sched.context_manager.get_node_metrics()}["kind-worker"]

    async def main():
        task = asyncio.create_task(sched.start())
        t0 = time.time()
        while count() != 1 and time.time() - t0 < 5:
            await asyncio.sleep(0.02)
        assert count() == 1
        with api._lock:                  # deleted behind the watch's back: no DELETED event
            api._pods.pop("default/ghost")
        api.stop_watches()               # the stream ends; the next one starts with a LIST
        t0 = time.time()
        while count() != 0 and time.time() - t0 < 5:
            await asyncio.sleep(0.02)
        sched.stop()
        await asyncio.wait_for(task, 5)

    asyncio.run(main())
    assert count() == 0
