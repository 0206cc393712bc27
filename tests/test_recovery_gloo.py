"""Engine failure recovery across ranks on the CPU (gloo): a follower rank that hits a collective failure reports
it through the process group's store, rank 0 fails its next decision fast (fallback), turns not-ready, and the
next decision resets every rank (control-channel reset command, collectives reset, bounded barrier) and goes
through the engine again (the GPU version with a real stalled xGMI peer is
tests/test_recovery_gpu.py)."""

import time

from mp_harness import run_ranks


def _rank(rank, world):
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.control import DecisionService, LocalEngineBackend
    from k8s_llm_scheduler_amd.control.breaker import CircuitBreaker
    from k8s_llm_scheduler_amd.control.prompt import PromptEngine
    from k8s_llm_scheduler_amd.engine import build_engine
    from k8s_llm_scheduler_amd.engine.synthetic import reference_cluster
    from k8s_llm_scheduler_amd.parallel import init_from_env, make_control_channel

    tp = init_from_env("cpu", backend="gloo")
    control = make_control_channel(tp)
    eng = build_engine("tiny", tp=tp, device="cpu", max_batch=2, max_model_len=512, num_blocks=128, seed=1,
                       control=control, watchdog_s=5.0)
    out = {}
    if rank == 1:
        eng.fault = ("raise", 2, 0.0)   # the second schedule message this follower receives fails
        eng.serve_worker()
        out = dict(health=dict(eng.health))
    else:
        svc = DecisionService(LocalEngineBackend(eng, ignore_eos=True), max_retries=3, max_tokens=4, timeout=30,
                              breaker=CircuitBreaker(50, 60), sleep=lambda s: None)
        nodes, pods = reference_cluster()
        prompt = PromptEngine().build(pods[0], nodes)
        d1 = svc.decide(prompt, pods[0], nodes)            # message 1: fine
        ok1 = d1.reasoning
        # message 2 makes rank 1 fail; rank 0 learns it through the store monitor
        time.sleep(0.2)
        d2 = svc.decide(PromptEngine().build(pods[1], nodes), pods[1], nodes)
        deadline = time.monotonic() + 10
        while eng.control.peer_failure() is None and time.monotonic() < deadline:
            time.sleep(0.05)
        saw_peer = eng.control.peer_failure()
        not_ready = not eng.health_probe()[1]          # /readyz turns 503 as soon as the report arrives
        failed_before = svc.get_stats()["failed_requests"]
        # the next decision: attempt 1 fails fast on the peer report, the retry recovers every rank (nothing to
        # drain on the CPU) and runs through the engine
        d3 = svc.decide(PromptEngine().build(pods[2], nodes), pods[2], nodes)
        out = dict(ok1=ok1, d2=d2.reasoning, saw_peer=saw_peer, not_ready=not_ready, d3=d3.reasoning,
                   d3_fallback=d3.fallback_needed, failed_delta=svc.get_stats()["failed_requests"] - failed_before,
                   ready=eng.ready, probe_ready=eng.health_probe()[1], health=dict(eng.health))
        eng.shutdown_workers()
    dist.barrier()
    dist.destroy_process_group()
    return out


def test_follower_failure_reported_then_recovered():
    res = run_ranks(_rank, 2, timeout_s=300)
    r0 = res[0]
    assert r0["saw_peer"] and "injected" in r0["saw_peer"], r0
    assert r0["not_ready"], r0
    assert "JSON" in r0["d3"] or not r0["d3_fallback"], r0    # answered by the engine (random weights: no JSON)
    assert r0["ready"] and r0["probe_ready"] and r0["health"]["recoveries"] == 1, r0
    assert res[1]["health"]["recoveries"] == 1, res[1]
