"""Engine-side failure detection: a peer that stops taking part in the
tensor-parallel collectives makes the xGMI kernels time out; the error word rides on the engine's own
per-step synchronisation, the engine raises, and the decision service retries, counts the failure and
falls back -- instead of decoding from partial all-reduce sums.

Two ranks share the one test GPU (gloo process group, xGMI peer-memory collectives, as in
test_xgmi_gpu.py); rank 1 builds its engine and then stops participating."""

import pytest
import torch

from mp_harness import run_ranks

pytestmark = pytest.mark.gpu


def _rank(rank, world):
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.control import DecisionService, LocalEngineBackend
    from k8s_llm_scheduler_amd.control.breaker import CircuitBreaker
    from k8s_llm_scheduler_amd.control.prompt import PromptEngine
    from k8s_llm_scheduler_amd.engine import build_engine
    from k8s_llm_scheduler_amd.engine.synthetic import reference_cluster
    from k8s_llm_scheduler_amd.parallel import init_from_env

    tp = init_from_env("cuda", backend="gloo", comm="xgmi")
    assert tp.xgmi is not None
    eng = build_engine("tiny", tp=tp, device="cuda", max_batch=2, max_model_len=512, num_blocks=128, seed=1)
    dist.barrier()
    out = {}
    if rank == 0:
        sleeps = []
        svc = DecisionService(LocalEngineBackend(eng, ignore_eos=True), max_retries=3, max_tokens=8, timeout=120,
                              breaker=CircuitBreaker(5, 60), sleep=sleeps.append)
        nodes, pods = reference_cluster()
        d = svc.decide(PromptEngine().build(pods[0], nodes), pods[0], nodes)
        st = svc.get_stats()
        out = dict(fallback=d.fallback_needed, reasoning=d.reasoning, failed=st["failed_requests"],
                   sleeps=sleeps, breaker_failures=svc.circuit_breaker.failures, tp_failed=tp.failed,
                   node=d.selected_node, nodes=[n.name for n in nodes])
    dist.barrier()     # rank 1 keeps its IPC region mapped until rank 0 is done
    dist.destroy_process_group()
    return out


def test_xgmi_peer_stall_raises_into_retry_breaker_and_fallback():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = run_ranks(_rank, 2, env={"K8S_XGMI_TIMEOUT_S": "0.3", "K8S_TP_COMM": "xgmi"}, timeout_s=300)
    r0 = res[0]
    assert r0["fallback"] and r0["node"] in r0["nodes"], r0
    assert "xGMI collective timed out" in r0["reasoning"], r0["reasoning"]
    assert r0["failed"] == 1 and r0["sleeps"] == [1.0, 2.0], r0
    assert r0["breaker_failures"] == 3 and r0["tp_failed"], r0
