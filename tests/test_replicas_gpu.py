"""Data parallelism over engine replicas on the GPU (SURVEY 2.6 P-DP): WORLD_SIZE = 4 real rank processes on the one
test GPU as 2 replicas x TP = 2, each replica with its own xGMI peer-memory collectives and captured decode graphs.

Rank 0 deals the batch round-robin over the replicas (``ReplicaRouterBackend``); global rank 2 leads replica 1 and
answers its share over the gloo link; ranks 1 and 3 follow their leaders' schedules.  Every prompt is sent twice in a
row, so both replicas decode the same prompts as the same batch: their texts must agree exactly, and match a TP = 1
engine on the same GPU (greedy; TP = 2 and TP = 1 round differently, so a near-tie may flip a token: 4 of 5)."""

import pytest
import torch

from mp_harness import run_ranks

pytestmark = pytest.mark.gpu

SYSTEM = "You are an intelligent Kubernetes scheduler. Respond only with valid JSON."
USERS = [f"pod-{i} needs {i * 100}m cpu; nodes: kind-worker, kind-worker2" for i in range(5)]


def _requests(dup: int = 1):
    from k8s_llm_scheduler_amd.control.decision import GenerationRequest

    return [GenerationRequest(SYSTEM, u, max_tokens=6, temperature=0.0) for u in USERS for _ in range(dup)]


def _rank(rank, world):
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.control.backends import LocalEngineBackend
    from k8s_llm_scheduler_amd.engine import build_engine
    from k8s_llm_scheduler_amd.parallel import init_from_env, make_control_channel
    from k8s_llm_scheduler_amd.parallel.replicas import ReplicaRouterBackend, make_replica_links, serve_replica

    tp = init_from_env("cuda", backend="gloo", comm="xgmi", tp_size=2)
    assert tp.xgmi is not None and tp.world == 2 and tp.replicas == 2
    control = make_control_channel(tp)
    links = make_replica_links(tp)
    eng = build_engine("tiny", tp=tp, device="cuda", max_batch=8, max_model_len=512, num_blocks=128, seed=1,
                       control=control)
    local = LocalEngineBackend(eng, ignore_eos=True)
    out = {"role": "follower", "graph_replays": 0}
    if tp.global_rank == 0:
        router = ReplicaRouterBackend(local, links)
        out.update(role="router", texts=router.complete(_requests(dup=2)), dispatched=list(router.dispatched))
        # continuous serving: local engine in its background loop, 10 single-pod calls from 5 threads
        from concurrent.futures import ThreadPoolExecutor

        from k8s_llm_scheduler_amd.control.scheduler import start_backend_loop

        assert start_backend_loop(router)
        reqs = _requests()
        before = list(router.dispatched)
        with ThreadPoolExecutor(5) as ex:
            conc = list(ex.map(lambda i: router.complete([reqs[i % 5]])[0], range(10)))
        out.update(conc=conc, conc_dispatch=[b - a for a, b in zip(before, router.dispatched)])
        eng.stop_background()
        router.shutdown()
        eng.shutdown_workers()
    elif tp.rank == 0:
        serve_replica(local, links[0], eng)
        out["role"] = "leader"
    else:
        eng.serve_worker()
    out["graph_replays"] = eng.stats["graph_replays"]
    out["xgmi_err"] = tp.xgmi.error()
    dist.barrier()
    dist.destroy_process_group()
    return out


def test_two_replicas_of_tp2_share_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_scheduler_amd.control.backends import LocalEngineBackend
    from k8s_llm_scheduler_amd.engine import build_engine

    eng = build_engine("tiny", device="cuda", max_batch=8, max_model_len=512, num_blocks=128, seed=1)
    want = LocalEngineBackend(eng, ignore_eos=True).complete(_requests())
    del eng
    res = run_ranks(_rank, 4, env={"K8S_TP_BACKEND": "gloo", "K8S_TP_COMM": "xgmi"}, timeout_s=150)
    assert sorted(r["role"] for r in res.values()) == ["follower", "follower", "leader", "router"]
    assert all(r["xgmi_err"] == 0 for r in res.values())
    assert all(r["graph_replays"] > 0 for r in res.values()), res   # every rank decoded through its graphs
    router = res[0]
    assert router["dispatched"] == [5, 5]            # least loaded, ties rotate: even positions local, odd remote
    assert min(router["conc_dispatch"]) >= 3, router["conc_dispatch"]   # continuous mode: both replicas serve
    texts = router["texts"]
    rep0, rep1 = texts[0::2], texts[1::2]            # the same five prompts on each replica, as the same batch
    assert rep0 == rep1
    assert sum(a == b for a, b in zip(rep0, want)) >= 4, (rep0, want)
    conc = router["conc"]
    assert sum(conc[i] in (rep0[i % 5], rep1[i % 5]) for i in range(10)) >= 8, (conc, rep0)
    print(f"2 replicas x TP=2 on one GPU: replica texts identical, {sum(a == b for a, b in zip(rep0, want))}/5 "
          f"equal to TP=1")
