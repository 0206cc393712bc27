"""Data parallelism over engine replicas on CPU (gloo): WORLD_SIZE = 4 as 2 replicas x TP=2.

Rank 0 runs the router backend (the control plane's view), global rank 2 leads replica 1 and
answers rank 0's share over its link, ranks 1 and 3 follow their leaders' engine schedules.  The
texts must equal those of one TP=1 engine given the same requests (greedy decoding), in request
order, and both replicas must have received work."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from k8s_llm_scheduler_amd.control.backends import LocalEngineBackend
from k8s_llm_scheduler_amd.control.decision import GenerationRequest
from k8s_llm_scheduler_amd.engine import build_engine

SYSTEM = "You are an intelligent Kubernetes scheduler. Respond only with valid JSON."
USERS = [f"pod-{i} needs {i * 100}m cpu; nodes: kind-worker, kind-worker2" for i in range(5)]


def _requests():
    return [GenerationRequest(SYSTEM, u, max_tokens=6, temperature=0.0) for u in USERS]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, tp_size, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from k8s_llm_scheduler_amd.parallel import init_from_env, make_control_channel
    from k8s_llm_scheduler_amd.parallel.replicas import ReplicaRouterBackend, make_replica_links, serve_replica

    try:
        tp = init_from_env("cpu", backend="gloo", tp_size=tp_size)
        control = make_control_channel(tp)
        links = make_replica_links(tp)
        eng = build_engine("tiny", tp=tp, device="cpu", max_batch=4, max_model_len=512, num_blocks=128, seed=1,
                           control=control)
        local = LocalEngineBackend(eng, ignore_eos=True)
        if tp.global_rank == 0:
            router = ReplicaRouterBackend(local, links)
            texts = router.complete(_requests())
            again = router.complete(_requests()[:1])      # a lone request: the next replica in rotation
            batch_dispatch = list(router.dispatched)
            # continuous serving: the local engine runs its background loop, 20 single-pod calls from 8
            # threads -- every call goes to the least-loaded replica
            from concurrent.futures import ThreadPoolExecutor

            from k8s_llm_scheduler_amd.control.scheduler import start_backend_loop

            assert start_backend_loop(router)
            reqs = _requests()
            with ThreadPoolExecutor(8) as ex:
                conc = list(ex.map(lambda i: router.complete([reqs[i % len(reqs)]])[0], range(20)))
            conc_dispatch = [b - a for a, b in zip(batch_dispatch, router.dispatched)]
            eng.stop_background()
            router.shutdown()
            eng.shutdown_workers()
            q.put(("router", texts, again, batch_dispatch, (tp.replica, tp.replicas, tp.world), conc,
                   conc_dispatch))
        elif tp.rank == 0:
            serve_replica(local, links[0], eng)
            q.put(("leader", tp.replica, tp.global_rank))
        else:
            eng.serve_worker()
            q.put(("follower", tp.replica, tp.global_rank))
    except BaseException as e:  # noqa: BLE001
        import traceback

        q.put(("error", rank, traceback.format_exc()))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_two_replicas_of_tp2_match_single_engine():
    eng = build_engine("tiny", device="cpu", max_batch=4, max_model_len=512, num_blocks=128, seed=1)
    want = LocalEngineBackend(eng, ignore_eos=True).complete(_requests())

    world, tp_size = 4, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, tp_size, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
    errors = [g for g in got if g[0] == "error"]
    assert not errors, errors[0][2]
    assert all(p.exitcode == 0 for p in procs)
    router = next(g for g in got if g[0] == "router")
    _, texts, again, dispatched, layout, conc, conc_dispatch = router
    assert layout == (0, 2, 2)
    assert texts == want
    assert again == want[:1]
    assert dispatched == [3, 2 + 1]          # least loaded, ties rotate: 0,1,0,1,0 then the lone one on 1
    assert conc == [want[i % len(want)] for i in range(20)]
    assert min(conc_dispatch) >= 8 and sum(conc_dispatch) == 20, conc_dispatch
    assert sorted(g[0] for g in got) == ["follower", "follower", "leader", "router"]


def test_world_not_multiple_of_tp_is_rejected(monkeypatch):
    from k8s_llm_scheduler_amd.parallel import init_from_env

    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "0")
    with pytest.raises(ValueError):
        init_from_env("cpu", backend="gloo", tp_size=3)


def test_link_failure_fails_pending_and_later_requests():
    """when the link's receive side breaks (remote leader died), every pending share fails instead of
    blocking its caller forever, and later submits fail at once; a remote share that never answers is bounded by
    the call deadline."""
    import threading
    import time as _t

    from k8s_llm_scheduler_amd.control.decision import GenerationRequest
    from k8s_llm_scheduler_amd.parallel.replicas import ReplicaLink, ReplicaRouterBackend

    gate = threading.Event()

    class _Link(ReplicaLink):
        sent = []

        def _bcast(self, obj, src, group):
            if group == "up":          # the receive thread: the peer goes away once a request is out
                gate.wait(10)
                raise RuntimeError("connection reset by peer")
            self.sent.append(obj)
            gate.set()
            return obj

    link = _Link(1, 4, "down", "up")
    fut = link.submit(["req"])
    try:
        fut.result(timeout=10)
        raise AssertionError("a dead link answered")
    except RuntimeError as e:
        assert "link failed" in str(e)
    assert link.dead and link.submit(["again"]).exception(timeout=1) is not None

    class _Silent(ReplicaLink):
        def _bcast(self, obj, src, group):
            if group == "up":
                _t.sleep(30)           # never answers within the test
            return obj

    class _Local:
        def complete(self, reqs):
            return ["local"] * len(reqs)

    router = ReplicaRouterBackend(_Local(), [_Silent(1, 4, "down", "up")])
    router.reply_grace_s = 0.2
    reqs = [GenerationRequest(system="s", user=f"u{i}", max_tokens=4, temperature=0.0, deadline_s=0.5)
            for i in range(2)]
    t0 = _t.monotonic()
    try:
        router.complete(reqs)
        raise AssertionError("expected a deadline error")
    except TimeoutError:
        pass
    assert _t.monotonic() - t0 < 5
    # the timed-out share left the link's pending table and the router's load figure
    assert router.links[0].inflight == 0 and not router.links[0]._pending


def test_idle_link_sends_keepalives_and_leader_answers_them():
    """links are bounded by a gloo timeout (K8S_REPLICA_LINK_TIMEOUT_S) instead of 7 days, so an
    idle link must keep both directions busy: rank 0 pings every quarter of the timeout, the remote leader pongs, and
    rank 0's receive thread drops the pongs."""
    import threading
    import time as _t

    from k8s_llm_scheduler_amd.parallel import replicas as R

    sent, up = [], []
    pong = threading.Event()

    class _Link(R.ReplicaLink):
        def _bcast(self, obj, src, group):
            if group == "up":
                if src == 0:                       # (not used: rank 0 never sends on up)
                    return obj
                pong.wait(5)
                pong.clear()
                return R._PONG
            sent.append(obj)
            return obj

    link = _Link(1, 4, "down", "up", timeout_s=0.2)
    link.start()
    _t.sleep(0.5)
    assert R._PING in sent and not link.dead
    pong.set()
    _t.sleep(0.05)
    assert not link.dead and link.inflight == 0

    # leader side: a ping is answered on the up link and never reaches the engine
    class _Leader(R.ReplicaLink):
        msgs = [R._PING, R._STOP]

        def receive(self):
            return self.msgs.pop(0)

        def reply(self, payload):
            up.append(payload)

    class _Backend:
        def complete(self, reqs):
            raise AssertionError("a keepalive reached the engine")

    R.serve_replica(_Backend(), _Leader(1, 4, "down", "up"), engine=None, workers=1)
    assert up == [R._PONG, R._STOP]
    link._closing.set()


def _idle_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), K8S_REPLICA_LINK_TIMEOUT_S="2")
    torch.set_num_threads(1)
    import time as _t

    from k8s_llm_scheduler_amd.parallel import init_from_env
    from k8s_llm_scheduler_amd.parallel.replicas import ReplicaRouterBackend, make_replica_links, serve_replica

    try:
        tp = init_from_env("cpu", backend="gloo", tp_size=1)
        links = make_replica_links(tp)
        assert links and links[0].timeout_s == 2.0
        eng = build_engine("tiny", tp=tp, device="cpu", max_batch=2, max_model_len=256, num_blocks=64, seed=1)
        local = LocalEngineBackend(eng, ignore_eos=True)
        if tp.global_rank == 0:
            router = ReplicaRouterBackend(local, links)     # no request yet: the link must stay up on its own
            _t.sleep(7.0)                                   # 3.5 x the gloo link timeout, idle
            texts = router.complete(_requests()[:2])        # one request per replica
            disp, dead = list(router.dispatched), links[0].dead
            router.shutdown()
            q.put(("router", texts, disp, dead))
        else:
            serve_replica(local, links[0], eng)
            q.put(("leader",))
    except BaseException:  # noqa: BLE001
        import traceback

        q.put(("error", rank, traceback.format_exc()))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_idle_router_keeps_remote_replica_alive_past_the_link_timeout():
    """a scheduler that sends no pod for longer than the link timeout must not lose its remote
    replicas.  The router starts each link's keepalive when it is built (not on the first submit), so the remote
    leader's receive is answered within a quarter of the timeout from the start; after idling 3.5 timeouts both
    replicas still answer."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_idle_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(60)
    errs = [g for g in got if g[0] == "error"]
    assert not errs, errs
    router = next(g for g in got if g[0] == "router")
    _, texts, disp, dead = router
    assert len(texts) == 2 and disp == [1, 1] and not dead, router
