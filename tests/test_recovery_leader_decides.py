"""Recovery decisions that must be the same on every rank of a TP replica:

- the RCCL communicator rebuild: a follower whose own communicator looks healthy still aborts it and joins the
  rebuild that the leader's aborted communicator needs, so the unique-id broadcast and the init line up
  (a fake RcclComm stands in for the native one; the sequence of gloo collectives is the real one);
- a request rejected at admission (it cannot fit an empty KV cache): the followers, which replay the leader's
  schedule, finish it as an error too and keep serving instead of leaving their loop."""

from mp_harness import run_ranks


class _FakeRccl:
    made = []

    def __init__(self, world, rank, uid, aborted=False):
        self.world, self.rank, self.uid, self.aborted = world, rank, uid, aborted
        _FakeRccl.made.append(self)

    @staticmethod
    def unique_id():
        return b"uid-from-the-leader"

    def abort(self):
        self.aborted = True

    def async_error(self):
        return ""


def _rebuild_rank(rank, world):
    import torch.distributed as dist

    from k8s_llm_scheduler_amd import ops
    from k8s_llm_scheduler_amd.parallel import init_from_env, make_control_channel

    tp = init_from_env("cpu", backend="gloo")
    control = make_control_channel(tp)

    class _Native:
        RcclComm = _FakeRccl

    ops.native = lambda: _Native()          # this rank process only
    old = _FakeRccl(world, rank, b"old", aborted=(rank == 0))   # only the leader's communicator was aborted
    tp.rccl = old
    tp.reset_collectives(control, timeout_s=30)
    out = dict(old_aborted=old.aborted, rebuilt=tp.rccl is not old, uid=tp.rccl.uid, failed=tp.failed)
    dist.barrier()
    dist.destroy_process_group()
    return out


def test_rccl_rebuild_is_decided_for_the_whole_replica():
    res = run_ranks(_rebuild_rank, 2, timeout_s=120)
    for r in (0, 1):
        assert res[r]["rebuilt"] and res[r]["old_aborted"], res
        assert res[r]["uid"] == b"uid-from-the-leader" and res[r]["failed"] is None


def _reject_rank(rank, world):
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.engine import build_engine
    from k8s_llm_scheduler_amd.engine.sampling import SamplingParams
    from k8s_llm_scheduler_amd.parallel import init_from_env, make_control_channel

    tp = init_from_env("cpu", backend="gloo")
    control = make_control_channel(tp)
    eng = build_engine("tiny", tp=tp, device="cpu", max_batch=2, max_model_len=512, num_blocks=64, seed=1,
                       control=control, watchdog_s=5.0)

    class _Tight:   # a KV cache that cannot hold a 300-token prompt even when empty (on every rank alike)
        def __init__(self, a):
            self._a = a

        def can_allocate(self, tokens, total):
            return len(tokens) < 200 and self._a.can_allocate(tokens, total)

        def __getattr__(self, k):
            return getattr(self._a, k)

    eng.allocator = _Tight(eng.allocator)
    out = {}
    if rank == 1:
        eng.serve_worker()                     # returns only on the leader's stop command
        out = dict(ready=eng.ready, left=len(eng.requests))
    else:
        from k8s_llm_scheduler_amd.engine.engine import RequestRejected

        try:
            eng.generate([list(range(1, 300))], SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))
            big = "served"
        except RequestRejected:
            big = "rejected"
        ok = eng.generate([list(range(1, 40))], SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
        out = dict(big=big, ok=ok[0].finish_reason, n=len(ok[0].token_ids))
        eng.shutdown_workers()
    dist.barrier()
    dist.destroy_process_group()
    return out


def test_follower_finishes_a_rejected_request_and_keeps_serving():
    res = run_ranks(_reject_rank, 2, timeout_s=180)
    assert res[0]["big"] == "rejected" and res[0]["ok"] == "length" and res[0]["n"] == 4, res
    assert res[1]["ready"], res


def _vote_rank(rank, world):
    import time

    import torch.distributed as dist

    from k8s_llm_scheduler_amd.parallel import init_from_env, make_control_channel
    from k8s_llm_scheduler_amd.parallel.comm import CollectiveError

    tp = init_from_env("cpu", backend="gloo")
    control = make_control_channel(tp)
    both = control.any_rank(rank == 1, timeout_s=30)        # every rank votes: the flag of any rank wins
    out = dict(both=both, raised=False, took=0.0)
    if rank == 0:                                            # rank 1 "died" after the barrier: it never votes
        t0 = time.monotonic()
        try:
            control.any_rank(False, timeout_s=2)
        except CollectiveError:
            out["raised"] = True
        out["took"] = time.monotonic() - t0
    dist.barrier()
    # rank 0's failed vote advanced only ITS round counter; the next reset generation (bumped by the leader)
    # restarts the rounds on every rank, so the ranks vote in the same round again -- and finished rounds leave no keys
    if rank == 0:
        control.request_reset()
    dist.barrier()
    out["after"] = control.any_rank(rank == 0, timeout_s=30)
    st = control.store()
    out["first_round_keys_left"] = st.check([f"k8s_vote/0/0.1/{r}" for r in range(world)])
    dist.barrier()
    dist.destroy_process_group()
    return out


def test_recovery_vote_is_bounded():
    """the RCCL-rebuild vote after the monitored barrier is bounded by the recovery timeout (a store
    vote), so a rank that dies between the two cannot park the others for the group's default timeout."""
    res = run_ranks(_vote_rank, 2, timeout_s=120)
    assert res[0]["both"] and res[1]["both"]
    assert res[0]["raised"] and res[0]["took"] < 10
    assert res[0]["after"] and res[1]["after"]
    assert not res[0]["first_round_keys_left"] and not res[1]["first_round_keys_left"]
