"""Vocab-parallel sampling on CPU: each TP rank samples its own vocabulary shard with noise keyed
by the global token id; the ranks exchange the row max and two integer bin histograms (top-p rows) and one best key
per row, instead of all-gathering rows x vocab fp32 logits.  The tokens must be those of the gathered path, bit for
bit: greedy, temperature sampling and top-p, single and batched, mixed prefill + decode steps, at TP = 2 and 4."""

import os
import threading

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from k8s_llm_scheduler_amd.ops import reference as ref

from test_tp_gloo import _free_port


def _thread_gather(world):
    """gather(t) for ``world`` threads standing in for ranks (one call per rank, in the same order on every rank)."""
    barrier = threading.Barrier(world)
    box, lock = {}, threading.Lock()

    def make(rank):
        n = [0]

        def gather(t):
            i = n[0]
            n[0] += 1
            with lock:
                box.setdefault(i, {})[rank] = t.clone()
            barrier.wait()
            out = torch.stack([box[i][r] for r in range(world)])
            barrier.wait()
            return out
        return gather
    return make


@pytest.mark.parametrize("world", [2, 4, 8])
def test_reference_vocab_parallel_equals_gathered(world):
    g = torch.Generator().manual_seed(world)
    B, V = 7, 4096
    L = torch.randn(B, V, generator=g) * 3
    L[3, 5:] -= 40.0                       # a peaked row: every other shard holds no nucleus token
    L[4, 100] = L[4, 3000] = 50.0          # a greedy tie across shards: the lowest id wins
    T = torch.tensor([0.0, 0.3, 0.8, 0.3, 0.0, 1.0, 0.7])
    P = torch.tensor([1.0, 1.0, 0.9, 0.5, 1.0, 0.95, 0.2])
    S = torch.arange(1, B + 1)
    C = torch.arange(10, 10 + B)
    want = ref.sample(L, T, P, S, C)
    assert int(want[4]) == 100
    Vs = V // world
    make = _thread_gather(world)
    got = {}

    def run(r):
        got[r] = ref.sample_vocab_parallel(L[:, r * Vs:(r + 1) * Vs], T, P, S, C, r, make(r))

    ths = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for r in range(world):
        assert torch.equal(got[r], want), (r, got[r], want)


def _engine_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine
        from k8s_llm_scheduler_amd.parallel import TPGroup

        tp = TPGroup(rank, world, dist.group.WORLD, "gloo")
        prompts = ["vocab parallel", "second request here", "x", "a longer fourth prompt about nodes"]
        params = [SamplingParams(max_tokens=9, temperature=0.0, ignore_eos=True),
                  SamplingParams(max_tokens=9, temperature=0.3, seed=5, ignore_eos=True),
                  SamplingParams(max_tokens=9, temperature=0.8, top_p=0.9, seed=7, ignore_eos=True),
                  SamplingParams(max_tokens=9, temperature=1.0, top_p=0.5, seed=8, ignore_eos=True)]
        res = {}
        for vp in ("1", "0"):
            os.environ["K8S_VOCAB_PARALLEL"] = vp
            eng = build_engine("tiny", tp=tp, device="cpu", max_batch=4, max_model_len=256, num_blocks=96, seed=1)
            assert eng.vocab_parallel == (vp == "1") and eng.model.gather_logits == (vp == "0")
            batched = [o.token_ids for o in eng.generate(prompts, params)]
            # mixed steps: a request arriving while another decodes rides the decode rows through the prefill
            long = [SamplingParams(**{**q.__dict__, "max_tokens": 24}) for q in params]
            reqs = [eng.add_request(prompts[0], long[1])]
            eng.step()
            eng.step()
            reqs.append(eng.add_request(prompts[3], long[3]))
            while eng.has_work():
                eng.step()
            res[vp] = (batched, [r.output_ids for r in reqs], eng.stats["mixed_steps"])
        q.put((rank, res))
    except BaseException as e:  # noqa: BLE001
        import traceback

        q.put((rank, traceback.format_exc()))
        raise e
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_engine_vocab_parallel_tokens_equal_gathered(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
    for r, v in got.items():
        assert isinstance(v, dict), f"rank {r}:\n{v}"
    r0 = got[0]
    batched, mixed, n_mixed = r0["1"]
    assert n_mixed >= 1
    assert (batched, mixed) == r0["0"][:2], "vocab-parallel tokens differ from the gathered path"
    assert all(len(t) == 9 for t in batched)
    assert all(got[r] == r0 for r in range(world)), "ranks drew different tokens"


@pytest.mark.parametrize("tp", [2, 4, 8])
def test_decode_buckets_capture_only_xgmi_sized_collectives(tp):
    """a decode bucket is captured only when all of its collectives fit the xGMI transports.  At
    Llama-3.3-70B shapes the gathered fp32 logits of 64 rows are 16.4 MB per rank at TP = 2 and 8.2 MB at TP = 4 --
    past the default slot, so those buckets used to capture an RCCL / gloo all-gather; with vocab-parallel sampling
    the largest sampling exchange is a 2 KiB histogram per row and every bucket fits."""
    from types import SimpleNamespace

    from k8s_llm_scheduler_amd.engine.common import BUCKETS
    from k8s_llm_scheduler_amd.engine.engine import LLMEngine
    from k8s_llm_scheduler_amd.parallel.comm import TPGroup, default_slot_bytes

    slot = default_slot_bytes(tp)
    group = TPGroup(0, tp, None, "nccl", xgmi=SimpleNamespace(slot_bytes=slot, max_allreduce_bytes=tp * slot))
    for gather in (True, False):
        model = SimpleNamespace(tp=group, cfg=SimpleNamespace(hidden=8192), lm_head=torch.empty(128256 // tp, 1),
                                gather_logits=gather)
        fake = SimpleNamespace(model=model)
        ok = {B: LLMEngine._decode_bucket_capturable(fake, B) for B in BUCKETS}
        if gather:
            assert ok[64] == (64 * (128256 // tp) * 4 <= slot), (tp, ok)
            if tp < 8:
                assert not ok[64]
        else:
            assert all(ok.values()), (tp, ok)
            assert 64 * 256 * 8 <= 1 << 20     # no sampling exchange above the 64-row residual all-reduce
