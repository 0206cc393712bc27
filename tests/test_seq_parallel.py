"""Sequence-parallel TP prefill (``LlamaModel._layers_folded_sp``, SURVEY 2.6 P-SP) on CPU over gloo: the residual
stream as row shards, reduce-scatter + all-gather instead of each all-reduce, must reproduce the all-reduce
prefill -- logits, the K/V it writes, and the engine's tokens -- including chunks whose length does not divide by
the TP degree (zero pad rows)."""

import os

import pytest
import torch

from mp_harness import run_ranks
from test_prefill_overlap import _run_chunk


def _cpu_rank(rank, world):
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine
    from k8s_llm_scheduler_amd.models.config import PRESETS
    from k8s_llm_scheduler_amd.models.llama import LlamaModel
    from k8s_llm_scheduler_amd.parallel import TPGroup

    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tp = TPGroup(rank, world, dist.group.WORLD, "gloo")
        m = LlamaModel(PRESETS["tiny"], tp, device="cpu", seed=3, max_model_len=512)
        out = {}
        for mode in ("0", "1"):
            os.environ["K8S_SEQ_PARALLEL"] = mode
            assert m.seq_parallel_at(30) == (mode == "1")
            out[mode] = _run_chunk(m, 0)          # a 160-token two-sequence chunk after a 30-token prefix
        (lg0, kv0), (lg1, kv1) = out["0"], out["1"]
        diffs = [float((lg0.float() - lg1.float()).abs().max()), float((kv0.float() - kv1.float()).abs().max()),
                 float(lg0.float().abs().max())]
        prompts = [" ".join(f"pod-{i} gpu {i % 3}" for i in range(12)),
                   " ".join(f"rack-{i} disk {i % 9}" for i in range(13))]
        toks = []
        for mode in ("1", "0"):
            os.environ["K8S_SEQ_PARALLEL"] = mode
            eng = build_engine("tiny", tp=TPGroup(rank, world, dist.group.WORLD, "gloo"), device="cpu", max_batch=2,
                               max_model_len=512, num_blocks=64, seed=1)
            toks.append([o.token_ids for o in eng.generate(prompts, SamplingParams(max_tokens=4, temperature=0.0,
                                                                                   ignore_eos=True))])
        return diffs, toks
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_seq_parallel_prefill_matches_all_reduce_gloo(world):
    # world 4: the 30-token prefix chunk does not divide by 4 -> two zero pad rows
    res = run_ranks(_cpu_rank, world, env={"K8S_SEQ_PARALLEL_MIN": "16", "K8S_PREFILL_OVERLAP": "0"}, timeout_s=300)
    for r in range(world):
        (d_lg, d_kv, scale), (sp_toks, plain_toks) = res[r]
        assert d_kv <= 1e-2, res[r]
        assert d_lg <= 1e-2 * scale + 1e-2, res[r]
        assert sp_toks == plain_toks == res[0][1][0]


def test_reduce_scatter_rows_single_rank_and_shapes():
    from k8s_llm_scheduler_amd.parallel import TPGroup

    tp = TPGroup()
    t = torch.arange(12.0).view(6, 2)
    assert torch.equal(tp.reduce_scatter_rows(t.clone(), residual=torch.ones(6, 2)), t + 1)
    assert torch.equal(tp.all_gather_rows(t), t)
    sim = TPGroup(rank=0, world=3, simulate=True)
    assert tuple(sim.reduce_scatter_rows(t.clone()).shape) == (2, 2)
    assert tuple(sim.all_gather_rows(t[:2]).shape) == (6, 2)
    with pytest.raises(ValueError):
        sim.reduce_scatter_rows(torch.zeros(7, 2))
