"""TP > 1 prefill as two micro-batches whose all-reduces overlap the other half's GEMMs
(``LlamaModel._layers_folded_overlap``, ``engine.split_prefill_meta``).  On CPU the split runs without
streams (``K8S_PREFILL_OVERLAP=cpu``) over gloo: the half metadata must reproduce the unsplit chunk."""

import os

import torch

from k8s_llm_scheduler_amd.engine.engine import split_prefill_meta

from mp_harness import run_ranks


def test_split_meta_straddling_sequence():
    # two sequences: 90 tokens (context 90) and 70 tokens continuing a 30-token prefix (context 100)
    h0, h1 = split_prefill_meta([0, 90, 160], [90, 100], 80)
    assert h0 == ([0, 80], [80], [0])                 # seq 0's first 80 tokens, its context ends at 80
    assert h1 == ([0, 10, 80], [90, 100], [0, 1])     # seq 0's last 10 tokens, then all of seq 1


def test_split_meta_on_a_boundary_and_single_sequence():
    h0, h1 = split_prefill_meta([0, 64, 128], [64, 64], 64)
    assert h0 == ([0, 64], [64], [0]) and h1 == ([0, 64], [64], [1])
    h0, h1 = split_prefill_meta([0, 200], [300], 96)    # one sequence after a 100-token prefix
    assert h0 == ([0, 96], [196], [0]) and h1 == ([0, 104], [300], [0])


def _chunk():
    """Sequence A: 90 fresh tokens; sequence B: 70 tokens after a 30-token prefix already in the cache."""
    a = [(i * 37 + 11) % 5000 + 3 for i in range(90)]
    b = [(i * 53 + 7) % 5000 + 3 for i in range(100)]
    return a, b


def _run_chunk(m, split_at, bs=16):
    """Prefill B's prefix, then the two-sequence chunk; returns (logits, kv cache).  ``split_at`` 0: unsplit."""
    i32 = lambda x: torch.tensor(x, dtype=torch.int32, device=m.device)   # noqa: E731
    m.allocate_kv(64, bs)
    a, b = _chunk()
    blocks_a, blocks_b = list(range(0, 8)), list(range(8, 16))
    bt = torch.zeros(2, 16, dtype=torch.int32)
    bt[0, :8] = torch.tensor(blocks_a)
    bt[1, :8] = torch.tensor(blocks_b)
    bt = bt.to(m.device)
    slot = lambda blocks, p: blocks[p // bs] * bs + p % bs   # noqa: E731
    # B's prefix (30 tokens), unsplit
    m.forward_prefill(i32(b[:30]), i32(list(range(30))), i32([slot(blocks_b, p) for p in range(30)]), i32([0, 30]),
                      i32([30]), bt[1:2].contiguous(), 30, i32([29]))
    ids = a + b[30:]
    pos = list(range(90)) + list(range(30, 100))
    slots = [slot(blocks_a, p) for p in range(90)] + [slot(blocks_b, p) for p in range(30, 100)]
    cu, ctx = [0, 90, 160], [90, 100]
    split = None
    if split_at:
        halves = []
        for c_h, x_h, seqs in split_prefill_meta(cu, ctx, split_at):
            halves.append((i32(c_h), i32(x_h), bt.index_select(0, torch.tensor(seqs, device=m.device)),
                           max(q - p for p, q in zip(c_h, c_h[1:]))))
        split = (split_at, halves[0], halves[1])
    lg = m.forward_prefill(i32(ids), i32(pos), i32(slots), i32(cu), i32(ctx), bt, 90, i32([89, 159]), split=split)
    return lg, m.kv_cache.clone()


def _cpu_rank(rank, world):
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.models.config import PRESETS
    from k8s_llm_scheduler_amd.models.llama import LlamaModel
    from k8s_llm_scheduler_amd.parallel import TPGroup

    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = LlamaModel(PRESETS["tiny"], TPGroup(rank, world, dist.group.WORLD, "gloo"), device="cpu", seed=3,
                       max_model_len=512)
        assert m.prefill_overlap
        lg0, kv0 = _run_chunk(m, 0)
        lg1, kv1 = _run_chunk(m, 80)
        out = [float((lg0.float() - lg1.float()).abs().max()), float((kv0.float() - kv1.float()).abs().max()),
               float(lg0.float().abs().max())]
        # the engine's eager varlen chunk of two prompts (229 tokens: split at 112), with and without the split
        from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine

        prompts = [" ".join(f"pod-{i} gpu {i % 3}" for i in range(12)),
                   " ".join(f"rack-{i} disk {i % 9}" for i in range(12))]
        toks = []
        for mode in ("cpu", "0"):
            os.environ["K8S_PREFILL_OVERLAP"] = mode
            eng = build_engine("tiny", tp=TPGroup(rank, world, dist.group.WORLD, "gloo"), device="cpu", max_batch=2,
                               max_model_len=512, num_blocks=64, seed=1)
            toks.append([o.token_ids for o in eng.generate(prompts, SamplingParams(max_tokens=4, temperature=0.0,
                                                                                   ignore_eos=True))])
            assert eng.stats["prefill_overlap_chunks"] == (mode == "cpu"), eng.stats
        return out, toks
    finally:
        dist.destroy_process_group()


def test_split_prefill_matches_unsplit_tp2_gloo():
    res = run_ranks(_cpu_rank, 2, env={"K8S_PREFILL_OVERLAP": "cpu", "K8S_PREFILL_OVERLAP_MIN": "128"}, timeout_s=300)
    for r in range(2):
        (d_lg, d_kv, scale), (split_toks, plain_toks) = res[r]
        assert d_kv <= 1e-2, res[r]                     # every token's K/V written once, at its own slot
        assert d_lg <= 1e-2 * scale + 1e-2, res[r]
        assert split_toks == plain_toks == res[0][1][0]
