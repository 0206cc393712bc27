"""Host side of the cascade decode attention (engine._shared_prefix): the running rows' longest common block-list
prefix in 64-token spans, cut at the earliest prompt end, recomputed only when the running set changes; and the
cascade group count the kernels and the host agree on.  The kernels themselves: tests/test_cascade_gpu.py."""

from types import SimpleNamespace

from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.engine.engine import LLMEngine


def _engine(rows):
    eng = SimpleNamespace(block_size=16, _cas_key=None, _cas_val=(0, 0), running={})
    for slot, (rid, prompt_len, blocks) in rows.items():
        eng.running[slot] = SimpleNamespace(slot=slot, rid=rid, prompt_ids=[0] * prompt_len, blocks=list(blocks))
    return eng


def _shared(eng):
    return LLMEngine._shared_prefix(eng)


def test_common_block_prefix_in_spans():
    common = list(range(100, 140))                          # 40 blocks = 640 tokens = 10 spans
    eng = _engine({3: (7, 700, common + [1, 2, 3, 4, 5, 6]), 0: (9, 720, common + [11, 12, 13, 14, 15, 16])})
    assert _shared(eng) == (10, 0)                          # reference slot: the lowest running slot


def test_cut_at_the_earliest_prompt_end():
    common = list(range(100, 160))                          # 60 blocks shared (960 tokens)...
    eng = _engine({0: (1, 500, common + [1]), 1: (2, 990, common + [2])})
    assert _shared(eng) == (500 // 16 * 16 // 64, 0)        # ...but a prompt ends at 500: 31 blocks -> 7 spans


def test_partial_span_and_diverging_rows():
    eng = _engine({0: (1, 800, [5, 6, 7, 8, 9, 1, 2]), 1: (2, 800, [5, 6, 7, 8, 9, 3, 4]),
                   2: (3, 800, [5, 6, 7, 8, 10, 3, 4])})
    assert _shared(eng) == (1, 0)                           # 4 common blocks = 64 tokens = 1 span
    eng = _engine({0: (1, 800, [5, 6, 7]), 1: (2, 800, [8, 6, 7])})
    assert _shared(eng) == (0, 0)


def test_recomputed_only_when_the_running_set_changes():
    eng = _engine({0: (1, 800, list(range(50))), 1: (2, 800, list(range(50)))})
    assert _shared(eng) == (12, 0)
    eng.running[1].blocks[:] = [999] * 50                   # (blocks never change under a running request)
    assert _shared(eng) == (12, 0)                          # cached for the same (slot, rid) set
    eng.running[1] = SimpleNamespace(slot=1, rid=3, prompt_ids=[0] * 800, blocks=list(range(20)) + [7] * 30)
    assert _shared(eng) == (5, 0)                           # a new request in slot 1: recomputed (20 blocks)


def test_group_counts_agree_with_the_kernels():
    for B, nq, nkv in ((2, 64, 8), (16, 64, 8), (64, 64, 8), (64, 8, 1), (8, 32, 8)):
        ngm = ops.cascade_groups_max(B, nq, nkv)
        assert 2 <= ngm <= 32
        for sh in (1, 5, 16, 17, 69, 500):
            spg = -(-sh // ngm)
            groups = -(-sh // spg)
            assert groups <= ngm and (groups - 1) * spg < sh <= groups * spg
    assert ops.cascade_ok(64, 8, 16, 128) and not ops.cascade_ok(64, 8, 32, 128) and not ops.cascade_ok(24, 8, 16, 128)
