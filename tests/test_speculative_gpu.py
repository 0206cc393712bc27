"""Prompt-lookup speculative decoding on the GPU: the verify forward runs the hand-written prefill kernels
(mgemm / GEMV, paged prefill attention) over several rows per sequence and the multi-workgroup sampler over every
row; the answers must equal the captured one-token decode graphs' answers, with the drafts accepted."""

import pytest
import torch

from test_speculative_cpu import CycleModel

pytestmark = pytest.mark.gpu


def _engine(spec, graphs):
    from k8s_llm_scheduler_amd.engine.engine import LLMEngine
    from k8s_llm_scheduler_amd.engine.tokenizer import Tokenizer
    from k8s_llm_scheduler_amd.models.config import PRESETS

    m = CycleModel(PRESETS["tiny"], device="cuda", seed=1, max_model_len=512)
    eng = LLMEngine(m, Tokenizer(None, model_vocab=m.cfg.vocab), max_batch=4, num_blocks=64, max_model_len=512,
                    cuda_graphs=graphs, seed=1, speculative_tokens=spec)
    eng.capture_graphs()
    return eng


@pytest.mark.parametrize("temperature", [0.0, 0.7])
def test_speculative_gpu_matches_graph_decode(temperature):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_scheduler_amd.engine import SamplingParams

    prompts = [[3, 4, 5, 6, 7], [100, 101, 102], [200, 12]]
    params = SamplingParams(max_tokens=40, temperature=temperature, seed=11, ignore_eos=True)
    plain = _engine(0, True)
    want = [o.token_ids for o in plain.generate(prompts, params)]
    assert plain.stats["graph_replays"] > 0
    spec = _engine(4, True)
    got = [o.token_ids for o in spec.generate(prompts, params)]
    assert got == want
    st = spec.stats
    assert st["spec_accepted"] >= 60 and st["spec_steps"] <= 20, st   # 120 tokens in <= 20 verify forwards


def test_speculative_gpu_single_sequence_replays_verify_graph():
    """One sequence: the verify forward replays its captured graph (SPEC_GRAPH_T rows, padding to the scratch
    slot) and the answer still equals the decode graphs' answer."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k8s_llm_scheduler_amd.engine import SamplingParams

    params = SamplingParams(max_tokens=37, temperature=0.0, ignore_eos=True)
    want = [o.token_ids for o in _engine(0, True).generate([[3, 4, 5, 6, 7]], params)]
    spec = _engine(4, True)
    assert spec.spec_graph is not None
    got = [o.token_ids for o in spec.generate([[3, 4, 5, 6, 7]], params)]
    assert got == want
    st = spec.stats
    assert st["spec_graph_replays"] >= 5 and st["spec_accepted"] >= 20, st
