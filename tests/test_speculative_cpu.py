"""Prompt-lookup speculative decoding (engine.speculative_tokens, LLMEngine._spec_decode) on CPU.

Exactness: every emitted token is the sampler's token for its position, so the answers equal the one-token decode
path's.  Acceptance: a model whose next token is a fixed function of the current one (a 5-token cycle, forced on
top of the tiny Llama's logits) repeats itself, so drafts copied from earlier in the answer are accepted and the
answer needs far fewer forwards than tokens."""

import pytest
import torch

from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine
from k8s_llm_scheduler_amd.engine.engine import LLMEngine, ngram_draft
from k8s_llm_scheduler_amd.engine.tokenizer import Tokenizer
from k8s_llm_scheduler_amd.models.config import PRESETS
from k8s_llm_scheduler_amd.models.llama import LlamaModel


def test_ngram_draft():
    assert ngram_draft([1, 2, 3, 4, 5, 1, 2, 3], 3) == [4, 5, 1]        # longest suffix first (n = 3)
    assert ngram_draft([1, 2, 3, 4, 5, 9, 2, 3], 3) == [4, 5, 9]        # falls back to n = 2
    assert ngram_draft([7, 8, 9], 3) == []
    assert ngram_draft([256, 1, 256, 1, 256], 2) == [1, 256]            # byte search stays token-aligned
    assert ngram_draft([1, 2, 1, 2], 0) == []


class CycleModel(LlamaModel):
    """Tiny Llama whose sampled next token is 10 + (t - 9) % 5 for t in 10..14 (10 otherwise): the real forward
    runs (paged KV, attention, GEMMs), then the logits are replaced by a near one-hot of that rule."""

    def _force(self, logits, inputs):
        out = torch.full_like(logits, -30.0)
        if logits.shape[0] == 1 and self.tp.world > 1 and self.tp.rank != 0:
            return out                                  # this rank's vocab shard (vocab-parallel): ids >= Vs only
        t = inputs.long().to(logits.device)
        nxt = torch.where((t >= 10) & (t < 15), 10 + (t - 9) % 5, torch.full_like(t, 10))
        out[0].scatter_(1, nxt.view(-1, 1), 30.0)      # capturable (no host index or value tensors)
        return out

    def forward_prefill(self, ids, positions, slot_mapping, cu_q, context_lens, block_tables, max_qlen, last_idx,
                        split=None):
        lg = super().forward_prefill(ids, positions, slot_mapping, cu_q, context_lens, block_tables, max_qlen,
                                     last_idx, split=split)
        return self._force(lg, ids[last_idx.long()])

    def forward_decode(self, tokens, context_lens, block_tables, max_context):
        return self._force(super().forward_decode(tokens, context_lens, block_tables, max_context), tokens)


def _cycle_engine(spec):
    m = CycleModel(PRESETS["tiny"], device="cpu", seed=1, max_model_len=512)
    return LLMEngine(m, Tokenizer(None, model_vocab=m.cfg.vocab), max_batch=4, num_blocks=64, max_model_len=512,
                     cuda_graphs=False, seed=1, speculative_tokens=spec)


@pytest.mark.parametrize("temperature", [0.0, 0.7])
def test_speculative_accepts_drafts_and_matches_plain_decode(temperature):
    prompts = [[3, 4, 5, 6, 7], [100, 101, 102]]
    params = SamplingParams(max_tokens=40, temperature=temperature, seed=11, ignore_eos=True)
    plain = _cycle_engine(0)
    want = [o.token_ids for o in plain.generate(prompts, params)]
    spec = _cycle_engine(4)
    got = [o.token_ids for o in spec.generate(prompts, params)]
    assert got == want
    assert want[0][:6] == [10, 11, 12, 13, 14, 10]
    st = spec.stats
    assert st["spec_accepted"] >= 50, st                # the cycle is drafted from the answer's own history
    assert st["spec_steps"] <= 20, st                   # 40 tokens per sequence in far fewer forwards
    assert st["decode_tokens"] == plain.stats["decode_tokens"] == 80


def test_speculative_matches_plain_decode_on_random_weights():
    """Random weights: drafts are rare (steps without any fall back to the one-token decode step) and rarely
    accepted; the answers must still be the plain decode's (greedy and sampled, two sequences decoding together)."""
    prompts = ["node-1 node-2 node-3 node-1 node-2 pick a node", "selected_node confidence reasoning {"]
    for temperature in (0.0, 0.8):
        params = SamplingParams(max_tokens=23, temperature=temperature, seed=5, ignore_eos=True)
        outs = []
        for spec in (0, 4):
            eng = build_engine("tiny", device="cpu", max_batch=4, max_model_len=512, num_blocks=64, seed=1,
                               speculative_tokens=spec)
            outs.append([o.token_ids for o in eng.generate(prompts, params)])
        assert outs[0] == outs[1]
        assert all(len(t) == 23 for t in outs[1])
