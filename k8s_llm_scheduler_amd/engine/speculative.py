"""Prompt-lookup speculative decoding: n-gram drafts from the sequence's own history, verified in one (graph-
replayed) forward per step while few sequences decode.  Mixed into :class:`~.engine.LLMEngine`.  The reference's JSON
answers copy node names from the prompt (``/root/reference/scheduler.py:407-424``), which is what the drafter exploits."""

from __future__ import annotations

import time
from typing import List

import torch

from .. import ops
from .common import SPEC_GRAPH_T, SPEC_MAX_BATCH, ngram_draft, Request


class SpeculativeMixin:
    """Prompt-lookup speculative decoding steps."""

    # ------------------------------------------------------------------ speculative decoding
    def _spec_ok(self) -> bool:
        return (self.speculative_tokens > 0 and 0 < len(self.running) <= SPEC_MAX_BATCH
                and all(r.params.forced_output_ids is None for r in self.running.values()))

    def _emit(self, r: Request, tkn: int) -> None:
        """Append one generated token to ``r`` with the stop checks of the decode path."""
        r.output_ids.append(tkn)
        self.stats["decode_tokens"] += 1
        if not self._stopped(r, tkn) and len(r.output_ids) >= r.params.max_tokens:
            self._finish(r, "length")

    def _spec_decode(self) -> List[Request]:
        """One prompt-lookup speculative step for every running sequence (no counterpart in the reference, whose
        provider decodes; SURVEY 3.6 decode loop).  Each sequence feeds its last token plus up to
        ``speculative_tokens`` drafted ones (``ngram_draft`` over prompt + answer) through ONE varlen forward over
        the paged cache (``forward_prefill`` with logits at every row), the sampler draws the token after every
        row with the counter of that position -- exactly what the one-token decode step would draw there -- and
        the longest prefix of drafts equal to those draws is accepted, plus the first draw that differs.  So the
        answer is the non-speculative answer (up to the kernels' rounding), in fewer forwards when the drafts hit:
        JSON keys and node names the model copies from the prompt.  K/V written for rejected drafts lies beyond
        the new context length and is overwritten by the next step.  Every TP rank drafts from the same host
        state and draws the same tokens, so the ranks stay in lock-step without an exchange."""
        t0 = time.perf_counter()
        finished: List[Request] = []
        dev = self.device
        fresh = [r for r in self.running.values() if not r.output_ids]
        if fresh:                         # first tokens, sampled by the prefill
            first = self._fetch(self.s_hist[:, 0].contiguous(), what="first tokens")[0].clone()
            for r in fresh:
                self._emit(r, int(first[r.slot]))
                if r.finished:
                    finished.append(r)
        rows = []
        for r in list(self.running.values()):
            seq = r.prompt_ids + r.output_ids
            p = len(seq) - 1              # position of the last token, whose K/V is not in the cache yet
            k = min(self.speculative_tokens, r.params.max_tokens - len(r.output_ids) - 1,
                    self.max_model_len - len(seq))
            rows.append((r, [seq[-1]] + ngram_draft(seq, k), p))
        if rows and all(len(fed) == 1 for _, fed, _ in rows):
            # nothing to verify: one step of the captured decode graph (the host stays current for drafting)
            self.stats["decode_time"] += time.perf_counter() - t0
            return finished + self._decode(max_steps=1)
        if rows:
            bs = self.block_size
            ids, pos, slots, cu, ctx = [], [], [], [0], []
            temp, top_p, seeds, ctr = [], [], [], []
            bt = torch.zeros(len(rows), self.max_blocks_per_seq, dtype=torch.int32)
            for i, (r, toks, p) in enumerate(rows):
                n = len(toks)
                ids += toks
                pos += range(p, p + n)
                slots += [r.blocks[q // bs] * bs + q % bs for q in range(p, p + n)]
                cu.append(cu[-1] + n)
                ctx.append(p + n)
                bt[i, :len(r.blocks)] = torch.tensor(r.blocks, dtype=torch.int32)
                temp += [r.params.temperature] * n
                top_p += [r.params.top_p] * n
                seeds += [r.seed] * n
                ctr += range(p + 1, p + n + 1)     # the decode step's sampler counter: the context length
            t = self._dev
            if len(rows) == 1 and self.spec_graph is not None and len(ids) <= SPEC_GRAPH_T:
                # one sequence: replay the captured verify forward (padding rows write K/V to the scratch slot
                # and their draws are ignored)
                r0, fed0, p0 = rows[0]
                pad = SPEC_GRAPH_T - len(ids)
                self._fill_prefill_state(ids, pos, slots, ctx[0], r0.blocks, SPEC_GRAPH_T)
                graph, logits = self.spec_graph
                graph.replay()
                self.stats["spec_graph_replays"] += 1
                temp, top_p, seeds, ctr = temp + temp[-1:] * pad, top_p + top_p[-1:] * pad, seeds + seeds[-1:] * pad, \
                    ctr + [1] * pad
            else:
                logits = self.model.forward_prefill(t(ids), t(pos), t(slots), t(cu), t(ctx),
                                                    self._dev(bt), max(len(x[1]) for x in rows),
                                                    t(list(range(len(ids)))))
            toks = ops.sample(logits, t(temp, torch.float32), t(top_p, torch.float32), t(seeds), t(ctr),
                              shards=logits.shape[0], nucleus=self._wants_nucleus(r for r, _, _ in rows),
                              tp=self.model.tp)
            self.model.tp.snapshot_health()
            drawn = self._fetch(toks, what="speculative verify")[0].tolist()
            self.model.tp.check_health()
            self.stats["spec_steps"] += 1
            i = 0
            for r, fed, p in rows:
                n = len(fed)
                emit = []
                for j in range(n):
                    emit.append(drawn[i + j])
                    if j + 1 >= n or fed[j + 1] != drawn[i + j]:
                        break
                i += n
                self.stats["spec_drafted"] += n - 1
                self.stats["spec_accepted"] += len(emit) - 1
                for tkn in emit:
                    self._emit(r, tkn)
                    if r.finished:
                        break
                if r.finished:
                    finished.append(r)
                    continue
                # device decode state of the slot, as the one-token decode path leaves it
                slot = r.slot
                self.s_tokens[slot:slot + 1].fill_(r.output_ids[-1])     # fill_: no pageable host copy
                self.s_ctx[slot:slot + 1].fill_(len(r.prompt_ids) + len(r.output_ids))
                self.s_steps[slot:slot + 1].fill_(len(r.output_ids))
        self.stats["decode_steps"] += 1
        self.stats["decode_time"] += time.perf_counter() - t0
        if self.metrics is not None:
            self.metrics.engine_tokens(sum(len(r.output_ids) for r in finished), self.kv_utilization())
        return finished
