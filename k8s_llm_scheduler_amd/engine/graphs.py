"""hipGraph capture of the decode step (per batch bucket x context class x nucleus) and of the bucketed prefill /
speculative-verify forwards, plus the static device state those graphs read.  Mixed into :class:`~.engine.LLMEngine`.
Replaces the per-token remote generation of the reference (``/root/reference/scheduler.py:425-433``)."""

from __future__ import annotations

import gc
import os
from typing import Optional, Sequence

import torch

from .. import ops
from ..utils.tracing import trace
from .common import BUCKETS, PREFILL_GRAPH_BUCKETS, _P_SPLIT, SPEC_GRAPH_T


def logits_exchange_bytes(model, rows: int) -> int:
    """Per-rank bytes of the largest collective the sampling of ``rows`` logits rows issues: the gathered fp32 logits,
    or (vocab-parallel sampling) a top-p row's 256-bin u64 histogram."""
    if getattr(model, "gather_logits", True):
        return rows * model.lm_head.shape[0] * 4
    return rows * 256 * 8


class GraphCaptureMixin:
    """Decode / prefill / verify graph capture and the static state the graphs read."""

    def _decode_step(self, B: int, max_context: Optional[int] = None, nucleus: bool = False,
                     cascade: bool = False) -> None:
        m = self.model
        kw = {"cascade": (self.s_cas, ops.cascade_groups_max(B, m.nq, m.nkv))} if cascade else {}
        logits = m.forward_decode(self.s_tokens[:B], self.s_ctx[:B], self.s_bt[:B], max_context or self.max_model_len,
                                  **kw)
        ops.sample(logits, self.s_temp[:B], self.s_top_p[:B], self.s_seeds[:B], self.s_ctx[:B],
                   shards=logits.shape[0], tokens_out=self.s_tokens[:B], ctx_inc=self.s_ctx[:B],
                   hist=self.s_hist[:B], steps=self.s_steps[:B], nucleus=nucleus, stop=self._stop_args(),
                   tp=self.model.tp)

    @staticmethod
    def _wants_nucleus(reqs) -> bool:
        return any(r.params.temperature > 0 and r.params.top_p < 1 for r in reqs)

    def _bucket(self, n: int) -> int:
        for b in BUCKETS:
            if b >= n and b <= self.max_batch:
                return b
        return self.max_batch

    def capture_graphs(self, buckets: Optional[Sequence[int]] = None, nucleus: Optional[bool] = None) -> None:
        """Capture one decode-step graph per batch bucket (all slots must be idle: the kernels
        skip rows with context length 0, so warm-up and capture do not touch any state).
        ``nucleus`` (default ``self.capture_nucleus``): also capture the variants with the top-p
        passes; without them a chunk holding a top_p < 1 request decodes eagerly."""
        if not self.use_graphs:
            return
        tp = self.model.tp
        if tp.world > 1 and not tp.simulate:
            # every rank arrives (every rank captures at start-up) before any rank starts the warm-up steps, whose
            # collectives spin on the GPU until every peer has joined: a rank still in its local set-up (model init,
            # GEMM warm-up) must not share its GPU with peers that are already spinning (ranks time-sharing one GPU
            # in the rehearsals stalled for the whole xGMI timeout that way)
            tp.barrier()
        keep, tp.capture_on_xgmi = tp.capture_on_xgmi, True   # RCCL stays out of the graphs (TPGroup._xgmi_ok)
        # no cyclic garbage collection while graphs are captured: a collection inside a capture can finalize an
        # unreachable object that owns device resources (another engine's graphs and their private memory pool),
        # and freeing those is not a capturable call -- the capture fails and the graph destructor aborts the
        # process (seen once in the GPU suite: an earlier test's engine collected during the next one's capture)
        gc_on = gc.isenabled()
        gc.collect()
        gc.disable()
        try:
            with trace("engine.capture_graphs"):
                self._capture_graphs(buckets, self.capture_nucleus if nucleus is None else nucleus)
        finally:
            tp.capture_on_xgmi = keep
            if gc_on:
                gc.enable()

    def _capture_graphs(self, buckets: Optional[Sequence[int]], nucleus: bool) -> None:
        assert not self.running and not self.prefilling, "capture needs an idle engine"
        # (a max_batch that is not a bucket is its own top bucket: _bucket returns it for the rows above the last
        # bucket below it, which otherwise decoded eagerly)
        buckets = buckets or sorted({b for b in BUCKETS if b <= self.max_batch} | {self.max_batch})
        stream = torch.cuda.Stream(self.device)
        for B in sorted(set(buckets)):
            if not self._decode_bucket_capturable(B):
                continue    # decodes eagerly (its collectives do not all fit the graph-capturable transport)
            for mc in self._ctx_classes():
                # (cascade variants: batches of >= 2 rows without top-p passes; a top-p chunk decodes per row)
                for nuc, cas in [(n, c) for n in ((False, True) if nucleus else (False,))
                                 for c in ((False, True) if self.cascade and B >= 2 and not n else (False,))]:
                    if (B, mc, nuc, cas) in self.graphs:
                        continue
                    stream.wait_stream(torch.cuda.current_stream(self.device))
                    with torch.cuda.stream(stream):
                        self._decode_step(B, mc, nuc, cas)   # warm-up: allocator + lazy init outside capture
                    torch.cuda.current_stream(self.device).wait_stream(stream)
                    torch.cuda.synchronize(self.device)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=self._graph_pool, stream=stream):
                        self._decode_step(B, mc, nuc, cas)
                    if self._graph_pool is None:
                        self._graph_pool = g.pool()
                    self.graphs[(B, mc, nuc, cas)] = g
        if self.prefill_graphs_enabled():
            for Tb in PREFILL_GRAPH_BUCKETS:
                if Tb in self.prefill_graphs or not self._prefill_bucket_capturable(Tb):
                    continue
                if Tb > self.max_blocks_per_seq * self.block_size:
                    # no chunk of one sequence needs it, and its capture chunk (context Tb) would index past the
                    # block table and the RoPE table (found by the bounds-checked build, K8S_CHECKED=1): such a
                    # chunk runs eagerly
                    continue
                # a harmless chunk: Tb tokens of one sequence over block 0 whose K/V all go to the
                # scratch block (block 0 is only read)
                self._fill_prefill_state([0] * Tb, list(range(Tb)), [self.scratch_slot] * Tb, Tb, [0], Tb)
                stream.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(stream):
                    self._prefill_graph_body(Tb)
                torch.cuda.current_stream(self.device).wait_stream(stream)
                torch.cuda.synchronize(self.device)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self._graph_pool, stream=stream):
                    logits = self._prefill_graph_body(Tb)
                if self._graph_pool is None:
                    self._graph_pool = g.pool()
                self.prefill_graphs[Tb] = (g, logits)
        if self.speculative_tokens and self.speculative_tokens < SPEC_GRAPH_T and self.spec_graph is None \
                and self._prefill_bucket_capturable(SPEC_GRAPH_T, logits_rows=SPEC_GRAPH_T):
            # one sequence's verify forward (_spec_decode): SPEC_GRAPH_T rows, logits at every row
            Tb = SPEC_GRAPH_T
            self._fill_prefill_state([0] * Tb, list(range(Tb)), [self.scratch_slot] * Tb, Tb, [0], Tb)
            stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(stream):
                self._spec_graph_body()
            torch.cuda.current_stream(self.device).wait_stream(stream)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self._graph_pool, stream=stream):
                logits = self._spec_graph_body()
            if self._graph_pool is None:
                self._graph_pool = g.pool()
            self.spec_graph = (g, logits)
        torch.cuda.synchronize(self.device)

    def prefill_graphs_enabled(self) -> bool:
        """Prefill chunks of one sequence replay captured graphs (``K8S_PREFILL_GRAPHS=0`` turns them off).
        Multi-rank engines capture only the buckets whose collectives all stay on xGMI
        (``_prefill_bucket_capturable``); ``K8S_PREFILL_GRAPHS=1`` captures every bucket (RCCL included)."""
        env = os.environ.get("K8S_PREFILL_GRAPHS", "")
        return env != "0" and self.use_graphs and PREFILL_GRAPH_BUCKETS[-1] <= self.max_prefill_tokens

    def _decode_bucket_capturable(self, B: int) -> bool:
        """TP > 1: every collective of a B-row decode step (the two residual all-reduces per layer, B x hidden bf16,
        and the sampling exchange) fits the xGMI transports -- a gloo collective cannot be captured and RCCL stays out
        of the graphs (the prefill buckets' rule, ``_prefill_bucket_capturable``).  A bucket that does not fit decodes
        eagerly instead of capturing an RCCL / gloo call into its graph."""
        tp = self.model.tp
        if tp.world <= 1 or tp.simulate or os.environ.get("K8S_PREFILL_GRAPHS", "") == "1":
            return True
        if tp.xgmi is None:
            return False
        ar = B * self.model.cfg.hidden * 2
        return ar <= tp.xgmi.max_allreduce_bytes and logits_exchange_bytes(self.model, B) <= tp.xgmi.slot_bytes

    def _prefill_bucket_capturable(self, Tb: int, logits_rows: int = 1) -> bool:
        """TP > 1: a chunk of Tb tokens all-reduces Tb x hidden bf16 twice per layer and all-gathers
        ``logits_rows`` rows of fp32 logits (one for a prefill chunk, every row for the speculative verify
        forward); both must fit the xGMI transports, because a gloo collective cannot be captured (the 1-GPU
        rehearsals) and RCCL capture stays opt-in until it has run on a multi-GPU node.  A verify forward that
        does not fit runs eagerly."""
        tp = self.model.tp
        if tp.world <= 1 or tp.simulate or os.environ.get("K8S_PREFILL_GRAPHS", "") == "1":
            return True
        if tp.xgmi is None:
            return False
        sp = getattr(self.model, "seq_parallel_at", None)
        if sp is not None and sp(Tb) and tp.rccl is not None:
            return False                   # the reduce-scatters run on RCCL: eager, like every RCCL chunk
        ar_bytes = Tb * self.model.cfg.hidden * 2
        # captured with tp.capture_on_xgmi: every all-reduce that fits the capacity stays on xGMI
        return ar_bytes <= tp.xgmi.max_allreduce_bytes and logits_exchange_bytes(self.model, logits_rows) <= tp.xgmi.slot_bytes

    def _p_views(self, Tb: int):
        Tm = PREFILL_GRAPH_BUCKETS[-1]
        pk = self.p_packed
        return (pk[:Tb], pk[Tm:Tm + Tb], pk[2 * Tm:2 * Tm + Tb], pk[3 * Tm:3 * Tm + 2], pk[3 * Tm + 2:3 * Tm + 3],
                pk[3 * Tm + 3:3 * Tm + 4])

    def _seq_parallel_at(self, T: int) -> bool:
        """The model runs a T-token prefill chunk sequence-parallel (LlamaModel.seq_parallel_at)."""
        f = getattr(self.model, "seq_parallel_at", None)
        return bool(f(T)) if f is not None else False

    def _overlap_split_at(self, T: int) -> int:
        """Token at which a TP > 1 prefill chunk of T tokens splits into two micro-batches (0: no split)."""
        if T < self.model.prefill_overlap_min or not self.model.prefill_overlap or self._seq_parallel_at(T):
            return 0
        return max(16, T // 2 // 16 * 16)

    spec_graph: Optional[tuple] = None   # (graph, logits [tp, SPEC_GRAPH_T, Vs]) of the single-sequence verify forward

    def _spec_graph_body(self) -> torch.Tensor:
        ids, pos, slots, cu, ctx, _ = self._p_views(SPEC_GRAPH_T)
        return self.model.forward_prefill(ids, pos, slots, cu, ctx, self.p_bt, SPEC_GRAPH_T, self.v_last)

    def _prefill_graph_body(self, Tb: int) -> torch.Tensor:
        ids, pos, slots, cu, ctx, last = self._p_views(Tb)
        split = None
        T0 = self._overlap_split_at(Tb)
        if T0:
            o = 3 * PREFILL_GRAPH_BUCKETS[-1] + 4
            pk = self.p_packed
            split = (T0, (pk[o:o + 2], pk[o + 2:o + 3], self.p_bt, T0),
                     (pk[o + 3:o + 5], pk[o + 5:o + 6], self.p_bt, Tb - T0))
        return self.model.forward_prefill(ids, pos, slots, cu, ctx, self.p_bt, Tb, last, split=split)

    def _fill_prefill_state(self, ids, pos, slots, ctx_len: int, blocks, Tb: int) -> None:
        """One chunk of ONE sequence into the graph's static inputs; positions Tb-T.. are padding
        (token 0 at position 0, K/V into the scratch slot, outside cu_q).  The micro-batch halves (tokens
        [0, T0) and [T0, Tb), ``_overlap_split_at``) get their own cu_q / context length: a half holding
        only padding has no query tokens."""
        T, Tm = len(ids), PREFILL_GRAPH_BUCKETS[-1]
        pad = Tb - T
        host = torch.zeros(3 * Tm + 4 + _P_SPLIT, dtype=torch.int32)
        host[:T] = torch.tensor(ids, dtype=torch.int32)
        host[Tm:Tm + T] = torch.tensor(pos, dtype=torch.int32)
        host[2 * Tm:2 * Tm + T] = torch.tensor(slots, dtype=torch.int32)
        host[2 * Tm + T:2 * Tm + T + pad] = self.scratch_slot
        host[3 * Tm + 1] = T
        host[3 * Tm + 2] = ctx_len
        host[3 * Tm + 3] = T - 1
        T0 = self._overlap_split_at(Tb)
        if T0:
            n0, n1 = min(T, T0), max(0, T - T0)
            o = 3 * Tm + 4
            host[o + 1], host[o + 2] = n0, ctx_len - n1
            host[o + 4], host[o + 5] = n1, ctx_len
        bt = torch.zeros(1, self.max_blocks_per_seq, dtype=torch.int32)
        bt[0, :len(blocks)] = torch.tensor(blocks, dtype=torch.int32)
        self.p_packed.copy_(self._dev(host))
        self.p_bt.copy_(self._dev(bt))
