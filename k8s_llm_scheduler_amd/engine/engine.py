"""Decision engine: continuous-batched prefill + hipGraph-replayed decode over a paged KV cache.

Replaces the remote ``chat_completion`` of the reference (``scheduler.py:425-433``) with an
in-process Llama-3.

Per engine iteration (:meth:`LLMEngine.step`):

1. **Admit** waiting requests while a decode slot is free and the native block allocator can
   reserve KV for prompt + max_tokens (decode never allocates: a decode step needs no host work).
   Prompt prefixes already in the prefix cache (the scheduler's long system prompt) are skipped.
2. **Prefill** (chunked): up to ``max_prefill_tokens`` prompt tokens of several requests in one
   varlen forward; requests whose prompt completes sample their first token, which seeds the
   device-resident decode state of their slot.
3. **Decode**: ``decode_chunk`` steps over the active slots.  One step = embedding -> 80 x
   (norm, QKV GEMV, RoPE+KV write, paged attention, O GEMV, all-reduce, fused add+norm, SwiGLU
   GEMV, down GEMV, all-reduce) -> LM head -> sampler, where the sampler also advances the state
   (token, context length, history).  The whole step is captured once per batch bucket into a
   hipGraph (``torch.cuda.CUDAGraph``) and replayed, so the host only launches graphs; after the
   chunk, one small D2H copy of the token history drives stop checks (EOS, closed JSON object,
   max_tokens).

Every TP rank runs the identical deterministic schedule; sampling is deterministic given
(seed, position), so all ranks draw the same tokens without any extra broadcast.

This module is the scheduler core (admission, prefill, decode, stop checks, finishing).  The engine's other
concerns live in mixins: ``graphs.py`` (hipGraph capture of decode / prefill / verify forwards), ``recovery.py``
(bounded device waits, failure recovery, the multi-rank schedule), ``speculative.py`` (prompt-lookup speculative
decoding), ``serving.py`` (background loop, blocking ``generate``); shared types and constants are in ``common.py``.
"""

from __future__ import annotations

import inspect
import itertools
import math
import os
import random
import threading
import time
from collections import deque
from typing import Deque, Dict, List, Optional, Sequence, Union

import torch

from .. import ops
from ..control.jsonextract import json_object_closed
from ..models.llama import LlamaModel
from ..parallel.comm import CollectiveError
from .sampling import SamplingParams
from .tokenizer import Tokenizer
from ..utils.tracing import trace
from .common import (BUCKETS, MIXED_MIN_PROMPT_ROWS, PREFILL_GRAPH_BUCKETS, SPEC_GRAPH_T, SPEC_MAX_BATCH,  # noqa: F401
                     EngineStalled, EngineUnavailable, Output, Request, RequestRejected, _HostStage, _P_SPLIT,
                     _PyBlockAllocator, ngram_draft, split_prefill_meta)
from .graphs import GraphCaptureMixin
from .recovery import RecoveryMixin
from .serving import ServingMixin
from .speculative import SpeculativeMixin


class LLMEngine(GraphCaptureMixin, RecoveryMixin, SpeculativeMixin, ServingMixin):
    def __init__(self, model: LlamaModel, tokenizer: Tokenizer, *, max_batch: int = 64, block_size: int = 16,
                 num_blocks: Optional[int] = None, kv_cache_gb: float = 0.0, kv_cache_fraction: float = 0.85,
                 max_model_len: Optional[int] = None, max_prefill_tokens: int = 8192, cuda_graphs: bool = True,
                 prefix_caching: bool = True, decode_chunk: int = 4, seed: int = 0, metrics=None,
                 control=None, capture_nucleus: bool = False, speculative_tokens: int = 0,
                 watchdog_s: float = 60.0, on_unrecoverable: str = "stay", device_stop: bool = True,
                 mixed_steps: bool = True, mixed_step_rows: int = 256):
        self.model = model
        # Vocab-parallel sampling at TP > 1: the model returns this rank's logits shard and the
        # sampler exchanges a few bytes per row (ops.sample(tp=...)), so no step all-gathers rows x vocab x 4 B.
        # K8S_VOCAB_PARALLEL=0: all-gather the logits and sample the full rows (same tokens).
        self.vocab_parallel = model.tp.world > 1 and os.environ.get("K8S_VOCAB_PARALLEL", "1") != "0"
        model.gather_logits = not self.vocab_parallel
        # Device-side stop detection: the decode graphs' sampler finishes rows itself (EOS,
        # closed JSON object, max_tokens) and raises a host-mapped flag; the host checks it after every replay
        # instead of after a whole decode_chunk.  Mixed steps (item 5): a prefill step also advances every
        # running decode by one token in the same varlen forward, and new arrivals end a decode chunk early.
        self.device_stop = bool(device_stop)
        self.mixed_steps = bool(mixed_steps)
        # rows of a mixed step's varlen forward (prompt tokens + one per running decode) are kept within this many
        # (0: no cap), so an arrival's chunk plus the decode rows stays inside the GEMMs' 256-row plans: a 245-token
        # prompt with 5 decodes riding along is 250 rows (41 ms of GEMMs at 70B TP=1), where 261 rows fell into the
        # 384-row plans (62 ms, profiles/lastfwd_70b_tp1_arr3_r4.txt); the few prompt tokens over the cap go into
        # the next step, itself a cheap mixed step
        self.mixed_step_rows = max(0, int(mixed_step_rows))
        self._prefill_capped = False
        # Bounded device waits: every host wait for device results polls an event against
        # min(call deadline, step start + watchdog_s) instead of blocking in a synchronize, so a hung collective
        # surfaces as EngineStalled inside llm.timeout.  ``on_unrecoverable``: "exit" ends the process (exit code
        # 70) when recovery cannot drain the device, so the Deployment restarts the pod; "stay" keeps it
        # not-ready (tests, single-process runs).
        self.watchdog_s = float(watchdog_s)
        if on_unrecoverable not in ("exit", "stay"):
            raise ValueError("on_unrecoverable must be 'exit' or 'stay'")
        self.on_unrecoverable = on_unrecoverable
        self._call_deadline: Optional[float] = None
        self._step_t0 = time.monotonic()
        self._last_event = None
        self._pinned: Dict[tuple, torch.Tensor] = {}
        self.health = {"ready": True, "reason": "", "failures": 0, "recoveries": 0, "since": time.time()}
        # test fault injection on a follower rank: ("stall", step, seconds) sleeps before that step's device work,
        # ("raise", step, 0) fails that step with a CollectiveError after its collectives ran (step = 1-based
        # count of schedule messages)
        self.fault: Optional[tuple] = None
        self._steps = 0
        self._reset_seen = 0        # follower: the leader's last reset generation handled
        if control is not None and control.rank == 0:
            control.start_monitor()
        # prompt-lookup speculative decoding (_spec_decode): drafted tokens per step, 0 = off
        self.speculative_tokens = max(0, int(speculative_tokens))
        if self.speculative_tokens:
            # the verify steps emit tokens on the host without advancing the sampler's device stop state (JSON
            # depth, done flag), so a later one-token decode would see a stale brace depth and could end an answer
            # early: stop detection stays on the host (_emit) and prefills carry no decode rows
            self.device_stop = False
            self.mixed_steps = False
        # also capture decode graphs with the top-p passes (config llm.top_p < 1); otherwise chunks
        # holding a top_p < 1 request decode eagerly
        self.capture_nucleus = capture_nucleus
        # Multi-rank serving: rank 0 announces new requests / aborts to the other TP ranks at the
        # start of every step, so all ranks run the identical schedule (None: single rank, or
        # every rank is fed identical requests, as in bench.py).
        self.control = control
        self._outbox: List[Request] = []
        self.tok = tokenizer
        self.device = model.device
        self.gpu = self.device.type == "cuda"
        self.max_batch = max_batch
        self.block_size = block_size
        self.max_model_len = min(max_model_len or model.max_model_len, model.max_model_len)
        self.max_blocks_per_seq = math.ceil(self.max_model_len / block_size)
        self.max_prefill_tokens = max_prefill_tokens
        self.decode_chunk = max(1, decode_chunk)
        self.metrics = metrics
        self._rng = random.Random(seed)
        self._ids = itertools.count()
        if num_blocks is None:
            per_block = model.kv_bytes_per_block(block_size)
            if kv_cache_gb > 0:
                budget = kv_cache_gb * 1e9
            elif self.gpu:
                free, _ = torch.cuda.mem_get_info(self.device)
                budget = max(0.0, free * kv_cache_fraction - 2e9)
            else:
                budget = 64 * 1024 * 1024
            num_blocks = int(budget // per_block)
            # never more than every slot at full length needs
            num_blocks = min(num_blocks, max_batch * self.max_blocks_per_seq + 1)
        if num_blocks < self.max_blocks_per_seq:
            raise RuntimeError(f"KV cache too small: {num_blocks} blocks < one full sequence "
                               f"({self.max_blocks_per_seq})")
        self.num_blocks = num_blocks
        # one extra block past the allocator's range: the K/V sink of prefill-graph padding tokens
        model.allocate_kv(num_blocks + 1, block_size)
        self.scratch_slot = num_blocks * block_size
        self.prefix_caching = prefix_caching
        self._share_deferred = False
        self.allocator = ops.native().BlockAllocator(num_blocks, block_size, prefix_caching) if ops.available() \
            else _PyBlockAllocator(num_blocks, block_size, prefix_caching)
        self.max_new_cap = self.max_model_len
        self._alloc_state()
        self.waiting: Deque[Request] = deque()
        self.prefilling: List[Request] = []
        self.running: Dict[int, Request] = {}        # slot -> request
        self.requests: Dict[int, Request] = {}
        self.free_slots = list(range(max_batch - 1, -1, -1))
        self.use_graphs = cuda_graphs and self.gpu
        self.graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}   # (batch bucket, context class, nucleus, cascade)
        # cascade decode attention (ops.decode_attention_fused): a chunk whose running rows share a prefix of at least
        # K8S_DECODE_CASCADE_MIN tokens (batched decisions on one cluster snapshot with the cluster-first prompt
        # layout) attends it once for every row instead of once per row; K8S_DECODE_CASCADE=0 turns it off
        m = model
        self.cascade = (self.gpu and os.environ.get("K8S_DECODE_CASCADE", "1") != "0" and max_batch >= 2
                        and ops.cascade_ok(getattr(m, "nq", 0), getattr(m, "nkv", 0), block_size, getattr(m, "D", 0))
                        and "cascade" in inspect.signature(m.forward_decode).parameters)
        self.cascade_min = max(64, int(os.environ.get("K8S_DECODE_CASCADE_MIN", "512")))
        self._cas_key: Optional[tuple] = None
        self._cas_val = (0, 0)
        self.prefill_graphs: Dict[int, tuple] = {}             # token bucket -> (graph, logits)
        self._graph_pool = None
        self.lock = threading.RLock()
        # background serving loop (start_background): callers of generate() only touch the inbox and
        # wait on their requests' events, so a submitter never waits for a whole engine step
        self._inbox: List[Request] = []
        self._pf_events: List[tuple] = []   # (start, end) CUDA events of prefills not accounted yet
        self._inbox_lock = threading.Lock()
        self._wake = threading.Condition(self._inbox_lock)
        self._bg_thread: Optional[threading.Thread] = None
        self._abort_thread: Optional[threading.Thread] = None   # recover(): RCCL abort in flight
        self._stage: Optional["_HostStage"] = None               # pinned host -> device staging ring (_dev)
        self.recovery_trace: Deque[tuple] = deque(maxlen=512)    # (monotonic s, event) of recover() / resets
        self._trace_steps = os.environ.get("K8S_ENGINE_TRACE", "0") == "1"   # (tests) per-replay host timeline too
        self._bg_stop = False
        self._bg_error: Optional[BaseException] = None
        self.finished_log: Deque[tuple] = deque(maxlen=4096)
        self.stats = {"prefill_tokens": 0, "cached_tokens": 0, "decode_steps": 0, "decode_tokens": 0,
                      "graph_replays": 0, "prefill_graph_replays": 0, "prefill_overlap_chunks": 0, "prefill_time": 0.0,
                      "decode_time": 0.0, "spec_steps": 0, "spec_graph_replays": 0, "spec_drafted": 0,
                      "spec_accepted": 0, "stalls": 0, "mixed_steps": 0, "mixed_decode_rows": 0,
                      "early_chunk_stops": 0, "cascade_chunks": 0}

    def _dev(self, x, dtype=torch.int32) -> torch.Tensor:
        """Host data -> the engine's device without ever blocking the host.  A copy from pageable memory waits for
        the stream, and allocating new pinned memory (tensor.pin_memory()) was measured to block until the device
        drains too -- behind a stalled collective both are unbounded waits (tests/test_recovery_gpu.py).  So small
        tensors go through a ring of pre-pinned slots (_HostStage), each reused only after its previous copy ran."""
        t = x if isinstance(x, torch.Tensor) else torch.tensor(x, dtype=dtype)
        if not self.gpu:
            return t
        if self._stage is None:
            self._stage = _HostStage(self._wait_limit)
        return self._stage.to_device(t, self.device)

    # ------------------------------------------------------------------ device state
    def _alloc_state(self) -> None:
        B, dev = self.max_batch, self.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.s_tokens = torch.zeros(B, **i32)
        self.s_ctx = torch.zeros(B, **i32)
        self.s_bt = torch.zeros(B, self.max_blocks_per_seq, **i32)
        self.s_temp = torch.zeros(B, dtype=torch.float32, device=dev)
        self.s_top_p = torch.ones(B, dtype=torch.float32, device=dev)
        self.s_seeds = torch.zeros(B, **i32)
        self.s_steps = torch.zeros(B, **i32)
        self.s_hist = torch.zeros(B, self.max_new_cap, **i32)
        self.s_cas = torch.zeros(2, **i32)   # cascade: (shared 64-token spans, a slot holding them)
        # prefill-graph inputs, one packed buffer filled by one host->device copy per chunk:
        # [ids | positions | slots] x Tmax, then cu_q (2), context_lens (1), last_idx (1), then the two
        # micro-batch halves' cu_q / context_lens (_P_SPLIT)
        Tm = PREFILL_GRAPH_BUCKETS[-1]
        self.p_packed = torch.zeros(3 * Tm + 4 + _P_SPLIT, **i32)
        self.p_bt = torch.zeros(1, self.max_blocks_per_seq, **i32)
        self.v_last = torch.arange(SPEC_GRAPH_T, **i32)       # the verify graph's logits rows: all of them
        # device-side stop detection state (sampler.hip StopArgs)
        self.s_json = torch.full((B,), -2, **i32)
        self.s_cfg = torch.zeros(B, **i32)
        self.s_forced = torch.zeros(B, self.max_new_cap, **i32)
        self.s_forced_len = torch.full((B,), -1, **i32)
        self.stop_cls = ops.token_stop_classes(self.tok, self.model.cfg.vocab).to(dev)
        if self.gpu:
            host, devp = ops.native().host_mapped_alloc(4 * B)
            import ctypes

            import numpy as np

            self._done_ptr = devp
            self._done_host = np.ctypeslib.as_array((ctypes.c_int32 * B).from_address(host))
            self._done_mem = host
        else:
            self._done_cpu = torch.zeros(B, dtype=torch.int32)
            self._done_host = self._done_cpu.numpy()

    def _stop_args(self) -> Optional[dict]:
        if not self.device_stop:
            return None
        return {"cls": self.stop_cls, "json": self.s_json, "cfg": self.s_cfg, "forced": self.s_forced,
                "forced_len": self.s_forced_len, "eos_tok": self.tok.eot_id,
                "done": self._done_ptr if self.gpu else self._done_cpu}

    def _shared_prefix(self) -> tuple:
        """(64-token spans every running row shares, a slot holding them): the running rows' longest common block-list
        prefix, cut at the earliest prompt end (a row's new token always lies past its prompt, so the shared spans
        never reach one).  Recomputed only when the running set changes (the blocks of a request never do)."""
        rs = sorted(self.running.values(), key=lambda r: r.slot)
        key = tuple((r.slot, r.rid) for r in rs)
        if key != self._cas_key:
            first = rs[0].blocks
            n = min(min(len(r.blocks) for r in rs), min(len(r.prompt_ids) for r in rs) // self.block_size)
            lcp = 0
            while lcp < n and all(r.blocks[lcp] == first[lcp] for r in rs[1:]):
                lcp += 1
            self._cas_key, self._cas_val = key, ((lcp * self.block_size) // 64, rs[0].slot)
        return self._cas_val

    def _ctx_classes(self) -> List[int]:
        """Context-length classes with their own decode graph: contexts <= 1024 tokens (one
        attention partition per sequence: no partial buffers, no merge kernel) and the rest."""
        return sorted({min(1024, self.max_model_len), self.max_model_len})

    # ------------------------------------------------------------------ requests
    def render_chat(self, system: str, user: str) -> List[int]:
        return self.tok.chat_ids(system, user)

    def add_request(self, prompt: Union[str, List[int]], params: Optional[SamplingParams] = None) -> Request:
        params = (params or SamplingParams()).validate()
        ids = self.tok.encode(prompt) if isinstance(prompt, str) else list(prompt)
        if not ids:
            raise ValueError("empty prompt")
        max_new = min(params.max_tokens, self.max_model_len - len(ids))
        if max_new < 1:
            raise ValueError(f"prompt of {len(ids)} tokens exceeds max_model_len {self.max_model_len}")
        if max_new != params.max_tokens:
            params = SamplingParams(**{**params.__dict__, "max_tokens": max_new})
        seed = params.seed if params.seed is not None else self._rng.getrandbits(31)
        if self._bg_thread is not None:
            r = Request(next(self._ids), ids, params, seed, done=threading.Event())
            with self._wake:
                self._inbox.append(r)
                self._wake.notify()
            return r
        with self.lock:
            r = Request(next(self._ids), ids, params, seed)
            self._enqueue(r)
        return r

    def _enqueue(self, r: Request) -> None:
        self.requests[r.rid] = r
        self.waiting.append(r)
        if self.control is not None:
            self._outbox.append(r)

    def _drain_inbox(self) -> None:
        with self._inbox_lock:
            new, self._inbox = self._inbox, []
        for r in new:
            self._enqueue(r)

    def _reap_aborted(self) -> None:
        for r in sorted((r for r in self.requests.values() if r.aborted and not r.finished), key=lambda r: r.rid):
            if r in self.waiting:
                self.waiting.remove(r)
            self._finish(r, "abort")
        for rid in [rid for rid, r in self.requests.items() if r.aborted and r.finished]:
            self.requests.pop(rid, None)

    def abort(self, rid: int) -> None:
        """Mark a request aborted; it is removed at the start of the next step (on every rank)."""
        with self._inbox_lock:
            for r in self._inbox:
                if r.rid == rid:
                    r.aborted = True
        with self.lock:
            r = self.requests.get(rid)
            if r is not None and not r.finished:
                r.aborted = True

    def has_work(self) -> bool:
        return bool(self.waiting or self.prefilling or self.running)

    # ------------------------------------------------------------------ scheduling
    SHARE_MIN_BLOCKS = 2   # in-batch prefix sharing: defer a request that shares this many blocks

    def _shares_pending_prefix(self, r: Request) -> bool:
        """True when ``r`` shares at least SHARE_MIN_BLOCKS full KV blocks of its prompt with a request
        that is still prefilling them.  Admitting ``r`` now would recompute that prefix (blocks are
        published to the prefix cache only once their KV is written); one step later it is a cache
        hit.  This is what makes a batch of pods decided against one cluster snapshot prefill the
        shared part once (``compat.prompt_layout: cluster_first``)."""
        if not self.prefix_caching:
            return False
        bs = self.block_size
        ids = r.prompt_ids
        for p in self.prefilling:
            n = min(len(p.prompt_ids), len(ids)) - 1   # the last prompt token is never cached
            c = 0
            while c + bs <= n and p.prompt_ids[c:c + bs] == ids[c:c + bs]:
                c += bs
            if c // bs >= self.SHARE_MIN_BLOCKS and p.computed < c:
                return True
        return False

    def _admit(self) -> None:
        while self.waiting and self.free_slots:
            r = self.waiting[0]
            if r.aborted:
                self.waiting.popleft()
                self._finish(r, "abort")
                continue
            if self._shares_pending_prefix(r):
                self._share_deferred = True
                break   # admitted next step, with the shared prefix served from the cache
            total = len(r.prompt_ids) + r.params.max_tokens
            if not self.allocator.can_allocate(r.prompt_ids, total):
                if not self.running and not self.prefilling:
                    self.waiting.popleft()
                    raise RequestRejected(r, "request does not fit in an empty KV cache")
                break
            self.waiting.popleft()
            a = self.allocator.allocate(r.prompt_ids, total)
            r.blocks = list(a.blocks)
            r.cached = r.computed = int(a.cached_tokens)
            n_sub = int(getattr(a, "copy_tokens", 0))
            if n_sub > 0:   # sub-block prefix hit: those positions' K/V come from a cached block (copied now, on
                # the stream, before anything that could reuse the source block)
                self._copy_kv_positions(int(a.copy_src), r.blocks[(r.cached - n_sub) // self.block_size], n_sub)
                self.stats["sub_block_tokens"] = self.stats.get("sub_block_tokens", 0) + n_sub
            r.slot = self.free_slots.pop()
            self.prefilling.append(r)
            self.stats["cached_tokens"] += r.cached

    def _copy_kv_positions(self, src_block: int, dst_block: int, n: int) -> None:
        """K/V of positions [0, n) of ``src_block`` -> the same positions of ``dst_block``, every layer (the cache is
        [layers, 2, slots, kv heads, D]; TP ranks copy their own heads)."""
        kv = self.model.kv_cache
        bs = self.block_size
        src = self._dev(list(range(src_block * bs, src_block * bs + n)), torch.long)
        dst = self._dev(list(range(dst_block * bs, dst_block * bs + n)), torch.long)
        kv.index_copy_(2, dst, kv.index_select(2, src))

    def _prefill(self) -> None:
        if not self.prefilling:
            return
        if self._trace_steps:
            self.recovery_trace.append((time.monotonic(), f"prefill: {len(self.prefilling)} requests"))
        budget = self.max_prefill_tokens
        capped = False
        if self.mixed_steps and self.running and self.mixed_step_rows:
            # the cap is for a serving step that would land just past the cap (an arrival or two beside the
            # decodes); a throughput backlog (a batch of prompts, thousands of rows) keeps its big chunks
            rows = min(sum(len(r.prompt_ids) - r.computed for r in self.prefilling), budget) + len(self.running)
            if self.mixed_step_rows < rows <= 2 * self.mixed_step_rows:
                capped = True
                budget = min(budget, max(MIXED_MIN_PROMPT_ROWS, self.mixed_step_rows - len(self.running)))
        self._prefill_capped = capped
        chunk = []  # (req, start, end)
        for r in self.prefilling:
            if budget <= 0:
                break
            if capped and chunk and len(r.prompt_ids) - r.computed > budget:
                break   # under the row cap a second prompt joins only whole (a split one costs an extra step)
            n = min(len(r.prompt_ids) - r.computed, budget)
            chunk.append((r, r.computed, r.computed + n))
            budget -= n
        bs = self.block_size
        ids, pos, slots, cu, ctx, last = [], [], [], [0], [], []
        bt = torch.zeros(len(chunk), self.max_blocks_per_seq, dtype=torch.int32)
        for i, (r, s, e) in enumerate(chunk):
            ids += r.prompt_ids[s:e]
            pos += range(s, e)
            slots += [r.blocks[p // bs] * bs + p % bs for p in range(s, e)]
            cu.append(cu[-1] + (e - s))
            ctx.append(e)
            last.append(cu[-1] - 1)
            bt[i, :len(r.blocks)] = torch.tensor(r.blocks, dtype=torch.int32)
        dev = self.device
        t = self._dev
        t0 = time.perf_counter()
        if self.gpu:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        # mixed step: every running decode rides along as a 1-token sequence (its next token), so an arrival's
        # prefill does not stall the decodes in flight
        dec = sorted(self.running) if self.mixed_steps and self.running else []
        Tb = next((b for b in PREFILL_GRAPH_BUCKETS if b >= len(ids)), None) if len(chunk) == 1 and not dec else None
        if self.use_graphs and Tb is not None and Tb in self.prefill_graphs:
            r0 = chunk[0][0]
            self._fill_prefill_state(ids, pos, slots, ctx[0], r0.blocks, Tb)
            graph, logits = self.prefill_graphs[Tb]
            graph.replay()
            self.stats["prefill_graph_replays"] += 1
            self.stats["prefill_overlap_chunks"] += bool(self._overlap_split_at(Tb))
        elif dec:
            d = self._dev(dec, torch.long)
            ctx_d = self.s_ctx.index_select(0, d)
            # (a row the device finished has context 0: its position is clamped to 0 for the block lookup, and its
            # leftover token's K/V goes nowhere (slot -1, skipped by the KV write) -- position 0 of its first block
            # is usually a shared, published prefix block that other sequences and later prefix hits read)
            pos_d = (ctx_d - 1).clamp_min(0)
            blk = self.s_bt.index_select(0, d).gather(1, (pos_d // bs).long().unsqueeze(1)).squeeze(1)
            n_p = len(ids)
            ids_t = torch.cat([t(ids), self.s_tokens.index_select(0, d)])
            pos_t = torch.cat([t(pos), pos_d])
            slot_t = torch.cat([t(slots), torch.where(ctx_d > 0, blk * bs + pos_d % bs, torch.full_like(blk, -1))])
            cu_all = cu + [cu[-1] + k + 1 for k in range(len(dec))]
            ctx_t = torch.cat([t(ctx), ctx_d])
            bt_t = torch.cat([self._dev(bt), self.s_bt.index_select(0, d)])
            last_t = t(last + [n_p + k for k in range(len(dec))])
            logits = self.model.forward_prefill(ids_t, pos_t, slot_t, t(cu_all), ctx_t, bt_t,
                                                max(e - s for _, s, e in chunk), last_t)
            # the decode rows' tokens: the decode graphs' sampler (same counters, same stop detection), with the
            # state of each row's slot updated in place
            ld = logits[:, len(chunk):].contiguous()
            ops.sample(ld, self.s_temp.index_select(0, d), self.s_top_p.index_select(0, d),
                       self.s_seeds.index_select(0, d), ctx_d.clone(), shards=ld.shape[0], tokens_out=self.s_tokens,
                       ctx_inc=self.s_ctx, hist=self.s_hist, steps=self.s_steps,
                       nucleus=self._wants_nucleus(self.running[x] for x in dec), slots=d.to(torch.int32),
                       stop=self._stop_args(), tp=self.model.tp)
            logits = logits[:, :len(chunk)]
            self.stats["mixed_steps"] += 1
            self.stats["mixed_decode_rows"] += len(dec)
        else:
            bt_d = self._dev(bt)
            split = None
            T0 = self._overlap_split_at(len(ids))
            if T0:
                halves = []
                for c_h, x_h, seqs in split_prefill_meta(cu, ctx, T0):
                    idx = self._dev(seqs, torch.long)
                    halves.append((t(c_h), t(x_h), bt_d.index_select(0, idx),
                                   max(b - a for a, b in zip(c_h, c_h[1:]))))
                split = (T0, halves[0], halves[1])
                self.stats["prefill_overlap_chunks"] += 1
            logits = self.model.forward_prefill(t(ids), t(pos), t(slots), t(cu), t(ctx), bt_d,
                                                max(e - s for _, s, e in chunk), t(last), split=split)
        self.stats["prefill_tokens"] += len(ids)
        self.stats["prefill_steps"] = self.stats.get("prefill_steps", 0) + 1
        if self._trace_steps:
            self.recovery_trace.append((time.monotonic(), "prefill: forward enqueued"))
        done = [(i, r) for i, (r, s, e) in enumerate(chunk) if e == len(r.prompt_ids)]
        for r, s, e in chunk:
            r.computed = e
            self.allocator.commit_prefix(r.blocks, r.prompt_ids, e)
            if self._trace_steps:
                self.recovery_trace.append((time.monotonic(), "prefill: committed"))
        if done:
            idx = self._dev([i for i, _ in done], torch.long)
            sub = logits.index_select(1, idx).contiguous()   # [tp, n, Vs]
            rs = [r for _, r in done]
            temp = self._dev([r.params.temperature for r in rs], torch.float32)
            top_p = self._dev([r.params.top_p for r in rs], torch.float32)
            seeds = self._dev([r.seed for r in rs])
            if self._trace_steps:
                self.recovery_trace.append((time.monotonic(), "prefill: staged"))
            ctr = self._dev([len(r.prompt_ids) for r in rs])
            toks = ops.sample(sub, temp, top_p, seeds, ctr, shards=sub.shape[0], nucleus=self._wants_nucleus(rs),
                              tp=self.model.tp)
            if self._trace_steps:
                self.recovery_trace.append((time.monotonic(), "prefill: sample enqueued"))
            slots_t = self._dev([r.slot for r in rs], torch.long)
            forced0 = [(k, r.params.forced_output_ids[0]) for k, r in enumerate(rs) if r.params.forced_output_ids]
            if forced0:   # scripted answers replace the sampled first token too
                fk = self._dev([k for k, _ in forced0], torch.long)
                toks = toks.index_copy(0, fk, self._dev([v for _, v in forced0]))
            # index_copy_ / index_fill_, not `state[idx] = value`: a Python scalar assigned that way is copied to the
            # device from pageable memory, which waits for the stream -- behind a stalled collective, for good
            self._put(self.s_tokens, slots_t, toks)
            self._put(self.s_ctx, slots_t, ctr + 1)
            self._put(self.s_hist.select(1, 0), slots_t, toks)
            self.s_steps.index_fill_(0, slots_t, 1)
            self._put(self.s_temp, slots_t, temp)
            self._put(self.s_top_p, slots_t, top_p)
            self._put(self.s_seeds, slots_t, seeds)
            if self._trace_steps:
                self.recovery_trace.append((time.monotonic(), "prefill: state written"))
            self._init_stop_state(rs, slots_t)
            if self._trace_steps:
                self.recovery_trace.append((time.monotonic(), "prefill: stop state"))
            for r in rs:
                row = torch.zeros(self.max_blocks_per_seq, dtype=torch.int32)
                row[:len(r.blocks)] = torch.tensor(r.blocks, dtype=torch.int32)
                self.s_bt[r.slot] = self._dev(row)
            now = time.perf_counter()
            for r in rs:
                r.first_token_time = now
                self.prefilling.remove(r)
                self.running[r.slot] = r
        if self._trace_steps:
            self.recovery_trace.append((time.monotonic(), f"prefill: {len(done)} sampled"))
        if self.gpu:
            # no per-prefill wait: the decode that follows in this step waits (bounded) for both and checks the
            # collectives' health; only a step that prefills and decodes nothing bounds its device work here.
            # prefill_time is GPU time, from events read once they completed.
            self._pf_events.append((ev0, torch.cuda.Event(enable_timing=True)))
            self._pf_events[-1][1].record()
            if not self.running:
                self.model.tp.snapshot_health()
                self._wait_device("prefill")
                self.model.tp.check_health()
                self._account_prefill()
        else:
            self.stats["prefill_time"] += time.perf_counter() - t0

    def _account_prefill(self) -> None:
        """Add the GPU time of completed prefills to stats["prefill_time"] (after a device wait)."""
        keep = []
        for a, b in self._pf_events:
            if b.query():
                self.stats["prefill_time"] += a.elapsed_time(b) / 1e3
            else:
                keep.append((a, b))
        self._pf_events = keep

    @staticmethod
    def _put(dst: torch.Tensor, idx: torch.Tensor, src: torch.Tensor) -> None:
        """dst[idx] = src along dim 0, enqueued without a host sync."""
        dst.index_copy_(0, idx, src.to(dst.dtype))

    def _init_stop_state(self, rs: Sequence[Request], slots_t: torch.Tensor) -> None:
        """Device stop state of freshly prefilled slots: first token unclassified (-2), stop config (EOS / JSON
        close / max_tokens), the scripted answer of forced requests, done flag clear."""
        if not self.device_stop:
            return
        dev = self.device
        cfg, flen = [], []
        for r in rs:
            p = r.params
            c = (0 if p.ignore_eos else 1) | (2 if p.stop_on_json_close and not p.ignore_eos else 0)
            cfg.append(c | (min(p.max_tokens, self.max_new_cap) << 8))
            f = p.forced_output_ids
            flen.append(-1 if f is None else min(len(f), self.max_new_cap))
            if f is not None and f:
                n = min(len(f), self.max_new_cap)
                self.s_forced[r.slot, :n] = self._dev(f[:n])
            self._done_host[r.slot] = 0
        self.s_json.index_fill_(0, slots_t, -2)
        self._put(self.s_cfg, slots_t, self._dev(cfg))
        self._put(self.s_forced_len, slots_t, self._dev(flen))

    def _decode(self, max_steps: Optional[int] = None) -> List[Request]:
        if not self.running:
            return []
        remaining = min(r.params.max_tokens - len(r.output_ids) - (1 if not r.output_ids else 0)
                        for r in self.running.values())
        steps = max(1, min(self.decode_chunk if max_steps is None else max_steps, remaining))
        B = self._bucket(max(self.running) + 1)
        # context length reached by the end of this chunk decides the graph variant
        top = max(len(r.prompt_ids) + max(len(r.output_ids), 1) for r in self.running.values()) + steps
        mc = next(c for c in self._ctx_classes() if top <= c)
        nuc = self._wants_nucleus(self.running.values())
        cas = False
        if self.cascade and not nuc and len(self.running) >= 2:
            sh, r0 = self._shared_prefix()
            if sh * 64 >= self.cascade_min:
                cas = True
                self.s_cas.copy_(self._dev([sh, r0]))
                self.stats["cascade_chunks"] += 1
                # the per-row attention covers only the tokens past the shared prefix: its context class (partition
                # count) follows the longest suffix
                mc = next(c for c in self._ctx_classes() if top - 64 * sh <= c)
        t0 = time.perf_counter()
        graph = self.graphs.get((B, mc, nuc, cas)) if self.use_graphs else None
        # device-side stop detection: the sampler sets a host-mapped done flag when an answer ends (EOS, closed
        # JSON object, max_tokens, end of a scripted answer), so the chunk ends after the replay that finished a
        # request instead of running its remaining replays.  The flags are read after a wait for the replay that
        # wrote them, so every TP rank takes the same decision; a new arrival ends the chunk too on a single-rank
        # engine (a TP engine's followers cannot see rank 0's arrivals mid-chunk).
        #
        # Every rank of a TP replica must run the same replays.  Single rank: wait for replay i, then decide
        # (exact: the chunk ends right after the replay that finished an answer).  TP: the leader decides and
        # broadcasts the decision (ControlChannel.decide, one int on the gloo group); it decides on replay i - 1
        # while replay i runs, so no rank's GPU idles (at most one extra replay, which finished slots skip).
        # A leader wait that hits its deadline decides "run the chunk out" -- the ranks stay matched and the
        # fetch below raises EngineStalled.
        early = self.device_stop and max_steps is None and steps > 1
        tp_ctl = self.control if self.control is not None and self.control.world > 1 else None
        lag = 1 if tp_ctl is not None else 0
        live = list(self.running)
        events: List = []
        ran = 0
        tr = self.recovery_trace if self._trace_steps else None
        if tr is not None:
            tr.append((time.monotonic(), f"decode: {steps} steps, graph {graph is not None}"))
        # decode_time on the GPU: from an event behind the work already queued (a prefill this step did not wait
        # for) to one after the last replay -- host time would charge that prefill to the decode
        ev_t = None
        if self.gpu:
            ev_t = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev_t[0].record()
        for i in range(steps):
            if graph is not None:
                graph.replay()
                self.stats["graph_replays"] += 1
            else:
                self._decode_step(B, mc, nuc, cas)
            ran += 1
            if tr is not None:
                tr.append((time.monotonic(), f"decode: replay {i} enqueued"))
            if early and self.gpu and lag:
                ev = torch.cuda.Event()
                ev.record()
                events.append(ev)
            if not early or i + 1 >= steps or i < lag:
                continue
            stop = 0
            if tp_ctl is None or tp_ctl.rank == 0:
                if self._poll_event(events[i - lag] if lag and self.gpu else None):
                    stop = int(bool(self._done_host[live].any()) or (tp_ctl is None and bool(self._inbox)))
                else:
                    stop = 2          # deadline: run the chunk out, the fetch raises
            if tr is not None:
                tr.append((time.monotonic(), f"decode: replay {i - lag} polled, stop {stop}"))
            if tp_ctl is not None:
                stop = tp_ctl.decide(stop)
            if stop == 1:
                self.stats["early_chunk_stops"] += 1
                break
            if stop == 2:
                early = False
        self.stats["decode_steps"] += ran
        if ev_t is not None:
            ev_t[1].record()
        tp = self.model.tp
        tp.snapshot_health()             # rides on the bounded wait below
        if tr is not None:
            tr.append((time.monotonic(), "decode: fetch"))
        hist, nsteps = self._fetch(self.s_hist[:B], self.s_steps[:B], what="decode")
        tp.check_health()                # a failed collective raises into the decision service
        self.stats["decode_time"] += (ev_t[0].elapsed_time(ev_t[1]) / 1e3) if ev_t is not None \
            else time.perf_counter() - t0
        finished = []
        for slot, r in list(self.running.items()):
            n = int(nsteps[slot])
            new = hist[slot, len(r.output_ids):n].tolist()
            self.stats["decode_tokens"] += len(new)
            forced = r.params.forced_output_ids
            for tkn in new:
                if forced is not None:  # scripted answer; past its end: EOS
                    i = len(r.output_ids)
                    tkn = forced[i] if i < len(forced) else self.tok.eot_id
                r.output_ids.append(tkn)
                if self._stopped(r, tkn):
                    break
            if not r.finished and self.device_stop and self._done_host[slot]:
                # the device ended the answer (its stop rules are the host's; this only guards a disagreement,
                # which would otherwise leave a request whose slot no replay advances)
                self._finish(r, "length" if len(r.output_ids) >= r.params.max_tokens else "stop")
            if r.finished:
                finished.append(r)
            elif len(r.output_ids) >= r.params.max_tokens:
                self._finish(r, "length")
                finished.append(r)
        if self.metrics is not None:
            self.metrics.engine_tokens(sum(len(r.output_ids) for r in finished), self.kv_utilization())
        return finished

    def _stopped(self, r: Request, tkn: int) -> bool:
        p = r.params
        if not p.ignore_eos and (tkn in self.tok.eos_ids or tkn in p.stop_token_ids):
            r.output_ids.pop()
            self._finish(r, "stop")
            return True
        if p.stop_on_json_close and not p.ignore_eos and tkn in self._brace_ids():
            if json_object_closed(self.tok.decode(r.output_ids)):
                self._finish(r, "json")
                return True
        if len(r.output_ids) >= p.max_tokens:
            self._finish(r, "length")
            return True
        return False

    _brace_cache: Optional[set] = None

    def _brace_ids(self) -> set:
        if self._brace_cache is None:
            vocab = self.tok._tok.get_vocab()
            self._brace_cache = {i for s, i in vocab.items() if "}" in s}
        return self._brace_cache

    def _finish(self, r: Request, reason: str) -> None:
        if r.finished:
            return
        r.finished = True
        r.finish_reason = reason
        r.finish_time = time.perf_counter()
        # (arrival, first token, finish, tokens) of the last requests: queueing vs service time
        self.finished_log.append((r.arrival, r.first_token_time or r.finish_time, r.finish_time, len(r.output_ids),
                                 len(r.prompt_ids), int(getattr(r, "cached", 0) or 0)))
        if r.done is not None:
            # background-loop request: its caller holds the object, so drop it from the table here (the
            # caller never waits for the engine lock, which the loop holds for a whole step)
            self.requests.pop(r.rid, None)
            r.done.set()
        if r.slot >= 0:
            # fill kernels, never a host->device copy: this also runs on error paths while the stream is stalled
            try:
                self.s_ctx[r.slot:r.slot + 1].fill_(0)
                self.s_steps[r.slot:r.slot + 1].fill_(0)
            except Exception as e:   # noqa: BLE001 -- a faulted device: the request still ends (and its caller
                # returns); the engine goes not-ready and recovery resets every slot before serving again
                self.health.update(ready=False, reason=f"device error: {e}")
            self.running.pop(r.slot, None)
            if r in self.prefilling:
                self.prefilling.remove(r)
            self.free_slots.append(r.slot)
            self.free_slots.sort(reverse=True)
            r.slot = -1
        if r.blocks:
            self.allocator.release(r.blocks)
            r.blocks = []

    def step(self) -> List[Request]:
        with self.lock:
            self._step_t0 = time.monotonic()
            worker = self.control is not None and self.control.rank != 0
            if not worker and not self.ready:
                raise EngineUnavailable(self.health["reason"] or "decision engine not ready")
            try:
                out = self._step(worker)
                f = self.fault
                if worker and f is not None and f[0] == "raise" and self._steps == f[1]:
                    # fault injection (tests): this follower's collectives of the step ran, then "failed"
                    self.fault = None
                    raise CollectiveError(f"injected collective failure on rank {self.control.rank}")
                return out
            except (CollectiveError, EngineStalled, ops.KernelCheckError) as e:
                self._fail(str(e))
                raise

    def _step(self, worker: bool) -> List[Request]:
        if not worker:
            self.model.tp.ensure_healthy()
        self._drain_inbox()
        sync = self._sync()
        if worker:
            self._step_t0 = time.monotonic()   # a follower's step starts when the leader's schedule arrives
        if sync is False:
            raise StopIteration("engine stopped by rank 0")
        if sync == "reset":
            return []
        self._reap_aborted()
        self._share_deferred = False
        self._admit()
        if self.prefilling or self.waiting:
            with trace("engine.prefill"):
                self._prefill()
            if self._prefill_capped and self.running and self.prefilling:
                # a prompt cut by the mixed-step row cap continues after ONE decode step instead of a whole decode
                # chunk.  That step is needed: it syncs the rows the device finished (their context is zeroed on
                # the device), which the next mixed step must not carry as decode rows
                with trace("engine.decode"):
                    return self._decode(max_steps=1)
        if self._share_deferred and not any(r.output_ids for r in self.running.values()):
            # requests are waiting for a prefix this step published: admit them before the
            # first decode, so the batch decodes in lock-step (no extra tail of decode steps)
            return []
        with trace("engine.decode"):
            if self._spec_ok():
                return self._spec_decode()
            return self._decode()

    def kv_utilization(self) -> float:
        return 1.0 - self.allocator.num_free / self.allocator.num_blocks
