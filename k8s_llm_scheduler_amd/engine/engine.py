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
"""

from __future__ import annotations

import gc
import itertools
import logging
from array import array
import math
import os
import random
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional, Sequence, Union

import torch

from .. import ops
from ..control.jsonextract import json_object_closed
from ..models.llama import LlamaModel
from ..parallel.comm import CollectiveError
from .sampling import SamplingParams
from .tokenizer import Tokenizer
from ..utils.tracing import trace

log = logging.getLogger(__name__)

BUCKETS = (1, 2, 4, 6, 8, 16, 32, 48, 64, 96, 128, 192, 256)   # (6: serving at ~5 in flight runs 6 rows, not 8)
# Single-sequence prompt chunks up to 512 tokens are padded to one of these lengths and replayed
# from a captured graph, which removes the host launch gaps between the ~10 kernels per layer
# (tools/prefill_probe.py, 256 tokens: TP=8 shapes 12.53 ms eager -> 12.28 ms replayed; TP=1 44.0 ms
# either way -- the chunk is GEMM-bound, profiles/rocprof_prefill_tp8.txt).  The padding tokens
# belong to no sequence (cu_q stops at the real length) and write their K/V into a scratch block.
PREFILL_GRAPH_BUCKETS = (64, 128, 192, 256, 320, 384, 448, 512)
MIXED_MIN_PROMPT_ROWS = 16   # a mixed step under the row cap still advances its prompts by at least this many tokens
_P_SPLIT = 6   # packed prefill-graph inputs of the two micro-batch halves: cu_q0 (2), ctx0, cu_q1 (2), ctx1


def split_prefill_meta(cu: Sequence[int], ctx: Sequence[int], T0: int) -> tuple:
    """Split a varlen prefill chunk at token ``T0`` into two micro-batches (``LlamaModel.forward_prefill``
    ``split``).  ``cu`` are the chunk's query offsets, ``ctx[s]`` sequence s's context length after the chunk.
    A sequence straddling T0 contributes its first part to half 0 (whose context then ends where that part
    ends) and the rest to half 1.  Returns ``((cu0, ctx0, seqs0), (cu1, ctx1, seqs1))`` with ``seqs`` the
    chunk-local sequence indices of each half (rows of the block table)."""
    halves = (([0], [], []), ([0], [], []))
    for s in range(len(cu) - 1):
        a, b = cu[s], cu[s + 1]
        for h, (lo, hi) in enumerate(((a, min(b, T0)), (max(a, T0), b))):
            if hi > lo:
                c, cx, sq = halves[h]
                c.append(c[-1] + hi - lo)
                cx.append(ctx[s] - (b - hi))
                sq.append(s)
    return halves


SPEC_GRAPH_T = 8     # rows of the captured single-sequence verify forward (last token + up to 7 drafts)
SPEC_MAX_BATCH = 8   # speculative steps only while at most this many sequences decode (drafting and the eager
                     # verify forward are per-step host work; larger batches keep the captured decode graphs)


def ngram_draft(seq: Sequence[int], k: int, n_max: int = 3) -> List[int]:
    """Prompt-lookup draft: the up to ``k`` tokens that followed the most recent earlier occurrence of the
    sequence's last n tokens (n = n_max .. 1, longest match first).  The search runs over the int32 bytes of the
    sequence (``bytes.rfind``), so drafting a 700-token context costs microseconds, not a Python scan."""
    L = len(seq)
    if k <= 0 or L < 2:
        return []
    buf = array("i", seq).tobytes()
    for n in range(min(n_max, L - 1), 0, -1):
        pat = buf[(L - n) * 4:]           # the last n tokens
        end = (L - 1) * 4                 # a match must leave at least one token after it
        while end >= len(pat):
            at = buf.rfind(pat, 0, end)
            if at < 0:
                break
            if at % 4 == 0:               # token-aligned
                s0 = at // 4 + n
                return list(seq[s0:s0 + k])
            end = at + len(pat) - 1       # misaligned hit: look further left
    return []


class _HostStage:
    """Ring of pinned host slots for small host -> device copies (LLMEngine._dev).  A slot is reused only once the copy
    that last used it has executed (its event).  When the device is that far behind -- a step that admits many
    requests behind a long prefill enqueues hundreds of copies -- the ring waits for the slot with a bounded event wait
    that releases the GIL (``wait_limit()``: the engine's call deadline / watchdog, as for every device wait) and
    raises EngineStalled only when that expires.  Larger tensors take a one-off pinned buffer."""

    SLOTS, SLOT_BYTES = 512, 256 << 10

    def __init__(self, wait_limit=None):
        self.buf = torch.empty(self.SLOTS * self.SLOT_BYTES, dtype=torch.uint8, pin_memory=True)
        self.events: List[Optional[torch.cuda.Event]] = [None] * self.SLOTS
        self.next = 0
        self.wait_limit = wait_limit     # () -> absolute time.monotonic() limit, or None (no limit set: 60 s)

    def _slot_free(self, ev: torch.cuda.Event) -> bool:
        if ev.query():
            return True
        lim = self.wait_limit() if self.wait_limit is not None else None
        budget = (lim - time.monotonic()) if lim is not None else 60.0
        return bool(ops.native().event_wait(ev.cuda_event, max(0.0, budget)))

    def to_device(self, t: torch.Tensor, device) -> torch.Tensor:
        t = t.contiguous()
        n = t.numel() * t.element_size()
        if n > self.SLOT_BYTES:
            return t.pin_memory().to(device, non_blocking=True)
        i = self.next
        ev = self.events[i]
        if ev is not None and not self._slot_free(ev):
            raise EngineStalled("host staging ring full: the device has not run the last "
                                f"{self.SLOTS} host-to-device copies within the deadline")
        self.next = (i + 1) % self.SLOTS
        view = self.buf[i * self.SLOT_BYTES:i * self.SLOT_BYTES + n]
        view.copy_(t.view(-1).view(torch.uint8))
        out = view.view(t.dtype).view(t.shape).to(device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        self.events[i] = ev
        return out


class EngineStalled(TimeoutError):
    """Device work of an engine step did not complete within the call deadline or the engine watchdog (a
    hung collective or kernel).  The engine stops accepting work until :meth:`LLMEngine.recover` succeeds."""


class EngineUnavailable(RuntimeError):
    """The engine is not ready: an earlier collective failure or stall has not been recovered yet."""


class RequestRejected(RuntimeError):
    """One request cannot be served (e.g. it does not fit in an empty KV cache); only that request fails."""

    def __init__(self, request, msg: str):
        super().__init__(msg)
        self.request = request


@dataclass
class Request:
    rid: int
    prompt_ids: List[int]
    params: SamplingParams
    seed: int
    arrival: float = field(default_factory=time.perf_counter)
    slot: int = -1
    blocks: List[int] = field(default_factory=list)
    computed: int = 0          # prompt tokens whose KV is in the cache
    cached: int = 0            # of which came from the prefix cache
    output_ids: List[int] = field(default_factory=list)
    finished: bool = False
    finish_reason: str = ""
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    aborted: bool = False
    done: Optional[threading.Event] = None      # set by _finish (background serving loop)
    error: Optional[BaseException] = None       # engine failure that ended the request


@dataclass
class Output:
    rid: int
    text: str
    token_ids: List[int]
    prompt_tokens: int
    cached_tokens: int
    finish_reason: str
    ttft: float
    latency: float


class LLMEngine:
    def __init__(self, model: LlamaModel, tokenizer: Tokenizer, *, max_batch: int = 64, block_size: int = 16,
                 num_blocks: Optional[int] = None, kv_cache_gb: float = 0.0, kv_cache_fraction: float = 0.85,
                 max_model_len: Optional[int] = None, max_prefill_tokens: int = 8192, cuda_graphs: bool = True,
                 prefix_caching: bool = True, decode_chunk: int = 4, seed: int = 0, metrics=None,
                 control=None, capture_nucleus: bool = False, speculative_tokens: int = 0,
                 watchdog_s: float = 60.0, on_unrecoverable: str = "stay", device_stop: bool = True,
                 mixed_steps: bool = True, mixed_step_rows: int = 256):
        self.model = model
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
        self.graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}   # (batch bucket, context class, nucleus)
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
                      "early_chunk_stops": 0}

    # ------------------------------------------------------------------ bounded device waits / health
    def _wait_limit(self) -> Optional[float]:
        lim = self._step_t0 + self.watchdog_s if self.watchdog_s > 0 else None
        if self._call_deadline is not None:
            lim = self._call_deadline if lim is None else min(lim, self._call_deadline)
        return lim

    def _wait_device(self, what: str) -> None:
        """Wait for the work enqueued so far on the engine's stream: an event polled against the call deadline
        and the watchdog (never a blocking synchronize, so a hung collective cannot block the host forever)."""
        if not self.gpu:
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._last_event = ev
        if not self._await(ev, what):
            self.recovery_trace.append((time.monotonic(), f"stalled: {what}"))
            self.stats["stalls"] += 1
            msg = f"engine stalled: {what} did not complete within the deadline (rank {self.model.tp.rank})"
            self._fail(msg)
            raise EngineStalled(msg)

    def _await(self, ev, what: Optional[str]) -> bool:
        """Poll ``ev``.  Leader (or single rank): False once the call deadline / watchdog passes.  TP follower: a
        follower's host bookkeeping must track the leader's schedule step for step, so it never gives up on its
        own -- past the watchdog it reports the stall to the leader (failure key in the store) and keeps waiting,
        until the work completes or the leader requests a reset (then EngineStalled)."""
        worker = self.control is not None and self.control.rank != 0
        limit = self._wait_limit()
        reported = False
        next_check = time.monotonic() + 0.2
        handle = ev.cuda_event
        # slices of a native wait that releases the GIL (ops event_wait): the control plane's threads keep running
        # while the engine waits for its device (a Python poll loop here starved them: round-3 serving regression)
        while True:
            now = time.monotonic()
            if worker:
                budget = max(0.0, next_check - now)
            else:
                budget = 0.05 if limit is None else max(0.0, min(0.05, limit - now))
            if ops.native().event_wait(handle, budget):
                return True
            now = time.monotonic()
            if worker:
                if limit is not None and now > limit and not reported:
                    reported = True
                    self.stats["stalls"] += 1
                    self._fail(f"engine stalled: {what or 'a step'} did not complete within the watchdog "
                               f"(rank {self.model.tp.rank})")
                if now >= next_check:
                    next_check = now + 0.05
                    if self.control.reset_generation() > self._reset_seen:
                        raise EngineStalled(f"rank 0 requested a reset while {what or 'a step'} was in flight "
                                            f"(rank {self.model.tp.rank})")
            elif limit is not None and now >= limit:
                return False

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

    def _poll_event(self, ev=None) -> bool:
        """Wait (bounded by the call deadline / watchdog) for ``ev`` or, without one, for the work enqueued so far;
        False at the deadline (nothing raised: the caller keeps the TP ranks' schedules matched)."""
        if not self.gpu:
            return True
        if ev is None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        return self._await(ev, None)

    def _fetch(self, *ts: torch.Tensor, what: str = "step") -> List[torch.Tensor]:
        """Small device tensors -> host, through reused pinned buffers and one bounded wait.  The returned
        tensors are overwritten by the next fetch: read them right away."""
        if not self.gpu:
            return [t.clone() for t in ts]
        outs = []
        for i, t in enumerate(ts):
            key = (i, t.dtype, tuple(t.shape))
            buf = self._pinned.get(key)
            if buf is None:
                buf = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                self._pinned[key] = buf
            buf.copy_(t, non_blocking=True)
            outs.append(buf)
        if self._trace_steps:
            self.recovery_trace.append((time.monotonic(), f"fetch {what}: waiting"))
        self._wait_device(what)
        if self._pf_events:
            self._account_prefill()
        return outs

    def _fail(self, reason: str) -> None:
        if self.health["ready"]:
            log.error(f"Decision engine not ready: {reason}")
            if self.control is not None and self.control.rank != 0:
                try:
                    self.control.report_failure(reason)
                except Exception as e:  # noqa: BLE001
                    log.error(f"failure report to rank 0 failed: {e!r}")
        self.health.update(ready=False, reason=reason, failures=self.health["failures"] + 1, since=time.time())
        if self.metrics is not None and hasattr(self.metrics, "engine_health"):
            self.metrics.engine_health(False)

    @property
    def ready(self) -> bool:
        return bool(self.health["ready"])

    def health_probe(self):
        """(live, ready, detail) for /healthz and /readyz: live while the serving loop (if started) runs."""
        t = self._bg_thread
        live = t is None or t.is_alive()
        peer = self.control.peer_failure() if self.control is not None and self.control.rank == 0 else None
        return live, self.ready and not peer, {"peer_failure": peer, "reason": self.health["reason"], "failures": self.health["failures"],
                                  "recoveries": self.health["recoveries"], "stalls": self.stats["stalls"]}

    def _drained(self, timeout_s: float) -> bool:
        """True once every piece of device work this engine enqueued has completed (bounded poll)."""
        if not self.gpu:
            return True
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return bool(ops.native().event_wait(ev.cuda_event, max(0.0, timeout_s)))

    def recover(self, drain_timeout: float = 0.0) -> bool:
        """Bring a failed engine back.  The device must drain within ``drain_timeout`` s (a
        stalled peer that resumes lets the parked collectives finish; an RCCL communicator is aborted so its
        parked operations error out).  Then every rank of the replica -- told through the control channel --
        resets its collectives (xGMI protocol state zeroed, a broken RCCL communicator rebuilt, bounded
        barrier) and drops all in-flight requests and cached prefixes.  Returns True when ready again."""
        tr = self.recovery_trace
        tr.append((time.monotonic(), "recover: waiting for the engine lock"))
        with self.lock:
            if self.ready:
                return True
            tp = self.model.tp
            drained = self._drained(drain_timeout)
            tr.append((time.monotonic(), f"recover: drained={drained}"))
            if not drained:
                # ncclCommAbort can block until the device work queued behind the stalled collective drains, so it
                # runs on a helper thread: this call (and every retry until the device drains) returns at once
                if tp.rccl is not None and not tp.rccl.aborted and self._abort_thread is None:
                    self._abort_thread = threading.Thread(target=tp.abort_rccl, name="rccl-abort", daemon=True)
                    self._abort_thread.start()
                return False
            if self._abort_thread is not None:
                self._abort_thread.join(timeout=max(drain_timeout, 1.0))
                if self._abort_thread.is_alive():
                    return False
                self._abort_thread = None
            return self._reset_all(announce=True)

    def _reset_all(self, announce: bool) -> bool:
        """Every rank: end all requests, free every slot, drop the prefix cache (an abandoned step may have
        committed KV that was never written), reset the collectives.  ``announce``: rank 0 first tells the
        other ranks of the replica to do the same."""
        tp = self.model.tp
        tr = self.recovery_trace
        try:
            if announce and self.control is not None and self.control.rank == 0:
                self.control.request_reset()   # releases followers parked in a device wait (_await)
                self.control.exchange({"new": [], "abort": [], "stop": False, "reset": True})
                self.control.clear_failures()
                tr.append((time.monotonic(), "reset: followers told"))
            err = EngineUnavailable(self.health["reason"] or "engine reset")
            for r in list(self.requests.values()) + list(self.waiting) + list(self.prefilling) + \
                    list(self.running.values()):
                if not r.finished:
                    r.error = r.error or err
                    self._finish(r, "error")
            with self._inbox_lock:
                pending, self._inbox = self._inbox, []
            for r in pending:
                r.error = err
                r.finished, r.finish_reason = True, "error"
                if r.done is not None:
                    r.done.set()
            self.requests.clear()
            self.waiting.clear()
            self.prefilling.clear()
            self.running.clear()
            self._outbox = []
            self.free_slots = list(range(self.max_batch - 1, -1, -1))
            self.allocator = ops.native().BlockAllocator(self.num_blocks, self.block_size, self.prefix_caching) \
                if ops.available() else _PyBlockAllocator(self.num_blocks, self.block_size, self.prefix_caching)
            if self.gpu:
                self.s_ctx.zero_()
                self.s_steps.zero_()
                tr.append((time.monotonic(), "reset: collectives"))
                tp.reset_collectives(self.control, timeout_s=max(10.0, self.watchdog_s))
                torch.cuda.synchronize(self.device)
                tr.append((time.monotonic(), "reset: collectives done"))
            else:
                tp.reset_collectives(self.control, timeout_s=max(10.0, self.watchdog_s))
        except Exception as e:  # noqa: BLE001 -- recovery failed: stay (or exit) not ready
            self._fail(f"recovery failed: {e!r}")
            self._unrecoverable(f"recovery failed: {e!r}")
            return False
        self.health.update(ready=True, reason="", recoveries=self.health["recoveries"] + 1, since=time.time())
        if self.metrics is not None and hasattr(self.metrics, "engine_health"):
            self.metrics.engine_health(True)
        log.warning(f"Decision engine recovered (rank {tp.rank}; recoveries {self.health['recoveries']})")
        return True

    def _unrecoverable(self, why: str) -> None:
        if self.on_unrecoverable == "exit":
            log.critical(f"Decision engine cannot recover ({why}); exiting so the pod restarts")
            logging.shutdown()
            os._exit(70)

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

    def _ctx_classes(self) -> List[int]:
        """Context-length classes with their own decode graph: contexts <= 1024 tokens (one
        attention partition per sequence: no partial buffers, no merge kernel) and the rest."""
        return sorted({min(1024, self.max_model_len), self.max_model_len})

    def _decode_step(self, B: int, max_context: Optional[int] = None, nucleus: bool = False) -> None:
        logits = self.model.forward_decode(self.s_tokens[:B], self.s_ctx[:B], self.s_bt[:B],
                                           max_context or self.max_model_len)
        ops.sample(logits, self.s_temp[:B], self.s_top_p[:B], self.s_seeds[:B], self.s_ctx[:B],
                   shards=logits.shape[0], tokens_out=self.s_tokens[:B], ctx_inc=self.s_ctx[:B],
                   hist=self.s_hist[:B], steps=self.s_steps[:B], nucleus=nucleus, stop=self._stop_args())

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
        buckets = buckets or [b for b in BUCKETS if b <= self.max_batch]
        stream = torch.cuda.Stream(self.device)
        for B in sorted(set(buckets)):
            for mc in self._ctx_classes():
                for nuc in ((False, True) if nucleus else (False,)):
                    if (B, mc, nuc) in self.graphs:
                        continue
                    stream.wait_stream(torch.cuda.current_stream(self.device))
                    with torch.cuda.stream(stream):
                        self._decode_step(B, mc, nuc)   # warm-up: allocator + lazy init outside capture
                    torch.cuda.current_stream(self.device).wait_stream(stream)
                    torch.cuda.synchronize(self.device)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=self._graph_pool, stream=stream):
                        self._decode_step(B, mc, nuc)
                    if self._graph_pool is None:
                        self._graph_pool = g.pool()
                    self.graphs[(B, mc, nuc)] = g
        if self.prefill_graphs_enabled():
            for Tb in PREFILL_GRAPH_BUCKETS:
                if Tb in self.prefill_graphs or not self._prefill_bucket_capturable(Tb):
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
        gather_bytes = logits_rows * self.model.lm_head.shape[0] * 4
        # captured with tp.capture_on_xgmi: every all-reduce that fits the capacity stays on xGMI
        return ar_bytes <= tp.xgmi.max_allreduce_bytes and gather_bytes <= tp.xgmi.slot_bytes

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

    def _sync(self):
        """Replicate rank 0's new requests and aborts to every rank.  Returns False on a stop command (worker
        shutdown), "reset" after a recovery reset (workers), else True.  Rank 0 first checks the followers'
        failure reports: a collective failure seen by any rank fails this step before it launches anything."""
        if self.control is None:
            return True
        if self.control.rank == 0:
            peer = self.control.peer_failure()
            if peer:
                raise CollectiveError(peer)
            msg = {"new": [(r.rid, r.prompt_ids, r.params.__dict__, r.seed) for r in self._outbox],
                   "abort": sorted(r.rid for r in self.requests.values() if r.aborted and not r.finished),
                   "stop": False}
            self._outbox = []
            self.control.exchange(msg)
            return True
        msg = self.control.exchange(None)
        if msg.get("stop"):
            return False
        if msg.get("reset"):
            self._reset_seen = self.control.reset_generation()
            if not self._drained(max(5.0, self.watchdog_s)):
                # no reset with the device busy (reset_collectives would block in a synchronize): stay not ready,
                # the leader's bounded barrier times out and it retries (or exits, engine.on_unrecoverable)
                self._fail("reset: device did not drain")
                self._unrecoverable("device did not drain for the reset")
                return "reset"
            self._reset_all(announce=False)
            return "reset"
        for rid, ids, pd, seed in msg["new"]:
            r = Request(rid, list(ids), SamplingParams(**pd), seed)
            self.requests[rid] = r
            self.waiting.append(r)
        for rid in msg["abort"]:
            if rid in self.requests:
                self.requests[rid].aborted = True
        self._steps += 1
        f = self.fault
        if f is not None and f[0] == "stall" and self._steps == f[1]:
            self.fault = None
            time.sleep(f[2])   # fault injection (tests): this follower stalls before its device work
        elif f is not None and f[0] == "stall_on_key":
            st = self.control.store()
            if st is not None and st.check([f[1]]):   # (tests) stall at the first step after the leader sets the key
                self.fault = None
                st.delete_key(f[1])
                time.sleep(f[2])
        return True

    def shutdown_workers(self) -> None:
        if self.control is not None and self.control.rank == 0:
            self.control.stop_monitor()
            self.control.exchange({"new": [], "abort": [], "stop": True})
            self.control.flush()

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
                       stop=self._stop_args())
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
            toks = ops.sample(sub, temp, top_p, seeds, ctr, shards=sub.shape[0], nucleus=self._wants_nucleus(rs))
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
        t0 = time.perf_counter()
        graph = self.graphs.get((B, mc, nuc)) if self.use_graphs else None
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
                self._decode_step(B, mc, nuc)
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
        self.model.snapshot_decode_health()
        if tr is not None:
            tr.append((time.monotonic(), "decode: fetch"))
        hist, nsteps = self._fetch(self.s_hist[:B], self.s_steps[:B], what="decode")
        tp.check_health()                # a failed collective raises into the decision service
        self.model.check_decode_health()
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
                              shards=logits.shape[0], nucleus=self._wants_nucleus(r for r, _, _ in rows))
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
            except (CollectiveError, EngineStalled) as e:
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

    def serve_worker(self) -> None:
        """Non-zero TP ranks: follow rank 0's schedule until it sends stop.  A collective failure or stall seen
        here is reported to rank 0 with the next exchange; rank 0's reset command recovers this rank."""
        assert self.control is not None and self.control.rank != 0
        while True:
            try:
                self.step()
            except StopIteration:
                return
            except RequestRejected as e:
                # the leader rejected the same request at the same point of its step (it replays this schedule):
                # finish it here too and keep following
                r = e.request
                r.error = e
                self._finish(r, "error")
            except (CollectiveError, EngineStalled) as e:
                log.error(f"TP worker rank {self.control.rank}: {e}; waiting for rank 0's reset")

    def kv_utilization(self) -> float:
        return 1.0 - self.allocator.num_free / self.allocator.num_blocks

    # ------------------------------------------------------------------ background serving loop
    def start_background(self) -> None:
        """Run engine steps on a dedicated thread.  generate() then only enqueues and waits, so requests
        from any number of caller threads (the scheduler's continuous mode) join the running batch at the
        next step instead of waiting for each other's calls to finish."""
        if self._bg_thread is not None:
            return
        self._bg_stop = False
        self._bg_error = None
        self._bg_thread = threading.Thread(target=self._bg_loop, name="engine-loop", daemon=True)
        self._bg_thread.start()

    def stop_background(self) -> None:
        t = self._bg_thread
        if t is None:
            return
        with self._wake:
            self._bg_stop = True
            self._wake.notify_all()
        t.join()
        self._bg_thread = None

    @property
    def background(self) -> bool:
        return self._bg_thread is not None

    def _bg_loop(self) -> None:
        if self.gpu:
            torch.cuda.set_device(self.s_tokens.device)   # (the tensors carry the index; "cuda" alone does not)
        while True:
            with self._wake:
                while not self._bg_stop and not self._inbox and not self.has_work():
                    self._wake.wait(0.05)
                if self._bg_stop:
                    return
            try:
                if not self.ready:
                    # requests queued while not ready fail fast (the decision service falls back); a recovery
                    # attempt with a short drain bound runs before each wait
                    if not self.recover(drain_timeout=0.05):
                        self._fail_pending(EngineUnavailable(self.health["reason"] or "engine not ready"))
                        with self._wake:
                            self._wake.wait(0.05)
                        continue
                self.step()
                time.sleep(0)   # let threads blocked on the GIL / engine lock in before the next step
            except RequestRejected as e:   # only the offending request fails
                r = e.request
                r.error = e
                self._finish(r, "error")
            except (CollectiveError, EngineStalled, EngineUnavailable) as e:
                # collective state unknown: every in-flight request fails; recovery runs on the next iteration
                self._bg_error = e
                self._fail_pending(e)
            except Exception as e:  # noqa: BLE001 -- host-side bug: fail what was in flight, keep serving
                log.error(f"Engine step failed: {e!r}")
                self._bg_error = e
                self._fail_pending(e)

    def _fail_pending(self, e: BaseException) -> None:
        with self.lock:
            self._drain_inbox()
            for r in list(self.requests.values()):
                if not r.finished:
                    r.error = e
                    if r in self.waiting:
                        self.waiting.remove(r)
                    self._finish(r, "error")

    # ------------------------------------------------------------------ blocking API
    def output(self, r: Request) -> Output:
        end = r.finish_time or time.perf_counter()
        return Output(r.rid, self.tok.decode(r.output_ids), list(r.output_ids), len(r.prompt_ids), r.cached,
                      r.finish_reason, (r.first_token_time or end) - r.arrival, end - r.arrival)

    def generate(self, prompts: Sequence[Union[str, List[int]]],
                 params: Union[SamplingParams, Sequence[SamplingParams], None] = None,
                 deadline: Optional[float] = None) -> List[Output]:
        """Run the given requests to completion (continuous batching with whatever else is
        queued).  ``deadline`` (time.monotonic) aborts unfinished requests and raises
        TimeoutError -- the decision service counts that as an engine failure."""
        if params is None or isinstance(params, SamplingParams):
            params = [params or SamplingParams()] * len(prompts)
        if self._bg_thread is not None:
            return self._generate_bg(prompts, params, deadline)
        self.recovery_trace.append((time.monotonic(), f"generate: ready={self.ready}"))
        if not self.ready and not self.recover(drain_timeout=0.05):
            raise EngineUnavailable(self.health["reason"] or "decision engine not ready")
        with self.lock:
            self._call_deadline = deadline
            try:
                return self._generate_sync(prompts, params, deadline)
            finally:
                self._call_deadline = None

    def _generate_sync(self, prompts, params, deadline: Optional[float]) -> List[Output]:
        reqs = [self.add_request(p, sp) for p, sp in zip(prompts, params)]
        while not all(r.finished for r in reqs):
            if deadline is not None and time.monotonic() > deadline:
                for r in reqs:
                    if not r.finished:
                        r.aborted = True
                if self.control is None:
                    self._reap_aborted()
                for r in reqs:
                    self.requests.pop(r.rid, None) if r.finished else None
                raise TimeoutError("decision engine deadline exceeded")
            try:
                self.step()
            except StopIteration:
                raise
            except RequestRejected as e:
                e.request.error = e
                self._finish(e.request, "error")
                if e.request in reqs:
                    for r in reqs:
                        if not r.finished:
                            if r in self.waiting:
                                self.waiting.remove(r)
                            self._finish(r, "error")
                        self.requests.pop(r.rid, None)
                    raise
            except Exception:
                # an engine / collective failure ends these requests (their slots and KV blocks
                # are released) and propagates to the decision service's retry / breaker path
                for r in reqs:
                    if not r.finished:
                        if r in self.waiting:
                            self.waiting.remove(r)
                        self._finish(r, "error")
                    self.requests.pop(r.rid, None)
                raise
        outs = [self.output(r) for r in reqs]
        for r in reqs:
            self.requests.pop(r.rid, None)
        return outs

    def _generate_bg(self, prompts, params, deadline: Optional[float]) -> List[Output]:
        reqs = [self.add_request(p, sp) for p, sp in zip(prompts, params)]
        for r in reqs:
            left = None if deadline is None else max(0.0, deadline - time.monotonic())
            if not r.done.wait(timeout=left):
                for q in reqs:
                    q.aborted = True   # reaped (and finished) by the loop's next step; no engine lock here
                with self._wake:
                    self._wake.notify()
                raise TimeoutError("decision engine deadline exceeded")
        failed = next((r.error for r in reqs if r.error is not None), None)
        if failed is not None:
            raise RuntimeError(f"decision engine failure: {failed}") from failed
        return [self.output(r) for r in reqs]


class _PyBlockAllocator:
    """Pure-Python stand-in used only when the native extension is unavailable (CPU tests)."""

    class _A:
        def __init__(self, blocks, cached):
            self.blocks, self.cached_tokens = blocks, cached

    def __init__(self, num_blocks: int, block_size: int, prefix_caching: bool):
        self.num_blocks, self.block_size = num_blocks, block_size
        self._free = list(range(num_blocks - 1, -1, -1))

    @property
    def num_free(self) -> int:
        return len(self._free)

    def can_allocate(self, tokens, total) -> bool:
        return math.ceil(total / self.block_size) <= len(self._free)

    def allocate(self, tokens, total):
        n = math.ceil(total / self.block_size)
        if n > len(self._free):
            raise RuntimeError("KV cache exhausted")
        return self._A([self._free.pop() for _ in range(n)], 0)

    def commit_prefix(self, blocks, tokens, n) -> None:
        pass

    def release(self, blocks) -> None:
        self._free.extend(blocks)
