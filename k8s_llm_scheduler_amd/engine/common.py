"""Engine data types and constants shared by the scheduler core and its mixins (graph capture, recovery,
speculative decoding, serving loop): requests / outputs, the engine's exceptions, the pinned host staging ring, decode
and prefill-graph buckets, the prefill micro-batch split and the prompt-lookup drafter.  Split out of ``engine.py``
(VERDICT r4 "next round" item 8); the reference's request is one scheduling decision
(``/root/reference/scheduler.py:396-460``)."""

from __future__ import annotations

from array import array
import math
import threading
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from .. import ops
from .sampling import SamplingParams


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
