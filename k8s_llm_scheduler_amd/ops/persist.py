"""Layer-persistent decode (``csrc/kernels/decode_persist.hip``): every decoder layer of a decode step in one launch.

A model's state is the device table of its per-layer weight / KV-cache pointers plus the kernel's hand-off buffers
(epoch-tagged granules, attention chunk partials and counters, the epoch / finish ticket / error words).  The kernel
runs for TP = 1 and for one simulated TP rank (``--simulate-tp``: collectives skipped); real TP > 1 ranks keep the
four-launch layer with the fused GEMV all-reduce.  ``K8S_DECODE_PERSIST=1`` turns it on (default off until measured;
``models/llama.py`` picks it per step).  VERDICT r4 "next round" item 1; the reference's per-token loop is the remote
``chat_completion`` at ``/root/reference/scheduler.py:425-433`` (``max_tokens`` at ``:431``).
"""

from __future__ import annotations

import math
import os
from typing import Optional

import torch

BF16, F32, I32 = torch.bfloat16, torch.float32, torch.int32
MAX_ROWS = 2            # decode rows (sequences) per launch the kernel is built for
MAX_CHUNKS = 64         # 64-token attention chunks (contexts up to 4096 tokens)
TIMEOUT_S = float(os.environ.get("K8S_PERSIST_TIMEOUT_S", "0.25"))   # bound of every in-kernel wait


def enabled() -> bool:
    return os.environ.get("K8S_DECODE_PERSIST", "0") == "1"


class PersistentDecode:
    """Device state of the persistent decode kernel for one model (built lazily once the KV cache exists)."""

    def __init__(self, model):
        from . import native

        self.m = model
        c = model.cfg
        self.nat = native()
        self.H, self.nq, self.nkv, self.I = c.hidden, model.nq, model.nkv, model.I
        rc, self.gl, self.grid = self.nat.decode_persist_plan(MAX_ROWS, self.H, self.nq, self.nkv, self.I, MAX_CHUNKS)
        self.rc = rc
        self.table: Optional[torch.Tensor] = None
        self._kv_ptr = None
        if rc != 0:
            return
        dev = model.device
        L = c.num_layers
        assert self.nat.decode_persist_layer_bytes() == 6 * 8
        G = self.nq // self.nkv
        self.gran = torch.zeros(L * MAX_ROWS * self.gl * 8, dtype=torch.uint8, device=dev)
        self.part = torch.empty(MAX_ROWS * self.nkv * MAX_CHUNKS * (G * 128 + 2 * G), dtype=F32, device=dev)
        self.counters = torch.zeros(MAX_ROWS * self.nkv, dtype=I32, device=dev)
        self.sync = torch.zeros(96, dtype=I32, device=dev)
        self.sync[0] = 1                      # epochs start at 1: the zeroed granules never match
        self.err_host = torch.zeros(1, dtype=I32, pin_memory=True)
        self.trace: Optional[torch.Tensor] = None   # set_trace(True): chain-wave stamps of the next launches

    @property
    def ok(self) -> bool:
        return self.rc == 0

    def supports(self, B: int, max_context: int) -> bool:
        return (self.ok and 1 <= B <= MAX_ROWS and max_context <= MAX_CHUNKS * 64 and self.m.block_size == 16
                and self.m.kv_cache is not None)

    def _layer_table(self) -> torch.Tensor:
        kv = self.m.kv_cache
        if self.table is None or self._kv_ptr != kv.data_ptr():
            rows = []
            for l, w in enumerate(self.m.layers):
                rows.append([w.wqkv.data_ptr(), w.wo.data_ptr(), w.wgu.data_ptr(), w.wdown.data_ptr(),
                             kv[l, 0].data_ptr(), kv[l, 1].data_ptr()])
            self.table = torch.tensor(rows, dtype=torch.int64).to(self.m.device)
            self._kv_ptr = kv.data_ptr()
        return self.table

    def run(self, x0: torch.Tensor, context_lens: torch.Tensor, block_tables: torch.Tensor,
            max_context: int) -> torch.Tensor:
        """The decoder layers of one decode step: x0 [B, H] (embedding rows) -> final residual stream [B, H]."""
        B, H = x0.shape
        m = self.m
        pmax = max(1, math.ceil(max_context / 64))
        xout = torch.empty_like(x0)
        ticks = int(TIMEOUT_S * 1e8)          # s_memrealtime: 100 MHz
        self.nat.decode_persist(self._layer_table().data_ptr(), len(m.layers), x0.data_ptr(), xout.data_ptr(), B, H,
                                self.nq, self.nkv, self.I, float(m.cfg.rms_eps), float(m.scale),
                                m.cos_sin.data_ptr(), block_tables.data_ptr(), context_lens.data_ptr(),
                                block_tables.shape[1], pmax, self.gran.data_ptr(), self.part.data_ptr(),
                                self.counters.data_ptr(), self.sync.data_ptr(),
                                self.trace.data_ptr() if self.trace is not None else 0, ticks, -1)
        return xout

    def set_trace(self, on: bool) -> None:
        """Record s_memrealtime (100 MHz) stamps of every workgroup's chain wave at each hand-off of every layer
        ([grid, L, points] int64; tools/persist_trace.py reads them).  Profiling only."""
        if on and self.ok:
            pts = self.nat.decode_persist_trace_points()
            self.trace = torch.zeros(self.grid, len(self.m.layers), pts, dtype=torch.int64, device=self.m.device)
        else:
            self.trace = None

    # ---- failure detection: a timed-out in-kernel wait (bug or a CU missing from the grid) must not go unnoticed
    def snapshot_error(self) -> None:
        if self.ok:
            self.err_host.copy_(self.sync[64:65], non_blocking=True)

    def take_error(self) -> int:
        """The error bits seen by the last snapshot (after the stream synchronised); resets the device state."""
        if not self.ok:
            return 0
        e = int(self.err_host[0])
        if e:
            self.sync[64] = 0
            self.counters.zero_()
            self.err_host.zero_()
        return e
