"""Llama-3 decoder (8B / 70B / tiny) with Megatron-style tensor parallelism.

Sharding per rank (TP = t): QKV and gate/up are column-parallel (this rank's heads / FFN slice,
fused into one weight each: ``wqkv`` = [q; k; v] rows, ``wgu`` = [gate; up] rows), O and down are
row-parallel (followed by an all-reduce), the LM head is vocabulary-parallel (fp32 logits are
all-gathered shard-major), the embedding is replicated (no collective on the input side).

Every op on a CUDA tensor is a hand-written gfx950 kernel from ``ops``; projections with more than
``ops.GEMV_MAX_M`` rows run the hand-written MFMA GEMM except the prefill-size shapes where its tuned
plan table measured hipBLASLt faster.  The same code runs on CPU through the fp32 reference ops, which
is how TP=k == TP=1 is tested with gloo.

Weights: deterministic hash-uniform random init (identical global tensors for every TP degree
and device; BASELINE allows random-init weights) or a HuggingFace safetensors checkpoint,
loaded shard-by-shard with ``safetensors`` (no pickle).  ``weight_dtype="fp8"`` (BASELINE
config 5) stores the four projection matrices of every layer as row-scaled OCP e4m3
(:class:`ops.Fp8Weight`, quantized on the device right after each layer is built); embedding,
norms and the LM head stay bf16 (``K8S_FP8_LM_HEAD=1``: the LM head too).
"""

from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional

import torch

from .. import ops
from ..ops import reference as ref
from ..parallel import TPGroup
from .config import LlamaConfig

_TID_EMBED, _TID_LM, _TID_NORM = 1_000_001, 1_000_002, 1_000_003


def _tid(layer: int, k: int) -> int:
    return layer * 16 + k


@dataclass
class LayerWeights:
    ln1: torch.Tensor
    wqkv: torch.Tensor
    wo: torch.Tensor
    ln2: torch.Tensor
    wgu: torch.Tensor
    wdown: torch.Tensor


class LlamaModel:
    def __init__(self, cfg: LlamaConfig, tp: Optional[TPGroup] = None, device: str | torch.device = "cpu",
                 dtype: torch.dtype = torch.bfloat16, seed: int = 0, weights: Optional[str] = None,
                 max_model_len: int = 8192, weight_dtype: str = "bf16", fold_norm: bool = True):
        self.cfg = cfg
        # RMSNorm weights are folded into the projection that follows them (W' = W * gamma, one
        # elementwise pass at load time): the decode GEMVs then apply only 1/rms, in their epilogue
        # (gemv.hip NORM == 2), and prefill normalises with gamma = 1.  Mathematically identical.
        self.norm_folded = fold_norm
        self.tp = tp or TPGroup()
        cfg.validate_tp(self.tp.world)
        self.device = torch.device(device)
        self.dtype = dtype
        if weight_dtype not in ("bf16", "fp8"):
            raise ValueError(f"weight_dtype must be bf16 or fp8, got {weight_dtype!r}")
        self.weight_dtype = weight_dtype
        self.seed = seed
        t, r = self.tp.world, self.tp.rank
        self.nq = cfg.num_heads // t
        if cfg.num_kv_heads >= t:
            self.nkv = cfg.num_kv_heads // t
            self.kv0 = r * self.nkv
        else:  # replicate kv heads when tp > num_kv_heads
            self.nkv = 1
            self.kv0 = r * cfg.num_kv_heads // t
        self.I = cfg.intermediate // t
        self.Vs = cfg.vocab // t
        self.D = cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.D)
        self.max_model_len = min(max_model_len, cfg.max_position)
        self.cos_sin = ref.rope_table(self.D, self.max_model_len, cfg.rope_theta, cfg.rope_scaling).to(self.device)
        self.layers: List[LayerWeights] = []
        if weights:
            self._load_safetensors(Path(weights))
        else:
            self._random_init()
        if self.norm_folded:
            self.lm_head = self._fold(self.lm_head, self.norm)
            self.norm = self._ones()
        if weight_dtype == "fp8" and os.environ.get("K8S_FP8_LM_HEAD", "0") == "1":
            # opt-in: the LM head as row-scaled e4m3 too (half its 2.1 GB stream per decode step at TP = 1); the
            # logits then carry e4m3 weight rounding, which sampling at temperature > 0 does not resolve
            self.lm_head = ops.quantize_fp8(self.lm_head)
        self.kv_cache: Optional[torch.Tensor] = None
        self.block_size = 16

    # ------------------------------------------------------------------ weights
    def _new(self, rows: int, cols: int) -> torch.Tensor:
        return torch.empty(rows, cols, dtype=self.dtype, device=self.device)

    def _random_init(self) -> None:
        c, r, s = self.cfg, self.tp.rank, self.seed
        H, D = c.hidden, self.D
        a = c.init_std * math.sqrt(3.0)          # uniform(-a, a) has std init_std
        a_out = a / math.sqrt(2.0 * c.num_layers)  # GPT-2 style residual-branch scaling
        ones = lambda tid: ops.hash_init_(self._new(1, H), H, 0, 0, s, tid, 0.05, 1.0).view(H)
        self.embed = ops.hash_init_(self._new(c.vocab, H), H, 0, 0, s, _TID_EMBED, a * 10)
        for l in range(c.num_layers):
            wqkv = self._new((self.nq + 2 * self.nkv) * D, H)
            nq_rows = self.nq * D
            kv_rows = self.nkv * D
            ops.hash_init_(wqkv[:nq_rows], H, r * nq_rows, 0, s, _tid(l, 0), a)
            ops.hash_init_(wqkv[nq_rows:nq_rows + kv_rows], H, self.kv0 * D, 0, s, _tid(l, 1), a)
            ops.hash_init_(wqkv[nq_rows + kv_rows:], H, self.kv0 * D, 0, s, _tid(l, 2), a)
            wo = ops.hash_init_(self._new(H, nq_rows), c.num_heads * D, 0, r * nq_rows, s, _tid(l, 3), a_out)
            wgu = self._new(2 * self.I, H)
            ops.hash_init_(wgu[:self.I], H, r * self.I, 0, s, _tid(l, 4), a)
            ops.hash_init_(wgu[self.I:], H, r * self.I, 0, s, _tid(l, 5), a)
            wd = ops.hash_init_(self._new(H, self.I), c.intermediate, 0, r * self.I, s, _tid(l, 6), a_out)
            self._add_layer(LayerWeights(ones(_tid(l, 7)), wqkv, wo, ones(_tid(l, 8)), wgu, wd))
        self.norm = ones(_TID_NORM)
        self.lm_head = ops.hash_init_(self._new(self.Vs, H), H, r * self.Vs, 0, s, _TID_LM, a)

    def _load_safetensors(self, path: Path) -> None:
        from safetensors import safe_open

        files = sorted(path.glob("*.safetensors"))
        if not files:
            raise FileNotFoundError(f"no *.safetensors in {path}")
        index: Dict[str, Path] = {}
        for f in files:
            with safe_open(str(f), framework="pt") as h:
                for k in h.keys():
                    index[k] = f
        handles: Dict[Path, object] = {}

        def sl(name: str, dim: int = -1, start: int = 0, stop: Optional[int] = None) -> torch.Tensor:
            f = index[name]
            if f not in handles:
                handles[f] = safe_open(str(f), framework="pt")
            s = handles[f].get_slice(name)
            if dim == 0:
                t = s[start:stop]
            elif dim == 1:
                t = s[:, start:stop]
            else:
                t = s[:]
            return t.to(dtype=self.dtype).to(self.device)

        c, r, D = self.cfg, self.tp.rank, self.D
        p = "model.layers.{}."
        q_rows, kv_rows = self.nq * D, self.nkv * D
        self.embed = sl("model.embed_tokens.weight")
        for l in range(c.num_layers):
            pre = p.format(l)
            q = sl(pre + "self_attn.q_proj.weight", 0, r * q_rows, (r + 1) * q_rows)
            k = sl(pre + "self_attn.k_proj.weight", 0, self.kv0 * D, self.kv0 * D + kv_rows)
            v = sl(pre + "self_attn.v_proj.weight", 0, self.kv0 * D, self.kv0 * D + kv_rows)
            o = sl(pre + "self_attn.o_proj.weight", 1, r * q_rows, (r + 1) * q_rows)
            g = sl(pre + "mlp.gate_proj.weight", 0, r * self.I, (r + 1) * self.I)
            u = sl(pre + "mlp.up_proj.weight", 0, r * self.I, (r + 1) * self.I)
            d = sl(pre + "mlp.down_proj.weight", 1, r * self.I, (r + 1) * self.I)
            self._add_layer(LayerWeights(sl(pre + "input_layernorm.weight"), torch.cat([q, k, v]).contiguous(),
                                         o.contiguous(), sl(pre + "post_attention_layernorm.weight"),
                                         torch.cat([g, u]).contiguous(), d.contiguous()))
        self.norm = sl("model.norm.weight")
        lm = "lm_head.weight" if "lm_head.weight" in index else "model.embed_tokens.weight"
        self.lm_head = sl(lm, 0, r * self.Vs, (r + 1) * self.Vs).contiguous()

    def _ones(self) -> torch.Tensor:
        if getattr(self, "_ones_t", None) is None:
            self._ones_t = torch.ones(self.cfg.hidden, dtype=self.dtype, device=self.device)
        return self._ones_t

    @staticmethod
    def _fold(w: torch.Tensor, gamma: torch.Tensor) -> torch.Tensor:
        """W[n, k] * gamma[k] (bf16 result), in place."""
        return w.mul_(gamma.view(1, -1).to(w.dtype))

    def _add_layer(self, lw: LayerWeights) -> None:
        if self.norm_folded:
            lw.wqkv, lw.wgu = self._fold(lw.wqkv, lw.ln1), self._fold(lw.wgu, lw.ln2)
            lw.ln1 = lw.ln2 = self._ones()
        if self.weight_dtype == "fp8":
            lw.wqkv, lw.wo, lw.wgu, lw.wdown = (ops.quantize_fp8(w) for w in (lw.wqkv, lw.wo, lw.wgu, lw.wdown))
        self.layers.append(lw)

    def weight_bytes(self) -> int:
        nb = lambda t: t.nbytes() if isinstance(t, ops.Fp8Weight) else t.numel() * t.element_size()
        n = sum(nb(t) for t in (self.embed, self.norm, self.lm_head))
        for w in self.layers:
            n += sum(nb(t) for t in (w.ln1, w.wqkv, w.wo, w.ln2, w.wgu, w.wdown))
        return n

    # ------------------------------------------------------------------ KV cache
    def allocate_kv(self, num_blocks: int, block_size: int) -> torch.Tensor:
        self.block_size = block_size
        self.kv_cache = torch.zeros(self.cfg.num_layers, 2, num_blocks * block_size, self.nkv, self.D,
                                    dtype=self.dtype, device=self.device)
        if ops.CHECKED and self.device.type == "cuda":   # bounds of the checked kernels (K8S_CHECKED=1)
            ops.check_enable(self.device, num_blocks * block_size, num_blocks, self.cfg.vocab)
        return self.kv_cache

    def kv_bytes_per_block(self, block_size: int) -> int:
        return self.cfg.num_layers * 2 * block_size * self.nkv * self.D * torch.finfo(self.dtype).bits // 8

    # ------------------------------------------------------------------ forward
    def _layers_folded(self, h, attn) -> torch.Tensor:
        """All decoder layers with the norm gammas folded into the weights (the default).  The residual stream
        ``r`` feeds the pre-norm projections directly: their RMS statistics are the GEMM's prologue
        (ops.linear_rms), and the row-parallel projections add their output into ``r`` in the GEMM epilogue
        (TP=1, ops.linear_residual) or in the all-reduce (TP>1, the xGMI kernels fuse it) -- no RMSNorm or
        residual-add kernels between the GEMMs.  Returns the final residual stream."""
        eps = self.cfg.rms_eps
        r_mx = None   # fp8 GEMM rows at TP = 1: the MX copy of r written by its producer (K16)
        if isinstance(h, tuple):   # (embedding rows, their MX copy)
            h, r_mx = h
        r = h.clone()
        tp1 = self.tp.world == 1 or self.tp.simulate
        L = len(self.layers)
        for l, w in enumerate(self.layers):
            qkv = ops.linear_rms(r, w.wqkv, eps, x_mx=r_mx)
            a = attn(l, qkv)
            if tp1:
                r, r_mx = ops.linear_residual(a, w.wo, r, mx_next=w.wgu)
            else:
                o = ops.linear(a, w.wo)
                self.tp.all_reduce_(o, residual=r)     # o = r + attention branch
                r = o
            g = ops.linear_rms(r, w.wgu, eps, ops.EPI_SWIGLU, mx_consumer=w.wdown, x_mx=r_mx)   # fp8: MX e4m3
            if tp1:
                if l + 1 < L:
                    r, r_mx = ops.linear_residual(g, w.wdown, r, mx_next=self.layers[l + 1].wqkv)
                else:
                    r = ops.linear_residual(g, w.wdown, r)
            else:
                d = ops.linear(g, w.wdown)
                self.tp.all_reduce_(d, residual=r)     # d = r + MLP branch
                r = d
        return r

    # ------------------------------------------------------------------ prefill all-reduce overlap
    # Chunks shorter than this many tokens are not split (``K8S_PREFILL_OVERLAP_MIN``).  Splitting costs a second,
    # half-size pass over every weight: measured at one TP = 8 rank's shapes (profiles/prefill_split_cost_tp8sim.jsonl)
    # +112 us per layer at 256 tokens, +172 at 2048, +28 at 8192, while the two all-reduces it hides grow with the
    # chunk (2 x 4 MiB two-shot xGMI at 256 tokens: well under the cost; 2 x 32 MiB RCCL at 2048: several times it).
    _comm_stream: Optional[torch.cuda.Stream] = None

    @property
    def prefill_overlap_min(self) -> int:
        return int(os.environ.get("K8S_PREFILL_OVERLAP_MIN", "2048"))

    @property
    def prefill_overlap(self) -> bool:
        """TP > 1 prefill runs as two token halves whose all-reduces overlap the other half's GEMMs
        (``K8S_PREFILL_OVERLAP=0`` turns it off; ``=cpu`` also splits on CPU, for the gloo tests; ``=sim`` also
        splits a simulated TP rank, whose skipped collectives leave the split's own cost: tools/overlap_probe.py)."""
        env = os.environ.get("K8S_PREFILL_OVERLAP", "1")
        if self.tp.world <= 1 or env == "0" or not self.norm_folded or (self.tp.simulate and env != "sim"):
            return False
        return self.device.type == "cuda" or env == "cpu"

    def _layers_folded_overlap(self, h: torch.Tensor, attn, T0: int) -> torch.Tensor:
        """``_layers_folded`` for TP > 1 prefill as two micro-batches (tokens [0, T0) and [T0, T)) on one
        compute stream, with every all-reduce on a comm stream.  Per layer the compute stream issues
        [QKV, attention, O] of half 0, then of half 1, then [gate/up, down] of half 0, then of half 1; each
        branch's all-reduce (residual fused, as in ``_layers_folded``) waits only for its own O / down GEMM, so

            AR(O0)    runs under  QKV1 + attention1 + O1
            AR(O1)    runs under  gate/up0 + down0
            AR(down0) runs under  gate/up1 + down1
            AR(down1) runs under  QKV0 + attention0 + O0 of the next layer.

        Half 1's attention reads the K/V half 0 wrote at the same layer (the compute stream orders them).
        The collectives stay in one fixed order on one stream (every rank issues the same sequence, as one
        communicator needs); nothing is allocated on the comm stream, and a tensor the comm stream touches
        is released only after the compute stream has waited for that collective, so the caching allocator
        cannot hand its memory to a later kernel early.  Captures into the prefill hipGraphs as a fork/join.
        (SURVEY 2.6 P-COMM / north star "all-reduce overlapped with GEMMs".)"""
        eps = self.cfg.rms_eps
        gpu = h.is_cuda
        if gpu:
            cs = torch.cuda.current_stream(self.device)
            if self._comm_stream is None:
                self._comm_stream = torch.cuda.Stream(self.device)
            ms = self._comm_stream

        def all_reduce(t: torch.Tensor, res: torch.Tensor):
            if not gpu:
                self.tp.all_reduce_(t, residual=res)
                return None
            ms.wait_stream(cs)
            with torch.cuda.stream(ms):
                self.tp.all_reduce_(t, residual=res)
            ev = torch.cuda.Event()
            ev.record(ms)
            return ev

        def wait(ev) -> None:
            if ev is not None:
                cs.wait_event(ev)

        r = [h[:T0].clone(), h[T0:].clone()]
        o: List[Optional[torch.Tensor]] = [None, None]
        pend: list = [None, None]          # event after which r[i] holds the layer's output on the comm stream
        for l, w in enumerate(self.layers):
            ev_o = [None, None]
            for i in (0, 1):
                wait(pend[i])
                o[i] = None                # the previous layer's o[i] was the residual of AR(down_i): released now
                qkv = ops.linear_rms(r[i], w.wqkv, eps)
                a = attn(l, qkv, i)
                o[i] = ops.linear(a, w.wo)
                ev_o[i] = all_reduce(o[i], r[i])     # o_i = r_i + attention branch
            for i in (0, 1):
                wait(ev_o[i])
                g = ops.linear_rms(o[i], w.wgu, eps, ops.EPI_SWIGLU)
                d = ops.linear(g, w.wdown)
                pend[i] = all_reduce(d, o[i])        # d_i = o_i + MLP branch
                r[i] = d                   # the old r[i] was read by AR(O_i), which the wait above covered
        wait(pend[0])
        wait(pend[1])
        return torch.cat(r)

    # ------------------------------------------------------------------ sequence parallelism (prefill)
    @property
    def seq_parallel_min(self) -> int:
        return int(os.environ.get("K8S_SEQ_PARALLEL_MIN", "2048"))

    def seq_parallel_at(self, T: int) -> bool:
        """TP > 1 prefill chunks of at least ``K8S_SEQ_PARALLEL_MIN`` tokens run sequence-parallel when
        ``K8S_SEQ_PARALLEL=1`` (``=sim`` also on a simulated TP rank, for profiling the shapes)."""
        env = os.environ.get("K8S_SEQ_PARALLEL", "0")
        if self.tp.world <= 1 or env == "0" or not self.norm_folded or (self.tp.simulate and env != "sim"):
            return False
        return T >= self.seq_parallel_min

    def _layers_folded_sp(self, h: torch.Tensor, attn) -> torch.Tensor:
        """``_layers_folded`` with Megatron sequence parallelism (SURVEY 2.6 P-SP): the residual stream lives as
        row shards, rank k holding rows [k n, (k + 1) n) of the chunk (n = ceil(T / tp)); every all-reduce becomes
        a reduce-scatter (residual added on the shard) and the next pre-norm projection's input an all-gather of
        the un-normalised shards (the RMS statistics are the GEMM prologue, as without SP).  The same bytes cross
        xGMI as with the all-reduce; what changes is that residual adds and the residual stream itself are 1/tp
        per rank, and the two halves of each collective are separate operations (docs/ARCHITECTURE.md, "TP = 8
        prefill communication").  Chunks whose length does not divide by tp carry zero rows at the end, which
        stay zero through every layer (zero input rows give zero RMS-scaled outputs)."""
        eps = self.cfg.rms_eps
        W, rk = self.tp.world, self.tp.rank
        T, H = h.shape
        n = -(-T // W)
        pad = n * W - T
        if pad:
            h = torch.cat([h, h.new_zeros(pad, H)])
        r = h[rk * n:(rk + 1) * n].clone()
        for l, w in enumerate(self.layers):
            x = self.tp.all_gather_rows(r)                          # [n W, H] residual stream, un-normalised
            qkv = ops.linear_rms(x[:T] if pad else x, w.wqkv, eps)
            a = attn(l, qkv)
            if pad:
                a = torch.cat([a, a.new_zeros(pad, a.shape[1])])
            r = self.tp.reduce_scatter_rows(ops.linear(a, w.wo), residual=r)      # r + attention branch
            x = self.tp.all_gather_rows(r)
            g = ops.linear_rms(x, w.wgu, eps, ops.EPI_SWIGLU)
            r = self.tp.reduce_scatter_rows(ops.linear(g, w.wdown), residual=r)   # r + MLP branch
        return self.tp.all_gather_rows(r)[:T]

    # True: forward_* return the logits all-gathered over the TP ranks ([tp, S, Vs], shard-major).  False (the
    # engine at TP > 1): this rank's vocab shard only ([1, S, Vs]), sampled vocab-parallel (ops.sample(tp=...)): a
    # decode step then moves a few bytes per row between the ranks instead of rows x vocab x 4 B.
    gather_logits = True

    def _gather(self, logits: torch.Tensor) -> torch.Tensor:
        if self.gather_logits or self.tp.world == 1:
            return self.tp.all_gather_shards(logits)                           # [tp, S, Vs]
        return logits.unsqueeze(0)                                             # [1, S, Vs]: this rank's shard

    def _logits_folded(self, r: torch.Tensor) -> torch.Tensor:
        logits = ops.linear_rms(r, self.lm_head, self.cfg.rms_eps, ops.EPI_F32)   # final norm folded: [S, Vs]
        return self._gather(logits)

    def _layers(self, h: torch.Tensor, attn) -> tuple:
        """Run all decoder layers.  ``attn(l, qkv) -> [T, nq*D]`` does rope + KV write + attention."""
        c = self.cfg
        res = h.clone()
        x = ops.rmsnorm(h, self.layers[0].ln1, c.rms_eps)
        for l, w in enumerate(self.layers):
            if l > 0:
                x = ops.rmsnorm(h, w.ln1, c.rms_eps, residual=res)
            qkv = ops.linear(x, w.wqkv)
            a = attn(l, qkv)
            o = ops.linear(a, w.wo)
            self.tp.all_reduce_(o)
            x = ops.rmsnorm(o, w.ln2, c.rms_eps, residual=res)
            g = ops.linear_swiglu(x, w.wgu)
            h = ops.linear(g, w.wdown)
            self.tp.all_reduce_(h)
        return h, res

    def _logits(self, h: torch.Tensor, res: torch.Tensor) -> torch.Tensor:
        x = ops.rmsnorm(h, self.norm, self.cfg.rms_eps, residual=res)
        logits = ops.linear(x, self.lm_head, out_dtype=torch.float32)   # [S, Vs]
        return self._gather(logits)

    def forward_prefill(self, ids: torch.Tensor, positions: torch.Tensor, slot_mapping: torch.Tensor,
                        cu_q: torch.Tensor, context_lens: torch.Tensor, block_tables: torch.Tensor,
                        max_qlen: int, last_idx: torch.Tensor, split: Optional[tuple] = None) -> torch.Tensor:
        """Varlen prefill (chunks of several sequences).  Returns gathered logits [tp, S, Vs] for
        the token at ``last_idx`` of each sequence.

        ``split`` = ``(T0, half0, half1)`` with ``half = (cu_q, context_lens, block_tables, max_qlen)`` of the
        tokens [0, T0) / [T0, T) (``split_prefill_meta``): TP > 1 runs the two halves as micro-batches whose
        all-reduces overlap the other half's GEMMs (``_layers_folded_overlap``)."""
        T = ids.shape[0]
        kv = self.kv_cache
        self.tp.phase = "prefill"

        def attn(l: int, qkv: torch.Tensor) -> torch.Tensor:
            q = ops.rope_kv_write(qkv, self.cos_sin, kv[l, 0], kv[l, 1], self.nq, self.nkv, self.D,
                                  positions=positions, slot_mapping=slot_mapping)
            a = ops.paged_prefill_attention(q, kv[l, 0], kv[l, 1], cu_q, context_lens, block_tables,
                                            self.scale, self.block_size, max_qlen)
            return a.view(T, self.nq * self.D)

        li = last_idx.long()
        if self.seq_parallel_at(T):
            r = self._layers_folded_sp(ops.embedding(ids, self.embed), attn)
            return self._logits_folded(r.index_select(0, li).contiguous())
        if split is not None and self.prefill_overlap:
            T0 = split[0]
            pieces = ((slice(0, T0), split[1]), (slice(T0, T), split[2]))

            def attn_half(l: int, qkv: torch.Tensor, i: int) -> torch.Tensor:
                sl, (cu, ctx, bt, mq) = pieces[i]
                n = qkv.shape[0]
                q = ops.rope_kv_write(qkv, self.cos_sin, kv[l, 0], kv[l, 1], self.nq, self.nkv, self.D,
                                      positions=positions[sl], slot_mapping=slot_mapping[sl])
                a = ops.paged_prefill_attention(q, kv[l, 0], kv[l, 1], cu, ctx, bt, self.scale, self.block_size,
                                                max(1, mq))
                return a.view(n, self.nq * self.D)

            r = self._layers_folded_overlap(ops.embedding(ids, self.embed), attn_half, T0)
            return self._logits_folded(r.index_select(0, li).contiguous())
        if self.norm_folded:
            r = self._layers_folded(ops.embedding(ids, self.embed), attn)
            return self._logits_folded(r.index_select(0, li).contiguous())
        h, res = self._layers(ops.embedding(ids, self.embed), attn)
        return self._logits(h.index_select(0, li).contiguous(), res.index_select(0, li).contiguous())

    def forward_decode(self, tokens: torch.Tensor, context_lens: torch.Tensor, block_tables: torch.Tensor,
                       max_context: int, cascade=None) -> torch.Tensor:
        """One decode step for B sequences (one token each, positions from context_lens).  ``cascade`` = (cas, ngm):
        the rows' shared prefix is attended once for the batch (ops.decode_attention_fused)."""
        B = tokens.shape[0]
        self.tp.phase = "decode"
        if self.device.type == "cuda" and B <= ops.GEMV_MAX_M and self.fused_decode:
            return self._forward_decode_fused(tokens, context_lens, block_tables, max_context, cascade)
        kv = self.kv_cache
        fused_attn = self.device.type == "cuda" and self.fused_decode   # batched decode (B > 8)
        # fp8 GEMM rows: the attention kernel writes the O projection's input as MX e4m3 (K16)
        mx = fused_attn and ops.mx_rows(B, self.layers[0].wo)

        def attn(l: int, qkv: torch.Tensor):
            if fused_attn:
                return ops.decode_attention_fused(qkv, self.cos_sin, kv[l, 0], kv[l, 1], block_tables, context_lens,
                                                  self.scale, self.block_size, max_context, self.nq, self.nkv, self.D,
                                                  mx=mx, cascade=cascade)
            q = ops.rope_kv_write(qkv, self.cos_sin, kv[l, 0], kv[l, 1], self.nq, self.nkv, self.D,
                                  context_lens=context_lens, block_tables=block_tables, block_size=self.block_size)
            a = ops.paged_decode_attention(q, kv[l, 0], kv[l, 1], block_tables, context_lens, self.scale,
                                           self.block_size, max_context)
            return a.view(B, self.nq * self.D)

        if self.norm_folded:
            mx0 = (self.tp.world == 1 or self.tp.simulate) and ops.mx_rows(B, self.layers[0].wqkv)
            return self._logits_folded(self._layers_folded(ops.embedding(tokens, self.embed, mx=mx0), attn))
        h, res = self._layers(ops.embedding(tokens, self.embed), attn)
        return self._logits(h, res)


    fused_decode = True

    # ------------------------------------------------------------------ decode weight prefetch (opt-in experiment)
    # K8S_DECODE_PREFETCH_MB = M > 0: after each layer's QKV GEMV a side stream reads the first M MB of that layer's
    # O and gate/up weights into the Infinity Cache while attention (latency-bound, a few CUs) runs on the main stream;
    # the branch joins at the end of the step (captured into the decode graphs as a fork / join).
    _pf_stream: Optional[torch.cuda.Stream] = None

    @property
    def prefetch_bytes(self) -> int:
        return int(float(os.environ.get("K8S_DECODE_PREFETCH_MB", "0")) * (1 << 20))

    def _pf_layer(self, w: LayerWeights, budget: int) -> None:
        cs = torch.cuda.current_stream(self.device)
        if self._pf_stream is None:
            self._pf_stream = torch.cuda.Stream(self.device)
        ps = self._pf_stream
        ps.wait_stream(cs)
        with torch.cuda.stream(ps):
            for t in (w.wo, w.wgu):
                if budget <= 0:
                    break
                q = t.q if isinstance(t, ops.Fp8Weight) else t
                n = min(budget, q.numel() * q.element_size())
                ops.prefetch(t, n)
                budget -= n

    def _pf_join(self) -> None:
        if self._pf_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._pf_stream)

    def _forward_decode_fused(self, tokens: torch.Tensor, context_lens: torch.Tensor, block_tables: torch.Tensor,
                              max_context: int, cascade=None) -> torch.Tensor:
        """Decode step with 5 kernels per layer: [norm+QKV GEMV] -> [RoPE+KV write+attention] ->
        [O GEMV] -> all-reduce -> [norm+gate/up GEMV+SwiGLU] -> [down GEMV] -> all-reduce.
        The residual stream ping-pongs between two buffers (a norm-GEMV reads one, writes the other)."""
        c, kv = self.cfg, self.kv_cache
        h = ops.embedding(tokens, self.embed)
        if self.tp.world > 1:
            return self._forward_decode_fused_tp(h, context_lens, block_tables, max_context, cascade)
        res_a = torch.empty_like(h)
        res_b = torch.empty_like(h)
        res_in = None
        pf = self.prefetch_bytes
        for w_l, w in enumerate(self.layers):
            qkv = ops.linear_norm(h, w.wqkv, None if self.norm_folded else w.ln1, c.rms_eps, res_in, res_b)
            if pf:
                self._pf_layer(w, pf)
            a = ops.decode_attention_fused(qkv, self.cos_sin, kv[w_l, 0], kv[w_l, 1], block_tables, context_lens,
                                           self.scale, self.block_size, max_context, self.nq, self.nkv, self.D,
                                           cascade=cascade)
            o = ops.linear(a, w.wo)
            self.tp.all_reduce_(o)
            g = ops.linear_norm(o, w.wgu, None if self.norm_folded else w.ln2, c.rms_eps, res_b, res_a,
                                epi=ops.EPI_SWIGLU)
            h = ops.linear(g, w.wdown)
            self.tp.all_reduce_(h)
            res_in = res_a
        if pf:
            self._pf_join()
        logits = ops.linear_norm(h, self.lm_head, None if self.norm_folded else self.norm, c.rms_eps, res_in, None,
                                 epi=ops.EPI_F32)
        return self._gather(logits)

    def _forward_decode_fused_tp(self, h: torch.Tensor, context_lens: torch.Tensor, block_tables: torch.Tensor,
                                 max_context: int, cascade=None) -> torch.Tensor:
        """TP > 1 decode: the residual add rides on the all-reduce (xGMI kernels add it before their
        single rounding: SURVEY K14 + K2), so the residual stream IS the all-reduce outputs and the
        norm-GEMV prologues read one tensor (no residual read, no residual write)."""
        c, kv = self.cfg, self.kv_cache
        B = h.shape[0]
        g1 = None if self.norm_folded else (lambda w: w.ln1)
        g2 = None if self.norm_folded else (lambda w: w.ln2)
        x = h
        pf = self.prefetch_bytes
        for l, w in enumerate(self.layers):
            qkv = ops.linear_norm(x, w.wqkv, g1(w) if g1 else None, c.rms_eps, None, None)
            if pf:
                self._pf_layer(w, pf)
            a = ops.decode_attention_fused(qkv, self.cos_sin, kv[l, 0], kv[l, 1], block_tables, context_lens,
                                           self.scale, self.block_size, max_context, self.nq, self.nkv, self.D,
                                           cascade=cascade)
            o = self.tp.linear_all_reduce(a, w.wo, residual=x)   # o = x + attention branch (AR in the GEMV)
            g = ops.linear_norm(o, w.wgu, g2(w) if g2 else None, c.rms_eps, None, None, epi=ops.EPI_SWIGLU)
            x = self.tp.linear_all_reduce(g, w.wdown, residual=o)    # x = o + MLP branch
        if pf:
            self._pf_join()
        logits = ops.linear_norm(x, self.lm_head, None if self.norm_folded else self.norm, c.rms_eps, None, None,
                                 epi=ops.EPI_F32)
        return self._gather(logits)



def save_hf_checkpoint(model: LlamaModel, path: Path) -> None:
    """Write a TP=1 model as a HuggingFace-layout safetensors checkpoint (tests/tools)."""
    from safetensors.torch import save_file

    assert model.tp.world == 1 and model.weight_dtype == "bf16"
    c, D = model.cfg, model.D
    t: Dict[str, torch.Tensor] = {"model.embed_tokens.weight": model.embed, "model.norm.weight": model.norm,
                                  "lm_head.weight": model.lm_head}
    for l, w in enumerate(model.layers):
        p = f"model.layers.{l}."
        q_rows, kv_rows = c.num_heads * D, c.num_kv_heads * D
        t[p + "self_attn.q_proj.weight"] = w.wqkv[:q_rows]
        t[p + "self_attn.k_proj.weight"] = w.wqkv[q_rows:q_rows + kv_rows]
        t[p + "self_attn.v_proj.weight"] = w.wqkv[q_rows + kv_rows:]
        t[p + "self_attn.o_proj.weight"] = w.wo
        t[p + "mlp.gate_proj.weight"] = w.wgu[:c.intermediate]
        t[p + "mlp.up_proj.weight"] = w.wgu[c.intermediate:]
        t[p + "mlp.down_proj.weight"] = w.wdown
        t[p + "input_layernorm.weight"] = w.ln1
        t[p + "post_attention_layernorm.weight"] = w.ln2
    path.mkdir(parents=True, exist_ok=True)
    save_file({k: v.detach().cpu().clone().contiguous() for k, v in t.items()}, str(path / "model.safetensors"))
    (path / "config.json").write_text(json.dumps({
        "hidden_size": c.hidden, "num_attention_heads": c.num_heads, "num_key_value_heads": c.num_kv_heads,
        "head_dim": c.head_dim, "intermediate_size": c.intermediate, "vocab_size": c.vocab,
        "num_hidden_layers": c.num_layers, "rms_norm_eps": c.rms_eps, "rope_theta": c.rope_theta,
        "rope_scaling": c.rope_scaling, "max_position_embeddings": c.max_position, "bos_token_id": c.bos_id,
        "eos_token_id": list(c.eos_ids)}))
