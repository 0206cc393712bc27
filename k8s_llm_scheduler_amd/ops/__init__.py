"""Device ops: gfx950 HIP kernels (``_C``) behind shape-checked wrappers.

Dispatch rule: CUDA (= HIP) tensors ALWAYS run the hand-written kernels; if the extension is
missing on a GPU the call raises (no silent PyTorch fallback).  CPU tensors run the fp32
reference in :mod:`.reference` -- that path exists for the CPU test-suite (gloo multi-process
tensor-parallel tests) and is the numerics oracle of the kernel tests.
"""

from __future__ import annotations

import functools
import importlib
import math
import os
from typing import Dict, Optional, Tuple

import torch

from . import reference as ref

_C = None
_C_ERR: Optional[BaseException] = None
# K8S_CHECKED=1 loads the bounds-checked build (python -m k8s_llm_scheduler_amd._build --checked): kernels range-check
# every index they derive from data and record violations, which the engine raises after each step (check_raise)
CHECKED = os.environ.get("K8S_CHECKED", "0") == "1"
try:  # torch must be imported first: the extension binds to torch's HIP runtime
    _C = importlib.import_module("k8s_llm_scheduler_amd.ops._C_checked" if CHECKED else "k8s_llm_scheduler_amd.ops._C")
except Exception as e:  # pragma: no cover - reported loudly on first GPU use
    _C_ERR = e

EPI_BF16, EPI_F32, EPI_SWIGLU = 0, 1, 2
BF16, F32, I32 = torch.bfloat16, torch.float32, torch.int32
DECODE_PARTITION = 64
FUSED_PARTITION = 1024
SPLIT_PARTITION = 64
# Decode attention with at most this many (sequence, kv head) pairs uses the small-grid kernel
# (attn_decode_split.hip: one wave per 64-token chunk, in-kernel merge); more pairs fill the chip
# with the one-workgroup-per-pair kernel (attn_decode_fused.hip).  Measured crossover at ctx 564
# (profiles/kbench_attn_split_vs_onewg.txt): split 11.7 vs 14.9 us at 32 pairs, 17.4 vs 14.9 at 64; in the
# 4096-token graph class the split grid is 4x larger and the crossover halves.  K8S_ATTN_SPLIT_PAIRS overrides.
SPLIT_MAX_PAIRS = int(os.environ.get("K8S_ATTN_SPLIT_PAIRS", "32"))


def _split_pairs_limit(max_context: int) -> int:
    return SPLIT_MAX_PAIRS if max_context <= 1024 else SPLIT_MAX_PAIRS // 2


def native():
    """The loaded extension module; raises with the build hint if it is missing."""
    if _C is None:
        raise RuntimeError("k8s_llm_scheduler_amd native extension (_C) is not built/loadable: "
                           f"{_C_ERR!r}. Run: python -m k8s_llm_scheduler_amd._build")
    return _C


def available() -> bool:
    return _C is not None


# ----------------------------------------------------------------------------- checked builds
class KernelCheckError(RuntimeError):
    """A checked kernel saw an index derived from data outside its bounds (csrc/kernels/common.h K8S_CHECKED)."""


CHECK_CODES = {1: "KV slot", 2: "KV block id", 3: "context length beyond the block table", 4: "token id"}
CHECK_UNITS = {1: "misc.hip (embedding)", 2: "rope_kv.hip", 3: "attn_decode_fused.hip", 4: "attn_decode_split.hip",
               5: "attn_prefill.hip", 6: "attn_decode.hip"}
_CHECK_REC: Dict[int, torch.Tensor] = {}


def check_enable(device, kv_slots: int, num_blocks: int, vocab: int) -> bool:
    """Checked builds: point every instrumented kernel unit at a fresh device record with these bounds (the model
    calls this when it allocates its KV cache).  False in release builds."""
    if _C is None or not getattr(_C, "checked", False):
        return False
    dev = torch.device(device)
    rec = torch.zeros(6, dtype=torch.int64, device=dev)   # K8sCheck: count/code/line/unit, value, 3 bounds
    rec[3], rec[4], rec[5] = int(kv_slots), int(num_blocks), int(vocab)
    with torch.cuda.device(dev):
        if _C.check_bind(rec.data_ptr()) != 0:
            raise RuntimeError("check_bind failed: the checked extension could not bind its device record")
    _CHECK_REC[dev.index if dev.index is not None else torch.cuda.current_device()] = rec
    return True


def check_read(device) -> Optional[dict]:
    """The first recorded violation since the last read (and the count), or None; resets the record.  Waits for the
    device work enqueued so far (call it after a step's results were fetched)."""
    dev = torch.device(device)
    rec = _CHECK_REC.get(dev.index if dev.index is not None else torch.cuda.current_device())
    if rec is None:
        return None
    words = rec[:3].cpu()
    head = words[:2].view(torch.int32)   # count, code, line, unit
    count = int(head[0])
    if count == 0:
        return None
    out = {"count": count, "code": int(head[1]), "line": int(head[2]), "unit": int(head[3]), "value": int(words[2]),
           "what": CHECK_CODES.get(int(head[1]), "?"), "where": CHECK_UNITS.get(int(head[3]), "?")}
    rec[:3].zero_()
    return out


def check_raise(device) -> None:
    """Raise KernelCheckError if a checked kernel recorded a violation (no-op in release builds)."""
    if not CHECKED:
        return
    v = check_read(device)
    if v is not None:
        raise KernelCheckError(f"{v['count']} bounds violation(s); first: {v['what']} = {v['value']} out of range in "
                               f"{v['where']} line {v['line']} (the index was clamped, nothing was written out of "
                               f"bounds)")


class Fp8Weight:
    """Row-scaled OCP e4m3 weight (fp8.hip): ``q`` [N, K] uint8 bit patterns, ``scale`` [N] fp32,
    w ~= e4m3(q) * scale[:, None].  Decode GEMVs stream ``q`` directly (half the HBM bytes of
    bf16); prefill GEMMs quantize the activations per token and run the row-scaled fp8 GEMM."""

    __slots__ = ("q", "scale")

    def __init__(self, q: torch.Tensor, scale: torch.Tensor):
        if q.dtype != torch.uint8 or q.dim() != 2 or scale.shape != (q.shape[0],) or scale.dtype != F32:
            raise ValueError("Fp8Weight needs q [N, K] uint8 and scale [N] fp32")
        self.q, self.scale = q.contiguous(), scale.contiguous()

    @property
    def shape(self):
        return self.q.shape

    @property
    def device(self):
        return self.q.device

    @property
    def is_cuda(self) -> bool:
        return self.q.is_cuda

    def numel(self) -> int:
        return self.q.numel()

    def nbytes(self) -> int:
        return self.q.numel() + self.scale.numel() * 4

    def __getitem__(self, rows) -> "Fp8Weight":
        return Fp8Weight(self.q[rows], self.scale[rows])

    def dequant(self, dtype=torch.bfloat16) -> torch.Tensor:
        if not self.is_cuda:
            return ref.dequant_fp8(self.q, self.scale, dtype)
        N, K = self.q.shape
        out = torch.empty(N, K, dtype=BF16, device=self.q.device)
        native().dequant_fp8_rows(out.data_ptr(), self.q.data_ptr(), self.scale.data_ptr(), N, K, -1)
        return out if dtype == BF16 else out.to(dtype)


def quantize_fp8(w: torch.Tensor) -> Fp8Weight:
    """bf16 [N, K] -> row-scaled fp8 (K % 16 == 0)."""
    if not w.is_cuda:
        q, s = ref.quantize_fp8(w)
        return Fp8Weight(q, s)
    N, K = w.shape
    q = torch.empty(N, K, dtype=torch.uint8, device=w.device)
    s = torch.empty(N, dtype=F32, device=w.device)
    native().quantize_fp8_rows(q.data_ptr(), s.data_ptr(), _chk(w, BF16, "w"), N, K, -1)
    return Fp8Weight(q, s)


def quantize_act_fp8(x: torch.Tensor, rms_eps: Optional[float] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-token (row) activation quantization: bf16 [T, K] -> (e4m3 bytes [T, K], scale [T] f32).
    ``rms_eps``: quantize RMSNorm(x) (gamma folded into the weights) -- the same e4m3 bytes as x's, with each row's
    1/rms folded into its scale (fp8.hip quantize_act_fp8_kernel): the pre-norm fp8 projections run no rmsnorm."""
    if not x.is_cuda:
        q, sc = ref.quantize_fp8(x)
        if rms_eps is not None:
            sc = sc * torch.rsqrt(x.float().pow(2).mean(-1) + rms_eps)
        return q, sc
    T, K = x.shape
    q = torch.empty(T, K, dtype=torch.uint8, device=x.device)
    s = torch.empty(T, dtype=F32, device=x.device)
    native().quantize_act_fp8_rms(q.data_ptr(), s.data_ptr(), _chk(x, BF16, "x"), T, K,
                                  1 if rms_eps is not None else 0, float(rms_eps or 0.0), -1)
    return q, s


class MxAct:
    """OCP MX e4m3 activations (K16 block-scaled; fp8.hip): ``q`` [M, K] uint8 e4m3 bit patterns, ``e`` the uint8
    E8M0 exponents in the kernels' layout [K / 128, M, 4] (common.h mx_scale_off: a k-tile's scales of consecutive
    rows are adjacent); :meth:`blocks` gives them as [M, K / 32], x[m, k] ~= e4m3(q[m, k]) * 2^(blocks[m, k // 32] -
    127).  The O and down projections of the fp8
    GEMM rows take their input in this form: the SwiGLU epilogue (mgemm / pgemm ``mx_out``) and the attention
    output write it, and the GEMMs feed the E8M0 bytes to the block-scaled MFMA's scale operand (mgemm / pgemm MX
    mode) -- no per-token absmax pass, no quantize launch between a producer and its consumer."""

    __slots__ = ("q", "e")

    def __init__(self, q: torch.Tensor, e: torch.Tensor):
        if (q.dtype != torch.uint8 or e.dtype != torch.uint8 or q.dim() != 2 or q.shape[1] % 128
                or e.shape != (q.shape[1] // 128, q.shape[0], 4)):
            raise ValueError("MxAct needs q [M, K] uint8 (K % 128 == 0) and e [K / 128, M, 4] uint8")
        self.q, self.e = q, e

    @staticmethod
    def empty(M: int, K: int, device) -> "MxAct":
        return MxAct(torch.empty(M, K, dtype=torch.uint8, device=device),
                     torch.empty(K // 128, M, 4, dtype=torch.uint8, device=device))

    def blocks(self) -> torch.Tensor:
        """The E8M0 scales as [M, K / 32]."""
        return ref.mx_scales_from_device_layout(self.e)

    @property
    def shape(self):
        return self.q.shape

    @property
    def device(self):
        return self.q.device

    @property
    def is_cuda(self) -> bool:
        return self.q.is_cuda

    def dequant(self, dtype=BF16) -> torch.Tensor:
        return ref.dequant_mx(self.q, self.e, torch.float32).to(dtype)


# K8S_MX=0: the fp8 O / down GEMM rows take per-token e4m3 activations (a quantize_act_fp8 launch each) instead of
# the MX form their producers write.  MX is used where the consuming GEMM is mgemm (batched decode, short chunks):
# measured there 1.1-1.5x faster than quantize + per-token GEMM (profiles/mgemm_mx_tune_r5.txt; fp8 batch-64 decode
# 20.0 -> 19.6 ms/step, one TP = 4 rank's shapes 8.40 -> 8.17).  pgemm's MX mode is correct but ~10 % slower than its
# per-token mode at prefill sizes (the MFMA-bound regime; profiles/mx_pgemm_bench_r5.txt), more than the quantize
# launch it saves, so prefill-size consumers stay per-token unless K8S_MX_PGEMM=1.
MX_ON = os.environ.get("K8S_MX", "1") != "0"
MX_PGEMM = os.environ.get("K8S_MX_PGEMM", "0") == "1"


def quantize_act_mx(x: torch.Tensor) -> MxAct:
    """bf16 [M, K] -> MxAct (stand-alone form of what the fused producers write; K % 128 == 0)."""
    if not x.is_cuda:
        q, e = ref.quantize_mx(x)
        return MxAct(q, ref.mx_scales_to_device_layout(e))
    M, K = x.shape
    a = MxAct.empty(M, K, x.device)
    native().quantize_act_mx(a.q.data_ptr(), a.e.data_ptr(), _chk(x, BF16, "x"), M, K, -1)
    return a


def _fp8_gemm(x: torch.Tensor, w: "Fp8Weight", out_dtype=None, act=None) -> torch.Tensor:
    """K8S_GEMM=library only (the A/B oracle): per-token e4m3 activations (``act`` = (q, scale) when already
    quantized) x row-scaled e4m3 weights on hipBLASLt's row-wise scaled fp8 GEMM (torch._scaled_mm), bf16 out."""
    xq, sx = act if act is not None else quantize_act_fp8(x.contiguous())
    f8 = torch.float8_e4m3fn
    return torch._scaled_mm(xq.view(f8), w.q.view(f8).t(), scale_a=sx.view(-1, 1), scale_b=w.scale.view(1, -1),
                            out_dtype=out_dtype or BF16)


def _ref_act_quant(x: torch.Tensor, w) -> torch.Tensor:
    """CPU oracle of the GPU dispatch: with fp8 weights, more than GEMV_MAX_M rows go through
    per-token e4m3 activations (_fp8_gemm), so the reference rounds its activations the same way."""
    if not isinstance(w, Fp8Weight):
        return x
    x2 = x.reshape(-1, x.shape[-1])
    if x2.shape[0] <= max(GEMV_MAX_M, SGEMV_MAX_M):   # GEMV / sgemv: bf16 activations against the fp8 weights
        return x
    q, s = ref.quantize_fp8(x2)
    return ref.dequant_fp8(q, s, torch.float32).to(x.dtype).view(x.shape)


def _is_fp8(w) -> bool:
    return isinstance(w, Fp8Weight)


def _gpu(*ts: torch.Tensor) -> bool:
    cuda = [t.is_cuda for t in ts if t is not None]
    if any(cuda) and not all(cuda):
        raise ValueError("mixed CPU/GPU tensors")
    return bool(cuda) and cuda[0]


def _chk(t: torch.Tensor, dtype, name: str) -> int:
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    return t.data_ptr()




# ----------------------------------------------------------------------------- norms
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """RMSNorm; with ``residual`` the kernel first does residual += x (in place) and normalises
    the sum (fused add + norm)."""
    if not _gpu(x, w, residual):
        y, _ = ref.rmsnorm(x, w, eps, residual)
        if out is not None:
            out.copy_(y)
            return out
        return y
    H = x.shape[-1]
    rows = x.numel() // H
    out = torch.empty_like(x) if out is None else out
    native().rmsnorm(_chk(out, BF16, "out"), _chk(x, BF16, "x"),
                     _chk(residual, BF16, "residual") if residual is not None else 0,
                     _chk(w, BF16, "w"), rows, H, float(eps), -1)
    return out


# ----------------------------------------------------------------------------- rope + kv
def rope_kv_write(qkv: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                  nq: int, nkv: int, D: int, *, positions: Optional[torch.Tensor] = None,
                  slot_mapping: Optional[torch.Tensor] = None, context_lens: Optional[torch.Tensor] = None,
                  block_tables: Optional[torch.Tensor] = None, block_size: int = 16) -> torch.Tensor:
    """Rotate q/k, write k/v into the paged cache; returns rotated q [T, nq, D].
    Prefill mode: positions + slot_mapping.  Decode mode: context_lens + block_tables."""
    T = qkv.shape[0]
    if qkv.shape[-1] != (nq + 2 * nkv) * D:
        raise ValueError("qkv width mismatch")
    if not _gpu(qkv, k_cache):
        if positions is None:
            positions, slot_mapping = ref.decode_positions(context_lens, block_tables, block_size)
        return ref.rope_kv_write(qkv, cos_sin, positions, slot_mapping, k_cache, v_cache, nq, nkv, D).view(T, nq, D)
    q = torch.empty(T, nq, D, dtype=qkv.dtype, device=qkv.device)
    if positions is not None:
        p_pos, p_slot, p_ctx, p_bt, mb = _chk(positions, I32, "positions"), _chk(slot_mapping, I32, "slots"), 0, 0, 0
    else:
        p_pos = p_slot = 0
        p_ctx, p_bt, mb = _chk(context_lens, I32, "context_lens"), _chk(block_tables, I32, "block_tables"), \
            block_tables.shape[1]
    native().rope_kv_write(q.data_ptr(), _chk(k_cache, BF16, "k_cache"), _chk(v_cache, BF16, "v_cache"),
                           _chk(qkv, BF16, "qkv"), _chk(cos_sin, F32, "cos_sin"), p_pos, p_slot, p_ctx, p_bt,
                           mb, block_size, T, nq, nkv, D, -1)
    return q


# ----------------------------------------------------------------------------- attention
def paged_decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                           context_lens: torch.Tensor, scale: float, block_size: int, max_context: int) -> torch.Tensor:
    """q [B, nq, D]; returns [B, nq, D].  ``max_context`` bounds the partition grid (fixed for
    a captured graph)."""
    if not _gpu(q, k_cache):
        return ref.paged_decode_attention(q, k_cache, v_cache, block_tables, context_lens, scale, block_size)
    B, nq, D = q.shape
    nkv = k_cache.shape[-2]
    pmax = max(1, math.ceil(max_context / DECODE_PARTITION))
    out = torch.empty_like(q)
    if pmax > 1:
        pacc = torch.empty(B * nq * pmax * D, dtype=F32, device=q.device)
        pml = torch.empty(B * nq * pmax * 2, dtype=F32, device=q.device)
        pa, pm = pacc.data_ptr(), pml.data_ptr()
    else:
        pa = pm = 0
    native().paged_decode_attention(out.data_ptr(), pa, pm, _chk(q, BF16, "q"), _chk(k_cache, BF16, "k_cache"),
                                    _chk(v_cache, BF16, "v_cache"), _chk(block_tables, I32, "block_tables"),
                                    _chk(context_lens, I32, "context_lens"), float(scale), B, nq, nkv, D, block_size,
                                    block_tables.shape[1], DECODE_PARTITION, pmax, -1)
    return out


def paged_prefill_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, cu_q: torch.Tensor,
                            context_lens: torch.Tensor, block_tables: torch.Tensor, scale: float, block_size: int,
                            max_qlen: int) -> torch.Tensor:
    """q [T, nq, D] (varlen over sequences by cu_q); causal over the paged cache."""
    if not _gpu(q, k_cache):
        return ref.paged_prefill_attention(q, k_cache, v_cache, cu_q, context_lens, block_tables, scale, block_size)
    T, nq, D = q.shape
    nkv = k_cache.shape[-2]
    out = torch.empty_like(q)
    native().paged_prefill_attention(out.data_ptr(), _chk(q, BF16, "q"), _chk(k_cache, BF16, "k_cache"),
                                     _chk(v_cache, BF16, "v_cache"), _chk(cu_q, I32, "cu_q"),
                                     _chk(context_lens, I32, "context_lens"), _chk(block_tables, I32, "block_tables"),
                                     float(scale), context_lens.shape[0], int(max_qlen), nq, nkv, D, block_size,
                                     block_tables.shape[1], -1)
    return out


# ----------------------------------------------------------------------------- linear
GEMV_KERNEL_MAX_M = 8   # rows the GEMV kernels (gemv.hip) accept
# rows up to which linear() / the decode step take the GEMV; above it the MFMA GEMM (mgemm.hip) is faster
# (profiles/mgemm_small_m.txt: at 4 rows mgemm wins every 70B projection at TP = 1 and 8, bf16 and fp8;
# at 2 rows the GEMV still wins or ties)
GEMV_MAX_M = int(os.environ.get("K8S_GEMV_MAX_M", "2"))
if not 1 <= GEMV_MAX_M <= GEMV_KERNEL_MAX_M:
    raise ValueError(f"K8S_GEMV_MAX_M must be 1..{GEMV_KERNEL_MAX_M}")


# Small decode batches, GEMV_MAX_M < rows <= SGEMV_MAX_M: csrc/kernels/sgemv.hip (x in registers, every weight
# streamed once, the RMS statistics and the residual add / SwiGLU fused; 3..4 rows on v_dot2, 5..16 on the matrix
# cores).  K8S_SGEMV=0 sends them to mgemm instead.
SGEMV_KERNEL_MAX_M = 16
SGEMV_MAX_M = SGEMV_KERNEL_MAX_M if os.environ.get("K8S_SGEMV", "1") != "0" else 0


def _sgemv(x2: torch.Tensor, w, epi: int, res: Optional[torch.Tensor] = None, rms_eps: Optional[float] = None,
           out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """epi(x2 @ w.T) for GEMV_MAX_M < M <= SGEMV_MAX_M rows on sgemv.hip (``rms_eps``: scaled by 1/rms of each x row,
    the norm gamma folded into ``w``; ``res``: plus ``res``, written to ``out`` which may be ``res``).  None where
    sgemv does not take the call (the caller routes it to mgemm)."""
    M, K = x2.shape
    if not GEMV_MAX_M < M <= SGEMV_MAX_M:
        return None
    fp8 = _is_fp8(w)
    N = w.shape[0] // 2 if epi == EPI_SWIGLU else w.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=F32 if epi == EPI_F32 else BF16, device=x2.device)
    ws = native().sgemv_workspace(M, N, K, epi, int(fp8))
    part = torch.empty(ws, dtype=F32, device=x2.device) if ws > 0 else None
    rc = native().sgemv(out.data_ptr(), part.data_ptr() if part is not None else 0, _chk(x2, BF16, "x"),
                        w.q.data_ptr() if fp8 else _chk(w, BF16, "w"), w.scale.data_ptr() if fp8 else 0,
                        _chk(res, BF16, "res") if res is not None else 0, M, N, K, epi,
                        1 if rms_eps is not None else 0, float(rms_eps or 0.0), -1)
    del part
    return None if rc == -5 else out


def _gemv(x: torch.Tensor, w, epi: int, out_dtype, norm_w=None, eps: float = 0.0, res_in=None,
          res_out=None, folded: bool = False) -> torch.Tensor:
    """Decode GEMV (M <= 8) for bf16 or fp8 weights, optionally with the fused pre-norm prologue
    (``folded``: the norm weight is already multiplied into ``w``; only 1/rms is applied)."""
    M, K = x.shape
    N = w.shape[0] // 2 if epi == EPI_SWIGLU else w.shape[0]
    out = torch.empty(M, N, dtype=out_dtype, device=x.device)
    mode = 2 if folded else (1 if norm_w is not None else 0)
    ks, splits = native().gemv_plan(M, N, K, epi, mode)
    part = torch.empty(splits * M * w.shape[0], dtype=F32, device=x.device) if splits > 1 else None
    pp = part.data_ptr() if part is not None else 0
    ri = _chk(res_in, BF16, "res_in") if res_in is not None else 0
    ro = _chk(res_out, BF16, "res_out") if res_out is not None else 0
    nw = _chk(norm_w, BF16, "norm_w") if norm_w is not None else 0
    if folded:
        native().gemv_rms(out.data_ptr(), pp, _chk(x, BF16, "x"), w.q.data_ptr() if _is_fp8(w) else _chk(w, BF16, "w"),
                          w.scale.data_ptr() if _is_fp8(w) else 0, M, N, K, epi, ri, ro, float(eps), -1)
    elif _is_fp8(w):
        native().gemv_fp8(out.data_ptr(), pp, _chk(x, BF16, "x"), w.q.data_ptr(), w.scale.data_ptr(), M, N, K, epi,
                          ri, ro, nw, float(eps), -1)
    elif norm_w is not None:
        native().gemv_norm(out.data_ptr(), pp, _chk(x, BF16, "x"), _chk(w, BF16, "w"), M, N, K, epi, ri, ro, nw,
                           float(eps), -1)
    else:
        native().gemv(out.data_ptr(), pp, _chk(x, BF16, "x"), _chk(w, BF16, "w"), M, N, K, epi, -1)
    del part
    return out




def prefetch(w, nbytes: Optional[int] = None, blocks: int = 256) -> None:
    """Read the first ``nbytes`` of weight ``w`` (bf16 tensor or Fp8Weight) with default-policy loads on the current
    stream, so they sit in the Infinity Cache when the GEMV that streams them runs (misc.hip prefetch_kernel)."""
    t = w.q if _is_fp8(w) else w
    n = t.numel() * t.element_size() if nbytes is None else min(int(nbytes), t.numel() * t.element_size())
    sink = _zeroed_scratch(t.device, "prefetch_sink", 4096)
    native().prefetch(t.data_ptr(), n & ~15, blocks, sink, -1)


def gemv_allreduce(comm, x: torch.Tensor, w, residual: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """residual + sum over TP ranks of x @ w.T in one kernel (gemv.hip GemvAr: the all-reduce rides in the GEMV
    epilogue over the xGMI peer regions of ``comm``, a native XgmiComm).  None where the shape does not fit the fused
    plan (nothing was launched: the caller runs GEMV + all-reduce)."""
    M, K = x.shape
    N = w.shape[0]
    if residual is not None and (residual.dtype != BF16 or tuple(residual.shape) != (M, N)):
        raise ValueError("residual must be a bf16 [M, N] tensor")
    out = torch.empty(M, N, dtype=BF16, device=x.device)
    fp8 = _is_fp8(w)
    rc = comm.gemv_allreduce(out.data_ptr(), _chk(x, BF16, "x"), w.q.data_ptr() if fp8 else _chk(w, BF16, "w"),
                             w.scale.data_ptr() if fp8 else 0, M, N, K,
                             _chk(residual, BF16, "residual") if residual is not None else 0, -1)
    return out if rc == 0 else None


# Row counts of the library GEMMs in the tuned table (engine/assets/tunableop_gfx950.csv, written by
# tools/tune_gemms.py): the engine's batched-decode buckets and the prefill buckets.  With the table
# loaded, a library GEMM of M rows in (8, 1024] is padded to the next bucket so that it runs the
# solution measured for that bucket instead of the library heuristic's pick for an odd M (TP=1,
# 256 prompt rows: down 315 -> 177 us, QKV 80 -> 64 us; tools/prefill_gemm_probe.py).
GEMM_M_BUCKETS = (16, 32, 48, 64, 96, 128, 192, 256, 320, 384, 448, 512, 640, 768, 896, 1024)


def _lib_linear(x2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    M = x2.shape[0]
    if M > GEMM_M_BUCKETS[-1] or M in GEMM_M_BUCKETS or not torch.cuda.tunable.is_enabled():
        return torch.nn.functional.linear(x2, w)
    Mp = next(b for b in GEMM_M_BUCKETS if b >= M)
    xp = torch.nn.functional.pad(x2, (0, 0, 0, Mp - M))
    return torch.nn.functional.linear(xp, w)[:M]


# ----------------------------------------------------------------------------- MFMA GEMM (M > GEMV_MAX_M)
# A plan is (cfg, grid): cfg indexes mgemm.hip's tile configurations; grid > 0 launches grid workgroups
# per output tile (split-K), grid < 0 launches min(-grid, work items) workgroups that stream equal shares
# of the (tile, k-step) items (stream-K: balanced whatever the tile count).
_MG_CFGS: Optional[list] = None
MG_GRIDS = (1, 2, 4, 8, 16, -256, -512, -768, -1024)


def mgemm_configs() -> list:
    """(BM, BN, threads, LDS bytes, SwiGLU-capable, row bytes per k-step) of every compiled mgemm.hip tile
    configuration."""
    global _MG_CFGS
    if _MG_CFGS is None:
        _MG_CFGS = [tuple(c) for c in native().mgemm_configs()]
    return _MG_CFGS


def _mg_occupancy(cfg: int) -> int:
    """Workgroups of a configuration resident per CU (LDS and the 32-wave limit)."""
    _, _, threads, lds, _, _ = mgemm_configs()[cfg]
    return max(1, min(160 * 1024 // lds, 2048 // threads))


def _mg_tiles(cfg: int, M: int, N: int, epi: int) -> int:
    bm, bn = mgemm_configs()[cfg][:2]
    feat = bn // 2 if epi == EPI_SWIGLU else bn
    return math.ceil(N / feat) * math.ceil(M / bm)


def mgemm_nwg(cfg: int, M: int, N: int, K: int, epi: int, fp8: bool, grid: int) -> int:
    total = _mg_tiles(cfg, M, N, epi) * (K * (1 if fp8 else 2) // mgemm_configs()[cfg][5])
    nwg = _mg_tiles(cfg, M, N, epi) * grid if grid > 0 else -grid
    return max(1, min(nwg, total))


def mgemm_valid(cfg: int, M: int, N: int, K: int, epi: int, fp8: bool, grid: int = 1, mx_out: bool = False) -> bool:
    """``fp8``: 0 / False bf16, 1 / True fp8 activations and weights, 3 MX activations (fp8 weights).  ``mx_out``: the SwiGLU epilogue writes MX e4m3 (fp8 / MX modes)."""
    if cfg < 0 or cfg >= len(mgemm_configs()):
        return False
    if int(fp8) == 3 and _mg_mode_lds(cfg, 3) < 0:
        return False
    if mx_out and (int(fp8) not in (1, 3) or N % 128 or
                   (_mg_mode_lds(cfg, 4) < 0 if epi == EPI_SWIGLU else (epi != EPI_BF16 or _mg_mode_lds(cfg, 5) < 0))):
        return False
    kb = K * (1 if fp8 else 2)
    if kb % mgemm_configs()[cfg][5] or N % 4 or M <= 0:
        return False
    if epi == EPI_SWIGLU and not mgemm_configs()[cfg][4]:
        return False
    return grid != 0


def _mgemm_ok(N: int, K: int, fp8: bool) -> bool:
    """Some mgemm configuration can run this shape (128-byte k-steps, 4-column output groups)."""
    return N % 4 == 0 and (K * (1 if fp8 else 2)) % 128 == 0


@functools.lru_cache(maxsize=256)
def _mg_mode_lds(cfg: int, mode: int) -> int:
    """LDS bytes of a configuration in a mode (3 MX activations; 4: 0 if its SwiGLU epilogue writes MX output), -1
    where the configuration is not built for it."""
    return native().mgemm_lds_bytes(cfg, mode)


def mgemm_mx_plan(M: int, N: int, K: int, epi: int, act_mx: bool, mx_out: bool) -> Optional[Tuple[int, int]]:
    """(cfg, grid) for fp8 weights with MX activations (``act_mx``; table key fp8 = 3) or MX SwiGLU output (key 4),
    or None: the tuned MX plan, else the tuned fp8 plan where that configuration runs the mode, else the fp8
    heuristic's, else the first weight-streaming / MFMA-dense configuration that does (same grid rule)."""
    mode = 3 if act_mx else 1
    if K % 128:
        return None
    for key in ((4 if epi == EPI_SWIGLU and mx_out else 3) if act_mx else 4, 3, 1):   # tuned MX plans, then fp8
        pick = _mg_table_row(M, N, K, epi, key)
        if pick is not None and mgemm_valid(pick[1], M, N, K, epi, mode, pick[2], mx_out):
            return pick[1], pick[2]
    cfg, grid = mgemm_heuristic(M, N, K, epi, 1)
    if mgemm_valid(cfg, M, N, K, epi, mode, grid, mx_out):
        return cfg, grid
    order = (12, 11, 8, 3, 2, 0, 13, 9, 5, 14, 15, 16, 19, 22) if M <= 128 else (15, 19, 22, 16, 17, 12)
    for c in order:
        if mgemm_valid(c, M, N, K, epi, mode, 1, mx_out):
            tiles = _mg_tiles(c, M, N, epi)
            steps = K // mgemm_configs()[c][5]
            split = 1
            while tiles * split * 2 <= 512 and steps // (split * 2) >= 8:
                split *= 2
            return c, split
    return None


@functools.lru_cache(maxsize=4096)
def _mg_plan_info(M: int, N: int, K: int, epi: int, fp8: bool, cfg: int, nwg: int) -> Tuple[int, int, int]:
    return tuple(native().mgemm_plan_info(M, N, K, epi, int(fp8), cfg, nwg))


def mgemm_heuristic(M: int, N: int, K: int, epi: int, fp8: bool, num_cus: int = 256) -> Tuple[int, int]:
    """Tile + grid choice for a shape the tuned table has never seen (tools/mgemm_tune.py measures the
    real choices; this only has to be reasonable)."""
    if M <= 64:    # weight streaming: small tiles, k-shared waves, one workgroup per tile
        cfg = (1 if epi == EPI_SWIGLU else 0) if M <= 16 else 7 if M <= 32 else 11
    elif M <= 128:
        cfg = 12
    elif M <= 256:
        cfg = 23
    else:
        cfg = 19
    if not mgemm_valid(cfg, M, N, K, epi, fp8):   # K not a multiple of the config's k-step: 128-byte k-steps
        cfg = 5 if M <= 16 else 9 if M <= 32 else 13 if M <= 64 else 15 if M <= 128 else 17
    tiles = _mg_tiles(cfg, M, N, epi)
    if tiles >= num_cus // 2:
        return cfg, 1
    steps = K * (1 if fp8 else 2) // mgemm_configs()[cfg][5]
    split = 1
    while tiles * split * 2 <= 2 * num_cus and steps // (split * 2) >= 8:
        split *= 2
    return cfg, split


# Tuned plans: engine/assets/mgemm_gfx950.json, written by tools/mgemm_tune.py, keyed
# "M_bucket,N,K,epi,fp8".  A row count between tuned buckets uses the plan of the nearest bucket
# above it (the largest one beyond the table).
_MG_TABLE: Optional[dict] = None
MG_TABLE_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "engine", "assets",
                             "mgemm_gfx950.json")


MG_M_BUCKETS = (2, 4, 8) + GEMM_M_BUCKETS   # row buckets of the mgemm plan table


def _mg_bucket(M: int) -> int:
    for b in MG_M_BUCKETS:
        if b >= M:
            return b
    return 1 << max(0, (M - 1).bit_length())


def _mg_load_table() -> dict:
    global _MG_TABLE
    if _MG_TABLE is None:
        _MG_TABLE = {}
        if os.environ.get("K8S_MGEMM_TABLE", "1") != "0" and os.path.isfile(MG_TABLE_PATH):
            import json

            with open(MG_TABLE_PATH) as f:
                plans = json.load(f).get("plans", {})
            # K8S_MGEMM_OVERRIDE="M,N,K,epi,fp8=cfg:grid;...": replace table rows (in-situ plan A/B runs)
            for item in filter(None, os.environ.get("K8S_MGEMM_OVERRIDE", "").split(";")):
                key, val = item.split("=")
                plans[key.strip()] = [int(t) for t in val.split(":")] + [0.0, 0.0]
            for k, v in plans.items():
                mb, n, kk, epi, fp8 = (int(t) for t in k.split(","))
                mg_us, lib_us = (float(v[2]), float(v[3])) if len(v) >= 4 else (0.0, 0.0)
                _MG_TABLE.setdefault((n, kk, epi, fp8), []).append((mb, int(v[0]), int(v[1]), mg_us, lib_us))
            for lst in _MG_TABLE.values():
                lst.sort()
    return _MG_TABLE


def _mg_table_row(M: int, N: int, K: int, epi: int, fp8: bool):
    rows = _mg_load_table().get((N, K, epi, int(fp8)))
    if not rows:
        return None
    mb = _mg_bucket(M)
    # nearest tuned bucket at or above M; past the largest tuned bucket the shape counts as untuned (a plan
    # tuned at 256 rows says nothing about an 8192-row prefill chunk)
    return next((r for r in rows if r[0] >= mb), None)


def mgemm_plan(M: int, N: int, K: int, epi: int, fp8: bool) -> Tuple[int, int]:
    pick = _mg_table_row(M, N, K, epi, fp8)
    if pick is not None and mgemm_valid(pick[1], M, N, K, epi, fp8, pick[2]):
        return pick[1], pick[2]
    return mgemm_heuristic(M, N, K, epi, fp8)


# split-K publish of mgemm (mgemm.hip): fence-free write-through slab stores + relaxed ticket (default) or the
# round-4 agent-scope release / acquire fences (K8S_MGEMM_FENCED=1); the same summation order, the same bits
MGEMM_FENCED = os.environ.get("K8S_MGEMM_FENCED", "0") == "1"


def mgemm(x: torch.Tensor, w, epi: int = EPI_BF16, cfg: Optional[int] = None,
          grid: Optional[int] = None, res: Optional[torch.Tensor] = None, rms_eps: Optional[float] = None,
          out: Optional[torch.Tensor] = None, act=None, mx_out: bool = False, fenced: Optional[bool] = None):
    """Hand-written MFMA GEMM (mgemm.hip): epi(x[M, K] @ w[N, K].T), any M (routed for M > GEMV_MAX_M).  ``w``: bf16 or
    Fp8Weight (activations are then quantized per token by quantize_act_fp8, or arrive as MX e4m3 in ``act``).
    SwiGLU: w = [Wg; Wu].  ``rms_eps``: RMSNorm prologue -- the result is scaled by 1/rms(x row) (the norm gamma must
    be folded into ``w``), so the un-normalised residual stream feeds the GEMM directly (bf16 or MX).  ``res``:
    residual epilogue (bf16 output only) -- out = x @ w.T + res, one rounding; ``out`` may be ``res`` (in place).
    ``act``: an :class:`MxAct` (mode 3, the block-scaled MFMA) or the (e4m3, per-token scale) pair of quantize_act_fp8.
    ``mx_out`` (fp8 weights, SwiGLU): returns the output as an :class:`MxAct` written by the epilogue.
    ``fenced``: split-K tiles publish their slabs with agent-scope release / acquire fences (the round-4 form) instead
    of the default fence-free write-through stores + relaxed ticket (None: ``K8S_MGEMM_FENCED``); same bits."""
    if isinstance(x, MxAct):
        act = x
    M, K = x.shape
    fp8 = _is_fp8(w)
    act_mx = isinstance(act, MxAct)
    mode = (3 if act_mx else 1) if fp8 else 0
    if (act_mx or mx_out) and not fp8:
        raise ValueError("mgemm: MX activations / output need fp8 weights")
    N = w.shape[0] // 2 if epi == EPI_SWIGLU else w.shape[0]
    if cfg is None:
        if act_mx or mx_out:
            plan = mgemm_mx_plan(M, N, K, epi, act_mx, mx_out)
            if plan is None:
                raise ValueError(f"mgemm: no MX configuration runs M={M} N={N} K={K} epi={epi}")
            cfg, grid = plan
        else:
            cfg, grid = mgemm_plan(M, N, K, epi, fp8)
    grid = grid or 1
    if not mgemm_valid(cfg, M, N, K, epi, mode, grid, mx_out):
        raise ValueError(f"mgemm: cfg {cfg} / grid {grid} invalid for M={M} N={N} K={K} epi={epi} mode={mode}"
                         f"{' mx_out' if mx_out else ''}")
    nwg = mgemm_nwg(cfg, M, N, K, epi, fp8, grid)
    tiles, cmax, n_ws = _mg_plan_info(M, N, K, epi, mode, cfg, nwg)
    if mode == 1 and rms_eps is not None:
        raise ValueError("mgemm: the RMS prologue needs bf16 or MX activations")
    if res is not None and (epi != EPI_BF16 or res.shape != (M, N)):
        raise ValueError("mgemm: residual epilogue needs a bf16 [M, N] residual and the bf16 epilogue")
    mxo = None
    if mx_out:
        if N % 128 or (epi == EPI_SWIGLU) == (res is not None):
            raise ValueError("mgemm: MX output is the SwiGLU or the residual epilogue's (N % 128 == 0)")
        mxo = MxAct.empty(M, N, x.device)
        if res is None:
            out = mxo.q   # SwiGLU: not written as bf16
    if out is None:
        out = torch.empty(M, N, dtype=F32 if epi == EPI_F32 else BF16, device=x.device)
    ws = torch.empty(n_ws, dtype=F32, device=x.device) if n_ws > 0 else None
    tk = _zeroed_scratch(x.device, "mgemm", 4 * tiles, 64 * 1024) if cmax > 1 else 0
    rp = _chk(res, BF16, "res") if res is not None else 0
    fn = int(MGEMM_FENCED if fenced is None else bool(fenced))
    rms, eps = (1, float(rms_eps)) if rms_eps is not None else (0, 0.0)
    oq, oe = (mxo.q.data_ptr(), mxo.e.data_ptr()) if mxo is not None else (0, 0)
    if act_mx:
        if act.shape != (M, K) or not act.q.is_cuda:
            raise ValueError(f"mgemm: MX activations {tuple(act.shape)} for x {(M, K)}")
        native().mgemm(out.data_ptr(), ws.data_ptr() if ws is not None else 0, tk, act.q.data_ptr(), w.q.data_ptr(),
                       act.e.data_ptr(), w.scale.data_ptr(), M, N, K, epi, 3, cfg, nwg, cmax, rp, rms, eps, -1, oq, oe,
                       fn)
    elif fp8:
        xq, sx = act if act is not None else quantize_act_fp8(x.contiguous())
        native().mgemm(out.data_ptr(), ws.data_ptr() if ws is not None else 0, tk, xq.data_ptr(), w.q.data_ptr(),
                       sx.data_ptr(), w.scale.data_ptr(), M, N, K, epi, 1, cfg, nwg, cmax, rp, 0, 0.0, -1, oq, oe, fn)
    else:
        native().mgemm(out.data_ptr(), ws.data_ptr() if ws is not None else 0, tk, _chk(x, BF16, "x"),
                       _chk(w, BF16, "w"), 0, 0, M, N, K, epi, 0, cfg, nwg, cmax, rp, rms, eps, -1, 0, 0, fn)
    del ws
    if mxo is not None:
        return (out, mxo) if res is not None else mxo
    return out


# ----------------------------------------------------------------------------- big-tile MFMA GEMM (prefill rows)
_PG_CFGS: Optional[list] = None


def pgemm_configs() -> list:
    """(BP weight rows, BQ tokens, LDS bytes) of every compiled pgemm.hip tile configuration."""
    global _PG_CFGS
    if _PG_CFGS is None:
        _PG_CFGS = [tuple(c) for c in native().pgemm_configs()]
    return _PG_CFGS


def pgemm_ok(N: int, K: int, fp8: bool) -> bool:
    """pgemm.hip can run this shape: 128-byte k-tiles, 4-column output groups."""
    return N % 4 == 0 and (K * (1 if fp8 else 2)) % 128 == 0


def pgemm_tiles(cfg: int, M: int, N: int, epi: int) -> int:
    bp, bq, _ = pgemm_configs()[cfg]
    feat = bp // 2 if epi == EPI_SWIGLU else bp
    return math.ceil(N / feat) * math.ceil(M / bq)


def pgemm(x: torch.Tensor, w, epi: int = EPI_BF16, cfg: int = 0, splits: int = 1, group_m: int = 4,
          res: Optional[torch.Tensor] = None, rms_eps: Optional[float] = None,
          out: Optional[torch.Tensor] = None, act=None, mx_out: bool = False):
    """Big-tile MFMA GEMM (pgemm.hip): epi(x[M, K] @ w[N, K].T) for prefill-size M.  Same contract as :func:`mgemm`
    (bf16 or Fp8Weight, SwiGLU with w = [Wg; Wu], residual epilogue, RMS prologue with the gamma folded into w, MX
    activations / MX SwiGLU output with fp8 weights); ``splits`` k-slices per output tile, ``group_m`` m-tiles per
    tile-order group."""
    if isinstance(x, MxAct):
        act = x
    M, K = x.shape
    fp8 = _is_fp8(w)
    act_mx = isinstance(act, MxAct)
    if (act_mx or mx_out) and not fp8:
        raise ValueError("pgemm: MX activations / output need fp8 weights")
    N = w.shape[0] // 2 if epi == EPI_SWIGLU else w.shape[0]
    if not pgemm_ok(N, K, fp8):
        raise ValueError(f"pgemm: unsupported shape N={N} K={K}")
    if fp8 and rms_eps is not None:
        raise ValueError("pgemm: the RMS prologue needs bf16 activations")
    if res is not None and (epi != EPI_BF16 or res.shape != (M, N)):
        raise ValueError("pgemm: residual epilogue needs a bf16 [M, N] residual and the bf16 epilogue")
    nwg, n_ws, n_tk = native().pgemm_plan(M, N, K, epi, int(fp8), cfg, splits)
    mxo = None
    if mx_out:
        if epi != EPI_SWIGLU or N % 128 or res is not None:
            raise ValueError("pgemm: MX output is the SwiGLU epilogue's (N % 128 == 0)")
        mxo = MxAct.empty(M, N, x.device)
        out = mxo.q   # (not written as bf16)
    if out is None:
        out = torch.empty(M, N, dtype=F32 if epi == EPI_F32 else BF16, device=x.device)
    ws = torch.empty(n_ws, dtype=F32, device=x.device) if n_ws > 0 else None
    tk = _zeroed_scratch(x.device, "pgemm", 4 * n_tk, 64 * 1024) if n_tk > 0 else 0
    rp = _chk(res, BF16, "res") if res is not None else 0
    rms, eps = (1, float(rms_eps)) if rms_eps is not None else (0, 0.0)
    oq, oe = (mxo.q.data_ptr(), mxo.e.data_ptr()) if mxo is not None else (0, 0)
    if act_mx:
        if act.shape != (M, K) or not act.q.is_cuda:
            raise ValueError(f"pgemm: MX activations {tuple(act.shape)} for x {(M, K)}")
        native().pgemm(out.data_ptr(), ws.data_ptr() if ws is not None else 0, tk, act.q.data_ptr(), w.q.data_ptr(),
                       act.e.data_ptr(), w.scale.data_ptr(), M, N, K, epi, 3, cfg, splits, group_m, rp, 0, 0.0, -1,
                       oq, oe)
    elif fp8:
        xq, sx = act if act is not None else quantize_act_fp8(x.contiguous())
        native().pgemm(out.data_ptr(), ws.data_ptr() if ws is not None else 0, tk, xq.data_ptr(), w.q.data_ptr(),
                       sx.data_ptr(), w.scale.data_ptr(), M, N, K, epi, 1, cfg, splits, group_m, rp, 0, 0.0, -1,
                       oq, oe)
    else:
        native().pgemm(out.data_ptr(), ws.data_ptr() if ws is not None else 0, tk, _chk(x, BF16, "x"),
                       _chk(w, BF16, "w"), 0, 0, M, N, K, epi, 0, cfg, splits, group_m, rp, rms, eps, -1)
    del ws
    return mxo if mxo is not None else out


_P4_CFGS: Optional[list] = None


def pgemm4_configs() -> list:
    """(BP weight rows, BQ tokens, LDS bytes) of every compiled pgemm4.hip tile configuration (4 waves)."""
    global _P4_CFGS
    if _P4_CFGS is None:
        _P4_CFGS = [tuple(c) for c in native().pgemm4_configs()]
    return _P4_CFGS


def pgemm4_tiles(cfg: int, M: int, N: int, epi: int) -> int:
    bp, bq, _ = pgemm4_configs()[cfg]
    feat = bp // 2 if epi == EPI_SWIGLU else bp
    return math.ceil(N / feat) * math.ceil(M / bq)


def pgemm4(x: torch.Tensor, w: torch.Tensor, epi: int = EPI_BF16, cfg: int = 0, splits: int = 1, group_m: int = 4,
           res: Optional[torch.Tensor] = None, rms_eps: Optional[float] = None,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """4-wave big-tile bf16 MFMA GEMM (pgemm4.hip): epi(x[M, K] @ w[N, K].T), K % 64 == 0.  ``splits`` k-slices per
    tile (fp32 slabs + a parallel combine kernel); residual epilogue and RMS prologue as :func:`mgemm`."""
    M, K = x.shape
    N = w.shape[0] // 2 if epi == EPI_SWIGLU else w.shape[0]
    if res is not None and (epi != EPI_BF16 or res.shape != (M, N)):
        raise ValueError("pgemm4: residual epilogue needs a bf16 [M, N] residual and the bf16 epilogue")
    _nwg, n_slab = native().pgemm4_plan(M, N, K, epi, cfg, splits)
    if out is None:
        out = torch.empty(M, N, dtype=F32 if epi == EPI_F32 else BF16, device=x.device)
    slab = torch.empty(n_slab, dtype=F32, device=x.device) if n_slab > 0 else None
    rp = _chk(res, BF16, "res") if res is not None else 0
    rms, eps = (1, float(rms_eps)) if rms_eps is not None else (0, 0.0)
    native().pgemm4(out.data_ptr(), slab.data_ptr() if slab is not None else 0, _chk(x, BF16, "x"), _chk(w, BF16, "w"),
                    M, N, K, epi, cfg, splits, group_m, rp, rms, eps, -1)
    del slab
    return out


# ----------------------------------------------------------------------------- GEMM routing (M > GEMV_MAX_M)
# Tuned big-tile plans: engine/assets/pgemm_gfx950.json, written by tools/pgemm_tune.py, keyed "M,N,K,epi,fp8" ->
# [kernel, cfg, splits, group_m, us, library us].  A row count between tuned buckets takes the plan of the nearest
# bucket at or above it; past the largest tuned bucket, the largest one's (big tiles, no split-K: it only gets
# better with more rows).
_PG_TABLE: Optional[dict] = None
PG_TABLE_PATH = os.environ.get("K8S_PGEMM_TABLE_PATH") or os.path.join(   # (override: in-situ table A/B runs)
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "engine", "assets", "pgemm_gfx950.json")
PG_MIN_M = 129      # below: mgemm's streaming tiles (batched decode, short prefill chunks)


def _pg_load_table() -> dict:
    global _PG_TABLE
    if _PG_TABLE is None:
        _PG_TABLE = {}
        if os.environ.get("K8S_PGEMM_TABLE", "1") != "0" and os.path.isfile(PG_TABLE_PATH):
            import json

            with open(PG_TABLE_PATH) as f:
                plans = json.load(f).get("plans", {})
            for k, v in plans.items():
                m, n, kk, epi, fp8 = (int(t) for t in k.split(","))
                _PG_TABLE.setdefault((n, kk, epi, fp8), []).append((m, str(v[0]), int(v[1]), int(v[2]), int(v[3]),
                                                                    float(v[4])))
            for lst in _PG_TABLE.values():
                lst.sort()
    return _PG_TABLE


def pgemm_heuristic(M: int, N: int, K: int, epi: int, fp8: bool, num_cus: int = 256) -> Tuple[str, int, int, int]:
    """Big-tile plan of a shape the table has never seen: 256 x 256 tiles (pgemm.hip), split-K until the grid
    covers the CUs."""
    cfg = 0
    tiles = pgemm_tiles(cfg, M, N, epi)
    kt = K * (1 if fp8 else 2) // 128
    s = 1
    while tiles * s * 2 <= num_cus and kt // (s * 2) >= 8:
        s *= 2
    return "pgemm", cfg, s, (1 if M <= 256 else 8)


def pgemm_plan_for(M: int, N: int, K: int, epi: int, fp8: bool) -> Tuple[Tuple[str, int, int, int], Optional[float]]:
    """((kernel, cfg, splits, group_m), tuned us or None) of the GEMM at M rows: kernel "pgemm" / "pgemm4", or "mgemm"
    where the tuner measured mgemm's own tuned plan faster."""
    rows = _pg_load_table().get((N, K, epi, int(fp8)))
    if rows:
        pick = next((r for r in rows if r[0] >= M), rows[-1])
        kern, cfg, sp, gm = pick[1:5]
        ok = kern == "mgemm" or (kern == "pgemm" and cfg < len(pgemm_configs())) or \
             (kern == "pgemm4" and not fp8 and cfg < len(pgemm4_configs()) and K % 64 == 0)
        if ok:
            return (kern, cfg, sp, gm), (pick[5] if pick[0] >= M else None)
    return pgemm_heuristic(M, N, K, epi, fp8), None


def gemm_route(M: int, N: int, K: int, epi: int, fp8: bool) -> Tuple[str, Optional[tuple]]:
    """Kernel of a GEMM with M > GEMV_MAX_M rows: ("mgemm", None), ("pgemm" | "pgemm4", (cfg, splits, group_m)) or
    ("library", None).  K8S_GEMM=auto (default): hand-written always -- mgemm for streaming row counts, the tuned
    fastest of mgemm and the big-tile kernels from PG_MIN_M rows on; =library: hipBLASLt / _scaled_mm (the A/B oracle);
    =mgemm / =pgemm force one hand-written kernel family."""
    if GEMM_BACKEND == "library":
        return "library", None
    mg_ok, pg_ok = _mgemm_ok(N, K, fp8), pgemm_ok(N, K, fp8)
    if GEMM_BACKEND == "mgemm" or (mg_ok and not pg_ok):
        return ("mgemm", None) if mg_ok else ("library", None)
    if not pg_ok:
        return "library", None
    plan, pg_us = pgemm_plan_for(M, N, K, epi, fp8)
    if GEMM_BACKEND == "pgemm":
        if plan[0] == "mgemm":
            plan = pgemm_heuristic(M, N, K, epi, fp8)
        return plan[0], plan[1:]
    if M < PG_MIN_M or plan[0] == "mgemm":   # (the tuner records "mgemm" where its tuned plan was faster)
        return "mgemm", None
    return plan[0], plan[1:]


def mx_rows(M: int, w) -> bool:
    """An fp8 GEMM of M rows against ``w`` (the consumer: O or down) takes its input as MX e4m3 (:class:`MxAct`):
    above the GEMV / sgemv rows (bf16 activations there), K % 128 == 0, on mgemm (or pgemm with K8S_MX_PGEMM=1)."""
    if not (MX_ON and _is_fp8(w) and M > max(GEMV_MAX_M, SGEMV_MAX_M)
            and GEMM_BACKEND != "library" and w.shape[1] % 128 == 0):
        return False
    return MX_PGEMM or gemm_route(M, w.shape[0], w.shape[1], EPI_BF16, True)[0] == "mgemm"


def _gemm_mx(act: MxAct, w, epi: int, res: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None, mx_res: bool = False):
    """An MX-activation GEMM on the routed kernel (mgemm MX mode / pgemm MX mode).  ``mx_res`` (residual
    epilogue on mgemm): returns (res, MxAct of the new residual stream), or (res, None) where no plan writes it."""
    M, K = act.shape
    N = w.shape[0] // 2 if epi == EPI_SWIGLU else w.shape[0]
    kern, plan = gemm_route(M, N, K, epi, True)
    if mx_res:
        if kern == "mgemm" and mgemm_mx_plan(M, N, K, epi, True, True) is not None:
            return mgemm(act, w, epi, res=res, out=out, mx_out=True)
        return _gemm_mx(act, w, epi, res=res, out=out), None
    if kern == "pgemm":
        cfg, sp, gm = plan
        return pgemm(act, w, epi, cfg=cfg, splits=sp, group_m=gm, res=res, out=out)
    if kern == "library":   # K8S_GEMM=library (the A/B oracle): per-token e4m3 of the dequantized MX rows
        y = _fp8_gemm(act.dequant(), w, F32 if epi == EPI_F32 else BF16) if epi != EPI_SWIGLU else \
            silu_mul(_fp8_gemm(act.dequant(), w))
        if res is not None:
            res.add_(y)
            return res
        return y
    return mgemm(act, w, epi, res=res, out=out)


def _gemm(x2: torch.Tensor, w, epi: int, res: Optional[torch.Tensor] = None, rms_eps: Optional[float] = None,
          out: Optional[torch.Tensor] = None, act=None, mx_out: bool = False):
    """Routed hand-written GEMM of M > GEMV_MAX_M rows (None: the library route).  ``act``: the fp8 activations
    (e4m3, per-token scales) when the caller quantized them already, or an :class:`MxAct`.  ``mx_out`` (fp8 SwiGLU):
    the result as an :class:`MxAct` where the routed kernel's plan writes it (else bf16)."""
    if isinstance(act, MxAct):
        return _gemm_mx(act, w, epi, res=res, out=out)
    M, K = x2.shape
    fp8 = _is_fp8(w)
    if mx_out and fp8 and act is not None:
        N = w.shape[0] // 2
        kern, plan = gemm_route(M, N, K, epi, True)
        if kern == "pgemm" and N % 128 == 0:
            cfg, sp, gm = plan
            return pgemm(x2, w, epi, cfg=cfg, splits=sp, group_m=gm, act=act, mx_out=True)
        if kern == "mgemm" and mgemm_mx_plan(M, N, K, epi, False, True) is not None and N % 128 == 0:
            return mgemm(x2, w, epi, act=act, mx_out=True)
    if M <= SGEMV_MAX_M and act is None:
        y = _sgemv(x2, w, epi, res=res, rms_eps=rms_eps, out=out)
        if y is not None:
            return y
    N = w.shape[0] // 2 if epi == EPI_SWIGLU else w.shape[0]
    kern, plan = gemm_route(M, N, K, epi, fp8)
    if kern == "library" or (fp8 and rms_eps is not None):
        return None   # (fp8: the activations are quantized after the norm, so the caller normalises first)
    if kern == "mgemm":
        return mgemm(x2, w, epi, res=res, rms_eps=rms_eps, out=out, act=act)
    cfg, sp, gm = plan
    if kern == "pgemm4":
        return pgemm4(x2, w, epi, cfg=cfg, splits=sp, group_m=gm, res=res, rms_eps=rms_eps, out=out)
    return pgemm(x2, w, epi, cfg=cfg, splits=sp, group_m=gm, res=res, rms_eps=rms_eps, out=out, act=act)


# bf16 rows in (SGEMV_MAX_M, RMS_PROLOGUE_MAX_UNFUSED] with at least RMS_UNFUSED_MIN_N output features take a
# separate RMSNorm + plain GEMM instead of mgemm's RMS prologue (K8S_RMS_UNFUSED_MAX_M; 0, the default = always the
# prologue).  Round 4 (profiles/bench_r4_rms_prologue_ab.txt) measured the separate norm faster for the TP = 1
# projections while the prologue squared x with v_dot2 in every k-step.  Round 5 takes the sums of squares from one
# extra MFMA (x . x^T diagonal, mgemm.hip) on the wide projections, which made gate/up's prologue the faster form
# (profiles/rms_policy_ab_r5.txt); with the QKV plans re-tuned for the prologue in situ the TP = 1 QKV's prologue wins
# too (batch 64 29.49 -> 29.09 ms/step, batch 32 26.63 -> 26.21 -- profiles/qkv_rms_ab_r5.txt).
RMS_PROLOGUE_MAX_UNFUSED = int(os.environ.get("K8S_RMS_UNFUSED_MAX_M", "0"))
# ... except gate/up (SwiGLU): its prologue always (K8S_RMS_PROLOGUE_SWIGLU=0: the round-4 rule for it too)
RMS_PROLOGUE_SWIGLU = os.environ.get("K8S_RMS_PROLOGUE_SWIGLU", "1") != "0"
RMS_UNFUSED_MIN_N = int(os.environ.get("K8S_RMS_UNFUSED_MIN_N", "8192"))


def linear_rms(r: torch.Tensor, w, eps: float, epi: int = EPI_BF16, mx_consumer=None, x_mx: Optional[MxAct] = None):
    """epi(rmsnorm(r) @ w.T) for M > GEMV_MAX_M rows with the norm gamma folded into ``w`` (LlamaModel folds it at
    load time): on the mgemm route the RMS statistics are the GEMM's prologue (no norm kernel, no normalised
    copy of the activations); otherwise a plain RMSNorm (unit gamma) + the routed GEMM.  ``mx_consumer`` (SwiGLU, fp8
    weights): the weight of the GEMM that consumes the result (down); where :func:`mx_rows` holds for it, the
    epilogue writes the result as an :class:`MxAct`.  ``x_mx``: the MX copy of ``r`` its producer wrote (residual
    epilogue): the GEMM runs on it, the RMS statistics taken from the dequantized MX values in its prologue."""
    M, K = r.shape
    mx_out = (mx_consumer is not None and epi == EPI_SWIGLU and _is_fp8(w) and mx_rows(M, mx_consumer)
              and (w.shape[0] // 2) % 128 == 0)
    if x_mx is not None and _is_fp8(w):
        if not x_mx.is_cuda:
            xa = x_mx.dequant(torch.float32)
            xa = xa * torch.rsqrt(xa.pow(2).mean(-1, keepdim=True) + eps)
            if epi == EPI_SWIGLU:
                y = ref.linear_swiglu(xa, w).to(BF16)
                return quantize_act_mx(y) if mx_out else y
            return ref.linear(xa, w, F32 if epi == EPI_F32 else BF16)
        n_out = w.shape[0] // 2 if epi == EPI_SWIGLU else w.shape[0]
        if gemm_route(M, n_out, K, epi, True)[0] == "mgemm" and \
                mgemm_mx_plan(M, n_out, K, epi, True, mx_out) is not None:
            return mgemm(x_mx, w, epi, rms_eps=eps, mx_out=mx_out)
    if _is_fp8(w) and M > max(GEMV_MAX_M, SGEMV_MAX_M):
        # fp8 GEMM rows: e4m3 of the UN-normalised rows with 1/rms folded into the per-token scales (one kernel
        # reads r once; no rmsnorm kernel, no normalised copy) -> the fp8 GEMM
        act = quantize_act_fp8(r.contiguous(), rms_eps=eps)
        if _gpu(r):
            y = _gemm(r.contiguous(), w, epi, act=act, mx_out=mx_out)
            if y is None:   # K8S_GEMM=library
                _library_allowed("linear_rms", r, w)
                y = _fp8_gemm(r, w, F32 if epi == EPI_F32 else BF16, act=act) if epi != EPI_SWIGLU else \
                    silu_mul(_fp8_gemm(r, w, act=act))
            return y
        xa = ref.dequant_fp8(act[0], act[1], torch.float32)
        if epi == EPI_SWIGLU:
            y = ref.linear_swiglu(xa, w).to(BF16)
            return quantize_act_mx(y) if mx_out else y
        return ref.linear(xa, w, F32 if epi == EPI_F32 else BF16)
    n_out = w.shape[0] // 2 if epi == EPI_SWIGLU else w.shape[0]
    if _gpu(r) and M > GEMV_MAX_M and (M <= SGEMV_MAX_M or M > RMS_PROLOGUE_MAX_UNFUSED or _is_fp8(w)
                                       or n_out < RMS_UNFUSED_MIN_N or (epi == EPI_SWIGLU and RMS_PROLOGUE_SWIGLU)):
        y = _gemm(r.contiguous(), w, epi, rms_eps=eps)
        if y is not None:
            return y
        if _is_fp8(w):   # small fp8 batches never quantize their activations (the CPU oracle assumes it)
            raise NoKernelForShape(f"linear_rms: sgemv declined fp8 x {tuple(r.shape)} (K needs > 1 k-group)")
    ones = _ones(K, r.device)
    x = rmsnorm(r, ones, eps)
    if epi == EPI_SWIGLU:
        return linear_swiglu(x, w)
    return linear(x, w, F32 if epi == EPI_F32 else None)


def linear_residual(x, w, res: torch.Tensor, mx_next=None):
    """res + x @ w.T (bf16), written into ``res`` (the residual stream).  mgemm route: the add is the GEMM's
    epilogue; otherwise GEMM + add.  ``x``: bf16, or an :class:`MxAct` (fp8 weights); bf16 rows of
    :func:`mx_rows` are turned into MX first (the producers that write MX themselves pass an MxAct).
    ``mx_next``: the weight of the pre-norm projection that reads the new residual stream next; then returns
    (res, MxAct or None) -- the residual epilogue writes the stream's MX copy where :func:`mx_rows` holds for it."""
    M, K = x.shape
    want_mx = mx_next is not None and mx_rows(M, mx_next) and res.shape[1] % 128 == 0
    if not isinstance(x, MxAct) and mx_rows(M, w) and K % 128 == 0:
        x = quantize_act_mx(x.contiguous())
    if isinstance(x, MxAct):
        if not x.is_cuda:
            y = ref.linear(x.dequant(torch.float32), w).to(BF16)
            res.copy_((res.float() + y.float()).to(res.dtype))
            if mx_next is not None:
                return res, (quantize_act_mx(res) if want_mx else None)
            return res
        if mx_next is not None:
            return _gemm_mx(x, w, EPI_BF16, res=res, out=res, mx_res=want_mx) if want_mx else \
                (_gemm_mx(x, w, EPI_BF16, res=res, out=res), None)
        return _gemm_mx(x, w, EPI_BF16, res=res, out=res)
    if mx_next is not None:
        return linear_residual(x, w, res), None
    if _gpu(x) and M > GEMV_MAX_M:
        y = _gemm(x.contiguous(), w, EPI_BF16, res=res, out=res)
        if y is not None:
            return y
    y = linear(x, w)
    if y.is_cuda:
        res.add_(y)
    else:
        res.copy_((res.float() + y.float()).to(res.dtype))
    return res


_ONES: dict = {}


def _ones(K: int, dev) -> torch.Tensor:
    key = (K, str(dev))
    if key not in _ONES:
        _ONES[key] = torch.ones(K, dtype=BF16, device=dev)
    return _ONES[key]


# GEMMs with more than GEMV_MAX_M rows: see gemm_route.
GEMM_BACKEND = os.environ.get("K8S_GEMM", "auto")
if GEMM_BACKEND not in ("mgemm", "pgemm", "library", "auto"):
    raise ValueError(f"K8S_GEMM must be auto, mgemm, pgemm or library (got {GEMM_BACKEND!r})")


def linear(x: torch.Tensor, w: torch.Tensor, out_dtype=None) -> torch.Tensor:
    """y = x @ w.T with w [N, K] (bf16 or Fp8Weight).  M <= GEMV_MAX_M rows: hand-written HBM-streaming GEMV;
    more rows (batched decode, prefill): hand-written MFMA GEMM (mgemm.hip)."""
    if isinstance(x, MxAct):   # MX rows (fp8 weights): the producer's quantized activations
        if not x.is_cuda:
            return ref.linear(x.dequant(torch.float32), w, out_dtype or BF16)
        return _gemm_mx(x, w, EPI_F32 if out_dtype == F32 else EPI_BF16)
    if not _gpu(x, w):
        return ref.linear(_ref_act_quant(x, w), w, out_dtype)
    x2 = x.reshape(-1, x.shape[-1])
    epi = EPI_F32 if out_dtype == F32 else EPI_BF16
    y = None
    if x2.shape[0] <= GEMV_MAX_M:
        y = _gemv(x2.contiguous(), w, epi, out_dtype or BF16)
    elif out_dtype in (None, BF16, F32):
        y = _gemm(x2.contiguous(), w, epi)
    if y is not None:
        pass
    elif _is_fp8(w):
        _library_allowed("linear", x2, w, out_dtype)
        y = _fp8_gemm(x2, w, out_dtype)
    else:
        _library_allowed("linear", x2, w, out_dtype)
        y = _lib_linear(x2, w)
        if out_dtype is not None and out_dtype != y.dtype:
            y = y.to(out_dtype)
    return y.view(*x.shape[:-1], y.shape[-1])


class NoKernelForShape(RuntimeError):
    """No hand-written kernel accepts this GEMM (and K8S_GEMM is not ``library``)."""


def _library_allowed(op: str, x2: torch.Tensor, w, out_dtype=None) -> None:
    """The library GEMMs (hipBLASLt / torch._scaled_mm) run only under K8S_GEMM=library, the A/B oracle: on the
    default route a shape no hand-written kernel accepts is an error, never a silent switch to the library."""
    if GEMM_BACKEND == "library":
        return
    t = w.q if _is_fp8(w) else w
    raise NoKernelForShape(
        f"{op}: no hand-written kernel for x {tuple(x2.shape)} @ w {tuple(t.shape)}^T ({'fp8' if _is_fp8(w) else 'bf16'}"
        f" weights, out {out_dtype or 'bf16'}; the GEMMs need N % 4 == 0 and 128-byte k-steps) under K8S_GEMM="
        f"{GEMM_BACKEND}; K8S_GEMM=library runs the library GEMMs")


def linear_norm(x: torch.Tensor, w, norm_w: Optional[torch.Tensor], eps: float,
                res_in: Optional[torch.Tensor], res_out: Optional[torch.Tensor], epi: int = EPI_BF16) -> torch.Tensor:
    """Decode-path fused pre-norm projection (M <= 8 rows):
    r = x + res_in (or x), res_out <- r, y = epi(rmsnorm(r) * norm_w @ w.T).
    ``norm_w=None``: the norm weight has been folded into ``w`` (LlamaModel does this at load time),
    so y = epi((r @ w.T) / rms(r)) and the kernel skips the normalisation pass.
    res_in and res_out must be distinct buffers (ping-pong).  ``w``: bf16 tensor or Fp8Weight."""
    if res_in is not None and res_out is not None and res_in.data_ptr() == res_out.data_ptr():
        raise ValueError("res_in and res_out must be different buffers")
    M, K = x.shape
    if not _gpu(x, w):
        r = x if res_in is None else (x.float() + res_in.float()).to(x.dtype)
        if res_out is not None:
            res_out.copy_(r)
        h, _ = ref.rmsnorm(r, norm_w if norm_w is not None else torch.ones(K, dtype=r.dtype), eps)
        if epi == EPI_SWIGLU:
            return ref.linear_swiglu(h, w)
        return ref.linear(h, w, F32 if epi == EPI_F32 else None)
    if M > GEMV_KERNEL_MAX_M:
        raise ValueError("linear_norm is the decode GEMV (M <= 8)")
    return _gemv(x, w, epi, F32 if epi == EPI_F32 else BF16, norm_w=norm_w, eps=eps, res_in=res_in, res_out=res_out,
                 folded=norm_w is None)


def cascade_groups_max(B: int, nq: int, nkv: int) -> int:
    """Prefix groups (partials per row and head) of the cascade decode attention at B rows: about 256 workgroups
    of decode_prefix_kernel over (groups, kv heads, column blocks), 2-32 groups (each group's partial is a row's
    D + 2 floats per head, so more groups trade prefix-kernel parallelism for partial-sum traffic)."""
    cb = -(-B // (8 * max(1, 16 // max(1, nq // nkv))))
    return max(2, min(32, 256 // max(1, nkv * cb)))


def cascade_ok(nq: int, nkv: int, block_size: int, D: int) -> bool:
    """Shapes the cascade (shared-prefix) decode attention takes."""
    G = nq // nkv if nkv else 0
    return block_size == 16 and D == 128 and nkv > 0 and nq % nkv == 0 and G in (1, 2, 4, 8, 16)


def decode_attention_fused(qkv: torch.Tensor, cos_sin: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                           block_tables: torch.Tensor, context_lens: torch.Tensor, scale: float, block_size: int,
                           max_context: int, nq: int, nkv: int, D: int, mx: bool = False, cascade=None):
    """RoPE + KV write of the new token + paged GQA attention, one kernel.  Returns [B, nq*D] bf16, or with ``mx``
    an :class:`MxAct` (the fp8 O projection's input: written as MX e4m3 by the one-workgroup kernel and its merge;
    the other forms quantize their bf16 output).

    ``cascade`` = (cas, ngm): the batch's shared prefix -- cas a device int32 [2] = (64-token spans every active row
    shares, a row holding them), written by the engine before the step -- is attended once for all rows by
    decode_prefix_kernel (ngm partials per row and head) and merged into the per-row attention, whose partitions
    start after it: ``max_context`` then bounds the tokens PAST the shared prefix (the suffix), not the context.
    Exact (the same keys, the same softmax); on the CPU the plain per-row attention runs."""
    B = qkv.shape[0]
    if cascade is not None and _gpu(qkv, k_cache) and cascade_ok(nq, nkv, block_size, D):
        cas, ngm = cascade
        if cas.dtype != I32 or cas.numel() < 2 or not cas.is_cuda:
            raise ValueError("cascade: cas must be a device int32 tensor of 2 values")
        G = nq // nkv
        ps = G * D + 2 * G                      # floats per partial record (attn_decode_split.hip's layout)
        part = torch.empty(B * nkv * ngm * ps, dtype=F32, device=qkv.device)
        native().decode_prefix(part.data_ptr(), ngm, _chk(qkv, BF16, "qkv"), _chk(cos_sin, F32, "cos_sin"),
                               _chk(k_cache, BF16, "k_cache"), _chk(v_cache, BF16, "v_cache"),
                               _chk(block_tables, I32, "block_tables"), _chk(context_lens, I32, "context_lens"),
                               cas.data_ptr(), float(scale), B, nq, nkv, D, block_size, block_tables.shape[1], ngm, -1)
        # (the suffix on the one-wave-per-chunk split kernel, its last arriver merging the prefix records as well,
        # measured 1.7-3.6x slower: one wave folds every record of a pair -- profiles/cascade_kbench_r6.txt)
        return _decode_attention_onewg(qkv, cos_sin, k_cache, v_cache, block_tables, context_lens, scale, block_size,
                                       max_context, nq, nkv, D, mx, (cas.data_ptr(), part, ngm, ngm))
    if mx:
        if not _gpu(qkv, k_cache) or block_size != 16 or (B * nkv <= _split_pairs_limit(max_context)
                                                          and max_context <= 64 * SPLIT_PARTITION):
            return quantize_act_mx(decode_attention_fused(qkv, cos_sin, k_cache, v_cache, block_tables, context_lens,
                                                          scale, block_size, max_context, nq, nkv, D))
    if not _gpu(qkv, k_cache) or block_size != 16:
        if _gpu(qkv, k_cache):  # general block sizes: unfused kernels
            q = rope_kv_write(qkv, cos_sin, k_cache, v_cache, nq, nkv, D, context_lens=context_lens,
                              block_tables=block_tables, block_size=block_size)
            return paged_decode_attention(q, k_cache, v_cache, block_tables, context_lens, scale, block_size,
                                          max_context).view(B, nq * D)
        q = rope_kv_write(qkv, cos_sin, k_cache, v_cache, nq, nkv, D, context_lens=context_lens,
                          block_tables=block_tables, block_size=block_size)
        return ref.paged_decode_attention(q, k_cache, v_cache, block_tables, context_lens, scale,
                                          block_size).view(B, nq * D)
    if B * nkv <= _split_pairs_limit(max_context) and max_context <= 64 * SPLIT_PARTITION:
        return _decode_attention_split(qkv, cos_sin, k_cache, v_cache, block_tables, context_lens, scale, block_size,
                                       max_context, nq, nkv, D)
    return _decode_attention_onewg(qkv, cos_sin, k_cache, v_cache, block_tables, context_lens, scale, block_size,
                                   max_context, nq, nkv, D, mx, None)


def _decode_attention_onewg(qkv, cos_sin, k_cache, v_cache, block_tables, context_lens, scale, block_size,
                            max_context, nq, nkv, D, mx, cascade):
    """The one-workgroup-per-(row, kv head, partition) kernel (+ its merge); ``cascade`` = (cas pointer, prefix
    records, ngm, records per pair) of a decode_prefix_kernel launch that ran first."""
    B = qkv.shape[0]
    part = fused_partition(B * nkv)
    pmax = max(1, math.ceil(max_context / part))
    mxo = MxAct.empty(B, nq * D, qkv.device) if mx else None
    out = mxo.q if mx else torch.empty(B, nq * D, dtype=BF16, device=qkv.device)
    if pmax > 1:
        pacc = torch.empty(B * nq * pmax * D, dtype=F32, device=qkv.device)
        pml = torch.empty(B * nq * pmax * 2, dtype=F32, device=qkv.device)
        pa, pm = pacc.data_ptr(), pml.data_ptr()
    else:
        pa = pm = 0
    native().decode_attention_fused(out.data_ptr(), pa, pm, _chk(qkv, BF16, "qkv"), _chk(cos_sin, F32, "cos_sin"),
                                    _chk(k_cache, BF16, "k_cache"), _chk(v_cache, BF16, "v_cache"),
                                    _chk(block_tables, I32, "block_tables"), _chk(context_lens, I32, "context_lens"),
                                    float(scale), B, nq, nkv, D, block_size, block_tables.shape[1], pmax, part, -1,
                                    mxo.q.data_ptr() if mx else 0, mxo.e.data_ptr() if mx else 0,
                                    *((cascade[0], cascade[1].data_ptr(), cascade[2], cascade[3])
                                      if cascade is not None else (0, 0, 0, 0)))
    return mxo if mx else out


# Context tokens per workgroup of the one-workgroup-per-pair decode attention: 1024 (16 waves, one workgroup per CU
# by LDS).  K8S_ATTN_FUSED_PART=512 selects 8-wave workgroups (two per CU): faster for short contexts at TP = 1 with
# 64 sequences (ctx 256: 30.1 vs 32.3 us) but slower at the bench's ~0.5k contexts, which then take two partitions
# and the merge kernel (40.8 vs 36.1 us, decode 31.1 vs 30.6 ms/step; profiles/kbench_attn_split_vs_onewg.txt).
FUSED_PART_ENV = int(os.environ.get("K8S_ATTN_FUSED_PART", "1024"))


def fused_partition(pairs: int) -> int:
    return FUSED_PART_ENV if FUSED_PART_ENV in (512, 1024) else FUSED_PARTITION


def _decode_attention_split(qkv, cos_sin, k_cache, v_cache, block_tables, context_lens, scale, block_size,
                            max_context, nq, nkv, D) -> torch.Tensor:
    B = qkv.shape[0]
    pmax = max(1, math.ceil(max_context / SPLIT_PARTITION))
    out = torch.empty(B, nq * D, dtype=BF16, device=qkv.device)
    part = None
    if pmax > 1:
        part = torch.empty(native().decode_split_workspace(B, nq, nkv, pmax), dtype=F32, device=qkv.device)
    counters = _zeroed_scratch(qkv.device, "attn_split", B * nkv * 4)
    native().decode_attention_split(out.data_ptr(), part.data_ptr() if part is not None else 0, counters,
                                    _chk(qkv, BF16, "qkv"), _chk(cos_sin, F32, "cos_sin"),
                                    _chk(k_cache, BF16, "k_cache"), _chk(v_cache, BF16, "v_cache"),
                                    _chk(block_tables, I32, "block_tables"), _chk(context_lens, I32, "context_lens"),
                                    float(scale), B, nq, nkv, D, block_size, block_tables.shape[1], pmax, -1)
    del part
    return out


def linear_swiglu(x: torch.Tensor, w_gate_up: torch.Tensor) -> torch.Tensor:
    """silu(x @ Wg.T) * (x @ Wu.T) with w_gate_up = [Wg; Wu] ([2I, K]); the SwiGLU is the GEMM's epilogue."""
    if not _gpu(x, w_gate_up):
        return ref.linear_swiglu(_ref_act_quant(x, w_gate_up), w_gate_up)
    x2 = x.reshape(-1, x.shape[-1])
    y = None
    if x2.shape[0] <= GEMV_MAX_M:
        y = _gemv(x2.contiguous(), w_gate_up, EPI_SWIGLU, BF16)
    else:
        y = _gemm(x2.contiguous(), w_gate_up, EPI_SWIGLU)
    if y is not None:
        pass
    elif _is_fp8(w_gate_up):
        _library_allowed("linear_swiglu", x2, w_gate_up)
        y = silu_mul(_fp8_gemm(x2, w_gate_up))
    else:
        _library_allowed("linear_swiglu", x2, w_gate_up)
        y = silu_mul(_lib_linear(x2, w_gate_up))
    return y.view(*x.shape[:-1], y.shape[-1])


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    if not _gpu(gu):
        return ref.silu_mul(gu)
    I = gu.shape[-1] // 2
    T = gu.numel() // (2 * I)
    out = torch.empty(*gu.shape[:-1], I, dtype=gu.dtype, device=gu.device)
    native().silu_mul(out.data_ptr(), _chk(gu, BF16, "gu"), T, I, -1)
    return out


def embedding(ids: torch.Tensor, table: torch.Tensor, mx: bool = False):
    """table[ids] (bf16).  ``mx``: returns (rows, their MX e4m3 copy) -- the first fp8 pre-norm projection's input,
    written by the gather itself (K16)."""
    if not _gpu(ids, table):
        out = ref.embedding(ids, table)
        return (out, quantize_act_mx(out)) if mx else out
    T = ids.numel()
    out = torch.empty(T, table.shape[1], dtype=table.dtype, device=table.device)
    mxo = MxAct.empty(T, table.shape[1], table.device) if mx else None
    native().embedding(out.data_ptr(), _chk(ids, I32, "ids"), _chk(table, BF16, "table"), T, table.shape[1],
                       table.shape[0], -1, mxo.q.data_ptr() if mx else 0, mxo.e.data_ptr() if mx else 0)
    return (out, mxo) if mx else out


# ----------------------------------------------------------------------------- sampling
def sample(logits: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, seeds: torch.Tensor,
           counter: torch.Tensor, *, shards: int = 1, tokens_out: Optional[torch.Tensor] = None,
           ctx_inc: Optional[torch.Tensor] = None, hist: Optional[torch.Tensor] = None,
           steps: Optional[torch.Tensor] = None, nucleus: Optional[bool] = None,
           slots: Optional[torch.Tensor] = None, stop: Optional[dict] = None, tp=None) -> torch.Tensor:
    """Sample one token per row.  logits: [B, V] or sharded [shards, B, Vs] fp32.  Optionally
    updates decode state in place: tokens_out[s] = tok, ctx_inc[s] += 1, hist[s, steps[s]] = tok,
    steps[s] += 1 (slots with ctx_inc[s] <= 0 are padding and untouched), where s = slots[b] (or b).

    ``nucleus``: run the top-p passes (rows with 0 < temperature and top_p < 1).  None = decide
    from the tensors (a device sync: not inside graph capture); False = top_p is ignored, which is
    what a graph captured for top_p = 1 requests does (three fewer launches per token).

    ``stop``: device-side stop detection of the decode graphs (sampler.hip StopArgs): dict with ``cls``
    [vocab, 2] int32 token classes, ``json`` / ``cfg`` [slots] int32, optional ``forced`` [slots, n] /
    ``forced_len`` [slots] scripted tokens, ``eos_tok`` and ``done`` (GPU: a host-mapped device pointer int;
    CPU: an int32 tensor).  A finished answer sets ctx_inc[s] = 0 and done[s] = 1.

    ``tp`` (a TPGroup of world > 1) with ``logits`` [1, B, Vs] = this rank's vocab shard (the model's
    ``gather_logits = False``): vocab-parallel sampling -- every rank samples its own shard with noise keyed by the
    GLOBAL token id and the ranks exchange 8 bytes per row (plus, for top-p rows, the row max and two 256-bin integer
    histograms), instead of all-gathering B x V fp32 logits.  Same tokens as the gathered path, bit for bit."""
    if logits.dim() == 3:
        S, B, Vs = logits.shape
    else:
        (B, Vs), S = logits.shape, 1
    vp = tp is not None and tp.world > 1 and S == 1 and logits.dim() == 3
    if not _gpu(logits):
        if vp:
            toks = ref.sample_vocab_parallel(logits[0], temperature, top_p, seeds, counter, tp.rank,
                                             tp.all_gather_shards)
        else:
            full = logits.permute(1, 0, 2).reshape(B, S * Vs) if logits.dim() == 3 else logits
            toks = ref.sample(full, temperature, top_p, seeds, counter)
        idx = [int(slots[b]) if slots is not None else b for b in range(B)]
        if stop is not None and hist is not None and ctx_inc is not None:
            for b, s in enumerate(idx):
                if int(ctx_inc[s]) > 0:
                    ref.write_token_stop(s, int(toks[b]), tokens_out, ctx_inc, hist, steps, stop)
            return toks
        active = [ctx_inc is None or int(ctx_inc[s]) > 0 for s in idx]
        for b, s in enumerate(idx):
            if not active[b]:
                continue
            if tokens_out is not None:
                tokens_out[s] = toks[b]
            if hist is not None:
                if int(steps[s]) < hist.shape[1]:
                    hist[s, int(steps[s])] = toks[b]
                steps[s] += 1
            if ctx_inc is not None:
                ctx_inc[s] += 1
        return toks
    if nucleus is None:
        nucleus = bool(((top_p < 1) & (temperature > 0)).any())
    out = tokens_out if tokens_out is not None else torch.empty(B, dtype=I32, device=logits.device)
    nuc = _zeroed_scratch(logits.device, "sample_nucleus", native().sample_nucleus_bytes(B, S),
                          native().sample_nucleus_bytes(64, S)) if nucleus else 0
    if stop is not None:
        fz = stop.get("forced")
        st_args = (_chk(stop["cls"], I32, "stop.cls"), _chk(stop["json"], I32, "stop.json"),
                   _chk(stop["cfg"], I32, "stop.cfg"), _chk(fz, I32, "stop.forced") if fz is not None else 0,
                   _chk(stop["forced_len"], I32, "stop.forced_len") if fz is not None else 0,
                   fz.shape[1] if fz is not None else 0, int(stop["eos_tok"]), int(stop["done"]))
    else:
        st_args = (0, 0, 0, 0, 0, 0, 0, 0)
    p_temp, p_top, p_ctx = _chk(temperature, F32, "temperature"), _chk(top_p, F32, "top_p"), \
        (_chk(ctx_inc, I32, "ctx_inc") if ctx_inc is not None else 0)
    p_slots = _chk(slots, I32, "slots") if slots is not None else 0
    p_hist = _chk(hist, I32, "hist") if hist is not None else 0
    p_steps = _chk(steps, I32, "steps") if steps is not None else 0
    hstride = hist.shape[1] if hist is not None else 0
    if not vp:
        native().sample(_chk(out, I32, "tokens"), _chk(logits, F32, "logits"), B, Vs, S, p_temp, p_top,
                        _chk(seeds, I32, "seeds"), _chk(counter, I32, "counter"), p_ctx, p_hist, hstride, p_steps,
                        _sample_scratch(logits.device, B), nuc, p_slots, *st_args, -1)
        return out
    # vocab-parallel (sampler.hip k8s_sample_nuc_local / _combine / k8s_sample_merge): the ranks exchange row maxima,
    # bin totals and best keys through tp.all_gather_shards (xGMI inside the decode graphs: a few KiB)
    dev, lg = logits.device, _chk(logits, F32, "logits")
    if nucleus:
        ld = (B + 3) // 4 * 4
        mine = _zeroed_tensor(dev, "sample_tp_max", 4096, torch.int32)[:ld]   # re-armed by the combine
        native().sample_nuc_local(-1, lg, B, Vs, p_temp, p_top, p_ctx, p_slots, nuc, mine.data_ptr(), -1)
        g = tp.all_gather_shards(mine)
        native().sample_nuc_combine(-1, g.data_ptr(), ld, tp.world, B, p_temp, p_top, p_ctx, p_slots, nuc,
                                    mine.data_ptr(), -1)
        for level in (0, 1):
            h = torch.empty(B, 256, dtype=torch.int64, device=dev)
            native().sample_nuc_local(level, lg, B, Vs, p_temp, p_top, p_ctx, p_slots, nuc, h.data_ptr(), -1)
            g = tp.all_gather_shards(h.view(torch.int32))
            native().sample_nuc_combine(level, g.data_ptr(), B, tp.world, B, p_temp, p_top, p_ctx, p_slots, nuc, 0, -1)
    ldk = (B + 1) // 2 * 2
    keys = torch.empty(ldk, dtype=torch.int64, device=dev)   # every live row's key is written; the rest unread
    native().sample(_chk(out, I32, "tokens"), lg, B, Vs, 1, p_temp, p_top, _chk(seeds, I32, "seeds"),
                    _chk(counter, I32, "counter"), p_ctx, p_hist, hstride, p_steps, _sample_scratch(dev, B), nuc,
                    p_slots, *st_args, -1, id_base=tp.rank * Vs, keys_out=keys.data_ptr(), nuc_passes=0)
    g = tp.all_gather_shards(keys.view(torch.int32))
    native().sample_merge(out.data_ptr(), g.data_ptr(), ldk, tp.world, B, p_ctx, p_hist, hstride, p_steps, p_slots,
                          *st_args, -1)
    return out


def _zeroed_tensor(dev: torch.device, kind: str, numel: int, dtype: torch.dtype) -> torch.Tensor:
    """A persistent zero-initialised device tensor that its kernels leave zeroed again (see _zeroed_scratch)."""
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    t = _SCRATCH.get((kind, "tensor", i))
    if t is None or t.numel() < numel:
        t = torch.zeros(numel, dtype=dtype, device=dev)
        _SCRATCH.setdefault(("keep", i), []).append(t)
        _SCRATCH[(kind, "tensor", i)] = t
    return t


_STOP_CLS: dict = {}


def token_stop_classes(tok, vocab: int) -> torch.Tensor:
    """[vocab, 2] int32 token classes for the sampler's device-side stop detection (EOS ids and brace counts of
    every token's decoded text; reference.token_stop_classes), built once per tokenizer."""
    key = (id(tok._tok), vocab)
    if key not in _STOP_CLS:
        n = min(vocab, tok._tok.get_vocab_size())
        texts = tok._tok.decode_batch([[i] for i in range(n)], skip_special_tokens=True)
        _STOP_CLS[key] = ref.token_stop_classes(texts, sorted(tok.eos_ids), vocab)
    return _STOP_CLS[key]


_SCRATCH: dict = {}


def _zeroed_scratch(dev: torch.device, kind: str, nbytes: int, min_bytes: int = 4096) -> int:
    """Zeroed scratch of a kernel that leaves it zeroed again after every launch (arrival counters,
    atomic keys).  Buffers are never freed because captured graphs keep their pointers; stream order
    serialises the launches that share one."""
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    buf = _SCRATCH.get((kind, i))
    if buf is None or buf.numel() < nbytes:
        buf = torch.zeros(max(nbytes, min_bytes), dtype=torch.uint8, device=dev)
        _SCRATCH.setdefault(("keep", i), []).append(buf)
        _SCRATCH[(kind, i)] = buf
    return buf.data_ptr()


def _sample_scratch(dev: torch.device, B: int) -> int:
    """Per-row (atomic key, arrival counter) scratch of the multi-workgroup sampler."""
    return _zeroed_scratch(dev, "sample", native().sample_scratch_bytes(B), native().sample_scratch_bytes(256))


# ----------------------------------------------------------------------------- init
def hash_init_(out: torch.Tensor, gcols: int, row0: int, col0: int, seed: int, tensor_id: int,
               scale: float, shift: float = 0.0) -> torch.Tensor:
    """Fill a 2-D bf16 shard with the deterministic hash-uniform init (see reference.hash_init)."""
    rows, cols = out.shape
    if not out.is_cuda:
        out.copy_(ref.hash_init(rows, cols, gcols, row0, col0, seed, tensor_id, scale, shift, out.dtype))
        return out
    native().hash_init(_chk(out, BF16, "out"), rows, cols, gcols, row0, col0, seed & 0xFFFFFFFF,
                       tensor_id & 0xFFFFFFFF, float(scale), float(shift), -1)
    return out
