"""Plain-PyTorch fp32 reference implementations of every HIP kernel.

They define the semantics the kernels are tested against (T3 numerics tests compare a kernel
with the function of the same name here) and they run the model on CPU for the multi-process
``gloo`` tests (TP=k vs TP=1).  They are never used for CUDA tensors: the wrappers in
``ops/__init__.py`` refuse to fall back on a GPU.
"""

from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np
import torch

U32 = 0xFFFFFFFF


# ----------------------------------------------------------------------------- hashing / RNG
def _fmix32(h: torch.Tensor) -> torch.Tensor:
    h = h & U32
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & U32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & U32
    h = h ^ (h >> 16)
    return h


def hash3(a, b, c: torch.Tensor) -> torch.Tensor:
    """Same bits as common.h hash3 (int64 tensors holding uint32 values)."""
    c = torch.as_tensor(c, dtype=torch.int64)
    b = torch.as_tensor(b, dtype=torch.int64, device=c.device)
    a = torch.as_tensor(a, dtype=torch.int64, device=c.device)
    inner = _fmix32((c + 0x7F4A7C15) & U32)
    mid = _fmix32((((b + 0x9E3779B9) & U32) ^ inner) & U32)
    return _fmix32((a ^ mid) & U32)


def u01(h: torch.Tensor) -> torch.Tensor:
    return ((h >> 8).to(torch.float64) + 0.5) * (1.0 / 16777216.0)


def hash_init(rows: int, cols: int, gcols: int, row0: int, col0: int, seed: int, tensor_id: int,
              scale: float, shift: float, dtype=torch.bfloat16, device="cpu") -> torch.Tensor:
    r = torch.arange(rows, dtype=torch.int64, device=device).unsqueeze(1) + row0
    c = torch.arange(cols, dtype=torch.int64, device=device).unsqueeze(0) + col0
    flat = (r * gcols + c) & U32
    u = u01(hash3(seed, tensor_id, flat)).to(torch.float32)
    return ((2.0 * u - 1.0) * scale + shift).to(dtype)


# ----------------------------------------------------------------------------- layers
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float,
            residual: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    if residual is not None:
        r = (x.float() + residual.float()).to(x.dtype)
        residual.copy_(r)
        x = r
    xf = x.float()
    out = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return out.to(x.dtype), residual


def rope_table(head_dim: int, max_pos: int, theta: float, scaling: Optional[dict] = None) -> torch.Tensor:
    """[max_pos, head_dim] fp32: cos in [:, :D/2], sin in [:, D/2:] (llama3 scaling if given)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling["low_freq_factor"], scaling["high_freq_factor"]
        old = scaling["original_max_position_embeddings"]
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        inv_l = torch.where(wl > lo_wl, inv / factor, inv)
        smooth = (old / wl - lo) / (hi - lo)
        smoothed = (1 - smooth) * inv_l / factor + smooth * inv_l
        medium = (wl >= hi_wl) & (wl <= lo_wl)
        inv = torch.where(medium, smoothed, inv_l)
    pos = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(pos, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float()


def _rotate(x: torch.Tensor, cs: torch.Tensor) -> torch.Tensor:
    # x [..., D] fp32, cs [..., D] (cos | sin)
    h = x.shape[-1] // 2
    c, s = cs[..., :h], cs[..., h:]
    x1, x2 = x[..., :h], x[..., h:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def rope_kv_write(qkv: torch.Tensor, cos_sin: torch.Tensor, positions: torch.Tensor, slot_mapping: torch.Tensor,
                  k_cache: torch.Tensor, v_cache: torch.Tensor, nq: int, nkv: int, D: int) -> torch.Tensor:
    T = qkv.shape[0]
    x = qkv.view(T, nq + 2 * nkv, D).float()
    cs = cos_sin[positions.long()].unsqueeze(1)
    q = _rotate(x[:, :nq], cs).to(qkv.dtype)
    k = _rotate(x[:, nq:nq + nkv], cs).to(qkv.dtype)
    v = x[:, nq + nkv:].to(qkv.dtype)
    keep = slot_mapping >= 0
    sl = slot_mapping[keep].long()
    k_cache.view(-1, nkv, D)[sl] = k[keep]
    v_cache.view(-1, nkv, D)[sl] = v[keep]
    return q.contiguous()


def decode_positions(context_lens: torch.Tensor, block_tables: torch.Tensor, block_size: int):
    pos = (context_lens - 1).clamp(min=0).long()
    blk = block_tables.long().gather(1, (pos // block_size).unsqueeze(1)).squeeze(1)
    slots = blk * block_size + pos % block_size
    slots = torch.where(context_lens > 0, slots, torch.full_like(slots, -1))
    return pos.int(), slots.int()


def _gather_kv(cache: torch.Tensor, bt_row: torch.Tensor, n: int, block_size: int, kvh: int) -> torch.Tensor:
    idx = torch.arange(n, device=cache.device)
    slots = bt_row.long()[idx // block_size] * block_size + idx % block_size
    return cache.view(-1, cache.shape[-2], cache.shape[-1])[slots, kvh].float()   # [n, D]


def paged_decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                           context_lens: torch.Tensor, scale: float, block_size: int) -> torch.Tensor:
    B, nq, D = q.shape
    nkv = k_cache.shape[-2]
    G = nq // nkv
    out = torch.zeros_like(q)
    for b in range(B):
        n = int(context_lens[b])
        if n <= 0:
            continue
        for kvh in range(nkv):
            K = _gather_kv(k_cache, block_tables[b], n, block_size, kvh)
            V = _gather_kv(v_cache, block_tables[b], n, block_size, kvh)
            qq = q[b, kvh * G:(kvh + 1) * G].float()
            p = torch.softmax(qq @ K.T * scale, dim=-1)
            out[b, kvh * G:(kvh + 1) * G] = (p @ V).to(q.dtype)
    return out


def paged_prefill_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, cu_q: torch.Tensor,
                            context_lens: torch.Tensor, block_tables: torch.Tensor, scale: float,
                            block_size: int) -> torch.Tensor:
    T, nq, D = q.shape
    nkv = k_cache.shape[-2]
    G = nq // nkv
    out = torch.zeros_like(q)
    cu = cu_q.tolist()
    for s in range(len(cu) - 1):
        q0, q1 = cu[s], cu[s + 1]
        qlen = q1 - q0
        if qlen == 0:
            continue
        ctx = int(context_lens[s])
        qpos = torch.arange(ctx - qlen, ctx, device=q.device)
        kpos = torch.arange(ctx, device=q.device)
        mask = kpos[None, :] <= qpos[:, None]
        for kvh in range(nkv):
            K = _gather_kv(k_cache, block_tables[s], ctx, block_size, kvh)
            V = _gather_kv(v_cache, block_tables[s], ctx, block_size, kvh)
            for g in range(G):
                h = kvh * G + g
                sc = (q[q0:q1, h].float() @ K.T) * scale
                sc = sc.masked_fill(~mask, float("-inf"))
                out[q0:q1, h] = (torch.softmax(sc, -1) @ V).to(q.dtype)
    return out


FP8_MAX = 448.0


def quantize_fp8(w: torch.Tensor):
    """Row-scaled OCP e4m3: returns (q [N, K] uint8 bit patterns, scale [N] fp32) with
    w ~= e4m3(q) * scale[:, None] (same recipe as fp8.hip)."""
    wf = w.float()
    amax = wf.abs().amax(dim=1)
    scale = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
    q = (wf * (1.0 / scale)[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), scale


def dequant_fp8(q: torch.Tensor, scale: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    return (q.view(torch.float8_e4m3fn).float() * scale.float()[:, None]).to(dtype)


MX_BLOCK = 32


def quantize_mx(x: torch.Tensor):
    """OCP MX e4m3 (fp8.hip quantize_act_mx_kernel): every 32 consecutive values of a row share the E8M0 scale
    e = the smallest power of two >= max|block| / 448 (byte 127 + log2; 127 for an all-zero block, clamped to
    [1, 253]).  Returns (q [M, K] uint8 e4m3 bit patterns, e [M, K / 32] uint8)."""
    M, K = x.shape
    xf = x.float().reshape(M, K // MX_BLOCK, MX_BLOCK)
    amax = xf.abs().amax(dim=-1)
    bits = (amax * (1.0 / FP8_MAX)).contiguous().view(torch.int32)
    e = (bits >> 23) + ((bits & 0x7FFFFF) != 0).to(torch.int32)
    e = torch.where(amax == 0, torch.full_like(e, 127), e).clamp(1, 253)
    inv = torch.ldexp(torch.ones_like(amax), (127 - e).float())
    q = (xf * inv[..., None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return q.view(torch.uint8).reshape(M, K), e.to(torch.uint8)


def mx_scales_to_device_layout(e: torch.Tensor) -> torch.Tensor:
    """[M, K / 32] E8M0 -> the kernels' layout [K / 128, M, 4] (csrc/kernels/common.h mx_scale_off)."""
    M, KB = e.shape
    return e.reshape(M, KB // 4, 4).permute(1, 0, 2).contiguous()


def mx_scales_from_device_layout(e: torch.Tensor) -> torch.Tensor:
    """[K / 128, M, 4] -> [M, K / 32]."""
    KT, M, _ = e.shape
    return e.permute(1, 0, 2).reshape(M, KT * 4)


def dequant_mx(q: torch.Tensor, e: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    """``e``: [M, K / 32] (logical) or the kernels' [K / 128, M, 4]."""
    if e.dim() == 3:
        e = mx_scales_from_device_layout(e)
    M, K = q.shape
    s = torch.ldexp(torch.ones(e.shape, dtype=torch.float32, device=q.device), e.float() - 127)
    v = q.view(torch.float8_e4m3fn).float().reshape(M, K // MX_BLOCK, MX_BLOCK) * s[..., None]
    return v.reshape(M, K).to(dtype)


def _wf(w) -> torch.Tensor:
    """fp32 view of a weight: a plain tensor or an ops.Fp8Weight (duck-typed: .q / .scale)."""
    if hasattr(w, "scale") and hasattr(w, "q"):
        return dequant_fp8(w.q, w.scale)
    return w.float()


def linear(x: torch.Tensor, w: torch.Tensor, out_dtype=None) -> torch.Tensor:
    y = x.float() @ _wf(w).T
    return y.to(out_dtype or x.dtype)


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    I = gu.shape[-1] // 2
    g, u = gu[..., :I].float(), gu[..., I:].float()
    return (torch.nn.functional.silu(g) * u).to(gu.dtype)


def linear_swiglu(x: torch.Tensor, w_gate_up: torch.Tensor) -> torch.Tensor:
    gu = x.float() @ _wf(w_gate_up).T
    I = gu.shape[-1] // 2
    return (torch.nn.functional.silu(gu[..., :I]) * gu[..., I:]).to(x.dtype)


def embedding(ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    return table[ids.long().clamp(0, table.shape[0] - 1)]


def _ord_key(l: torch.Tensor) -> torch.Tensor:
    u = l.float().contiguous().view(torch.int32).to(torch.int64) & U32
    neg = (u & 0x80000000) != 0
    return torch.where(neg, (~u) & U32, u | 0x80000000)


NUC_FS = float(np.float32(65536.0 / 28.0))   # sampler.hip NUC_FS


def nucleus_fine_mass(l: torch.Tensor, M: float, T: float):
    """Per token of an fp32 logits row: fine bin f = floor((M - l) / T * 65536/28) (65536 = none beyond 28) and the
    integer mass floor(exp((l - M) / T) * 2^40) (0 for none), as sampler.hip computes them for row max M."""
    l = l.float().cpu()
    invT = torch.tensor(1.0, dtype=torch.float32) / torch.tensor(T, dtype=torch.float32)
    M = torch.tensor(M, dtype=torch.float32)
    x = ((M - l) * invT) * torch.tensor(NUC_FS, dtype=torch.float32)
    valid = x < 65536.0
    f = torch.where(valid, x, torch.zeros_like(x)).to(torch.int64)
    f = torch.where(valid, f, torch.full_like(f, 65536))
    mass = (torch.exp((l - M) * invT) * 1099511627776.0).to(torch.int64)
    return f, torch.where(valid, mass, torch.zeros_like(mass))


def nucleus_coarse_hist(f: torch.Tensor, mass: torch.Tensor) -> torch.Tensor:
    return torch.zeros(257, dtype=torch.int64).index_add_(0, torch.clamp(f >> 8, max=256), mass)[:256]


def nucleus_fine_hist(f: torch.Tensor, mass: torch.Tensor, bstar: int) -> torch.Tensor:
    inb = (f >> 8) == bstar
    return torch.zeros(256, dtype=torch.int64).index_add_(0, (f & 255)[inb], mass[inb])


def nucleus_pick(hist: torch.Tensor, target: int, above: int = 0):
    """(first bin where above + the cumulative mass reaches target -- 255 if none --, mass before that bin)."""
    cum = above + torch.cumsum(hist, 0)
    hit = ((cum >= target) & (hist != 0)).nonzero()
    b = int(hit[0]) if len(hit) else 255
    return b, int(cum[b] - hist[b])


def nucleus_target(coarse: torch.Tensor, P: float) -> int:
    return int(float(int(coarse.sum())) * float(np.float32(P)))


def nucleus_mask(l: torch.Tensor, T: float, P: float) -> torch.Tensor:
    """The nucleus of sampler.hip for one row of fp32 logits: fine bin f = floor((M - l) / T * 65536/28)
    (none beyond 28), mass = floor(exp((l - M) / T) * 2^40) as an integer, target = floor(Z * P); the
    smallest f* with mass{f <= f*} >= target is found coarse (f >> 8) then fine (f & 255); keep f <= f*."""
    l = l.float().cpu()
    f, mass = nucleus_fine_mass(l, float(l.max()), T)
    coarse = nucleus_coarse_hist(f, mass)
    target = nucleus_target(coarse, P)
    bstar, above = nucleus_pick(coarse, target)
    fstar = bstar * 256 + nucleus_pick(nucleus_fine_hist(f, mass, bstar), target, above)[0]
    return f <= fstar


def sample_key(l: torch.Tensor, T: float, seed: int, ctr: int, id0: int, keep=None):
    """(score, global id) of the best token of one logits row whose token ids start at ``id0`` (a vocab shard):
    greedy (T <= 0) or Gumbel-max over ``keep``; ties to the lowest id, like sampler.hip's packed keys.  None if
    ``keep`` leaves no token."""
    l = l.float()
    vid = torch.arange(l.numel(), dtype=torch.int64, device=l.device) + id0
    if T <= 0:
        score = l
    else:
        u = u01(hash3(int(seed), int(ctr), vid)).float()
        score = l / T - torch.log(-torch.log(u))
    if keep is not None:
        score = torch.where(keep.to(score.device), score, torch.full_like(score, float("-inf")))
        if not bool(keep.any()):
            return None
    m = score.max()
    i = int((score == m).nonzero()[0])
    return float(m), int(vid[i])


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, seeds: torch.Tensor,
           counter: torch.Tensor) -> torch.Tensor:
    """logits [B, V] fp32 -> tokens [B] int32, bit-compatible with sampler.hip (up to fp rounding
    of the Gumbel scores and of the per-token masses at a nucleus boundary)."""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int32, device=logits.device)
    for b in range(B):
        l = logits[b].float()
        T, P = float(temperature[b]), float(top_p[b])
        keep = nucleus_mask(l, T, P) if T > 0 and P < 1.0 else None
        out[b] = sample_key(l, T, int(seeds[b]), int(counter[b]), 0, keep)[1]
    return out


def sample_vocab_parallel(local: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, seeds: torch.Tensor,
                          counter: torch.Tensor, rank: int, gather) -> torch.Tensor:
    """Vocab-parallel form of :func:`sample` (sampler.hip's TP path, on CPU): ``local`` [B, Vs] is this rank's vocab
    shard (global ids rank * Vs ..), ``gather(t)`` all-gathers a tensor over the ranks ([world, *t.shape]).  Nucleus
    rows combine the row max and the two integer bin histograms over the ranks, then every rank's best (score, id)
    is gathered and the best of them taken: the tokens of :func:`sample` over the concatenated shards."""
    B, Vs = local.shape
    id0 = rank * Vs
    nuc = [float(temperature[b]) > 0 and float(top_p[b]) < 1.0 for b in range(B)]
    keep = [None] * B
    if any(nuc):
        M = gather(local.float().max(dim=1).values).max(dim=0).values
        fm = [nucleus_fine_mass(local[b], float(M[b]), float(temperature[b])) if nuc[b] else None for b in range(B)]
        z = torch.zeros(256, dtype=torch.int64)
        coarse = gather(torch.stack([nucleus_coarse_hist(*fm[b]) if nuc[b] else z for b in range(B)])).sum(0)
        sel = {}
        for b in range(B):
            if nuc[b]:
                target = nucleus_target(coarse[b], float(top_p[b]))
                sel[b] = (target,) + nucleus_pick(coarse[b], target)
        fine = gather(torch.stack([nucleus_fine_hist(*fm[b], sel[b][1]) if nuc[b] else z for b in range(B)])).sum(0)
        for b in range(B):
            if nuc[b]:
                target, bstar, above = sel[b]
                keep[b] = fm[b][0] <= bstar * 256 + nucleus_pick(fine[b], target, above)[0]
    best = torch.full((B, 2), float("-inf"), dtype=torch.float64)
    for b in range(B):
        k = sample_key(local[b], float(temperature[b]), int(seeds[b]), int(counter[b]), id0, keep[b])
        if k is not None:
            best[b, 0], best[b, 1] = k[0], -k[1]
    g = gather(best)                                  # [world, B, 2]: (score, -id); max = best score, lowest id
    out = torch.empty(B, dtype=torch.int32)
    for b in range(B):
        cand = [tuple(g[r, b].tolist()) for r in range(g.shape[0])]
        out[b] = int(-max(cand)[1])
    return out


# ----------------------------------------------------------------------------- device-side stop detection (oracle)
def token_stop_classes(texts, eos_ids, vocab: int) -> torch.Tensor:
    """Per-token class words of sampler.hip's stop detection, [vocab, 2] int32, from each token's decoded text
    (``texts[i]`` for token i; missing / special tokens: no braces).  x = eos | net brace delta << 8 | min running
    depth relative to the entry << 16; y = has '{' | depth at the end counted from the token's first '{' << 8 |
    min depth after that '{' << 16 (int8 fields)."""
    def i8(v: int) -> int:
        return max(-128, min(127, v)) & 0xFF

    out = torch.zeros(vocab, 2, dtype=torch.int32)
    xs, ys = [0] * vocab, [0] * vocab
    for i, t in enumerate(texts[:vocab]):
        if not t or ("{" not in t and "}" not in t):
            continue
        d = m = 0
        for ch in t:
            if ch == "{":
                d += 1
            elif ch == "}":
                d -= 1
                m = min(m, d)
        xs[i] = (i8(d) << 8) | (i8(m) << 16)
        k = t.find("{")
        if k >= 0:
            d2, m2 = 1, 1
            for ch in t[k + 1:]:
                if ch == "{":
                    d2 += 1
                elif ch == "}":
                    d2 -= 1
                    m2 = min(m2, d2)
            ys[i] = 1 | (i8(d2) << 8) | (i8(m2) << 16)
    for e in eos_ids:
        if 0 <= e < vocab:
            xs[e] |= 1
    out[:, 0] = torch.tensor(xs, dtype=torch.int64).to(torch.int32)
    out[:, 1] = torch.tensor(ys, dtype=torch.int64).to(torch.int32)
    return out


def _i8(v: int) -> int:
    v &= 0xFF
    return v - 256 if v >= 128 else v


def json_step(state: int, cx: int, cy: int):
    """(new state, closed) -- sampler.hip json_step."""
    if state >= 1:
        amin, adelta = _i8(cx >> 16), _i8(cx >> 8)
        if state + amin <= 0:
            return 0, True
        return state + adelta, False
    if cy & 1:
        bmin, bend = _i8(cy >> 16), _i8(cy >> 8)
        if bmin <= 0:
            return 0, True
        return bend, False
    return state, False


def write_token_stop(s: int, tok: int, tokens, ctx_inc, hist, steps, stop) -> None:
    """sampler.hip write_token with stop detection, for state slot s (CPU reference of the decode graphs)."""
    st = int(steps[s])
    fin = False
    cls, cfg = stop["cls"], int(stop["cfg"][s])
    max_new = cfg >> 8
    state = int(stop["json"][s])
    if state == -2:
        t0 = int(hist[s, 0])
        state = -1
        if (cfg & 1) and (int(cls[t0, 0]) & 1):
            fin = True
        elif cfg & 2:
            state, fin = json_step(state, int(cls[t0, 0]), int(cls[t0, 1]))
        if not fin and st >= max_new:
            fin = True
        if fin:
            stop["json"][s] = state
            ctx_inc[s] = 0
            stop["done"][s] = 1
            return
    forced, flen = stop.get("forced"), stop.get("forced_len")
    if forced is not None and int(flen[s]) >= 0:
        tok = int(forced[s, st]) if st < int(flen[s]) else int(stop["eos_tok"])
    cx, cy = int(cls[tok, 0]), int(cls[tok, 1])
    if (cfg & 1) and (cx & 1):
        fin = True
    else:
        if cfg & 2:
            state, fin = json_step(state, cx, cy)
        if st + 1 >= max_new:
            fin = True
    stop["json"][s] = state
    tokens[s] = tok
    if st < hist.shape[1]:
        hist[s, st] = tok
    steps[s] = st + 1
    ctx_inc[s] = 0 if fin else int(ctx_inc[s]) + 1
    if fin:
        stop["done"][s] = 1
