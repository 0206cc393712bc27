"""K16 block-scaled activations (OCP MX e4m3, one E8M0 scale per 32 values): the stand-alone quantizer against the
CPU reference bit for bit, mgemm's MX mode (block-scaled 16x16x128 MFMA, the scales as its B scale operand) against
the fp32 oracle of the dequantized operands for every configuration built for it, and the SwiGLU epilogue's MX output
against quantizing the same GEMM's bf16 output (bit for bit)."""

import pytest
import torch

from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _act(M, K, seed, spread=True):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(M, K, generator=g)
    if spread:   # block magnitudes over 2^-8 .. 2^8, some all-zero blocks, one huge value
        x = x * torch.pow(2.0, torch.randint(-8, 9, (M, K // 32), generator=g).float()).repeat_interleave(32, 1)
        x[0, :32] = 0
        x[-1, 5] = 3.0e4
    return x.to(torch.bfloat16)


def _weights(rows, K, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return ops.quantize_fp8(((torch.rand(rows, K, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16).to(DEV))


@pytest.mark.parametrize("M,K", [(1, 128), (17, 256), (64, 8192), (130, 3584), (7, 28672)])
def test_quantize_act_mx_matches_reference_bit_for_bit(M, K):
    x = _act(M, K, M + K)
    a = ops.quantize_act_mx(x.to(DEV))
    q, e = ref.quantize_mx(x)
    assert torch.equal(a.blocks().cpu(), e)
    assert torch.equal(a.q.cpu(), q)
    back = a.dequant(torch.float32).cpu()
    blk = torch.ldexp(torch.ones(e.shape), e.float() - 127).repeat_interleave(32, 1)   # the block scales
    err = (back - x.float()).abs()
    assert bool((err <= 16 * blk).all())             # half an e4m3 ulp of the top binade (32), scaled
    normal = x.float().abs() >= 2 ** -6 * blk          # e4m3 normal range: relative error <= 2^-4
    assert bool((err[normal] <= 2 ** -4 * x.float().abs()[normal] + 1e-30).all())


def _mx_oracle(act, w, epi):
    xr = ref.dequant_mx(act.q.cpu(), act.e.cpu(), torch.float32)
    y = xr @ ref.dequant_fp8(w.q.cpu(), w.scale.cpu(), torch.float32).t()
    if epi == ops.EPI_SWIGLU:
        n = y.shape[1] // 2
        y = torch.nn.functional.silu(y[:, :n]) * y[:, n:]
    return y


@pytest.mark.parametrize("epi", [ops.EPI_BF16, ops.EPI_F32, ops.EPI_SWIGLU])
def test_mgemm_mx_every_config(epi):
    """MX activations x row-scaled e4m3 weights on every configuration built for the mode, one-workgroup-per-tile /
    split-K / stream-K grids, partial M tiles, the residual epilogue."""
    K, N = 1024, 192
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, 11)
    n_cfg = 0
    for cfg, (bm, *_rest) in enumerate(ops.mgemm_configs()):
        if not ops.mgemm_valid(cfg, 64, N, K, epi, 3):
            continue
        n_cfg += 1
        for M in (17, bm + 7):
            act = ops.quantize_act_mx(_act(M, K, cfg * 100 + M, spread=False).to(DEV))
            exp = _mx_oracle(act, w, epi)
            for grid in (1, 4, -7, -256):
                if not ops.mgemm_valid(cfg, M, N, K, epi, 3, grid):
                    continue
                y = ops.mgemm(act, w, epi, cfg=cfg, grid=grid).float().cpu()
                err = (y - exp).abs().max().item()
                assert err <= 1e-2 * exp.abs().max().item(), f"cfg {cfg} grid {grid} M {M}: {err}"
                if epi == ops.EPI_BF16:
                    res = ((torch.rand(M, N, device=DEV) * 2 - 1) * 8).to(torch.bfloat16)
                    want = exp + res.float().cpu()
                    out = ops.mgemm(act, w, epi, cfg=cfg, grid=grid, res=res, out=res)
                    err = (out.float().cpu() - want).abs().max().item()
                    assert err <= 1e-2 * want.abs().max().item(), f"res cfg {cfg} grid {grid} M {M}: {err}"
    assert n_cfg >= 6


@pytest.mark.parametrize("act_mx", [False, True])
def test_mgemm_swiglu_mx_output_is_the_quantized_bf16_output(act_mx):
    """The SwiGLU epilogue's MX output equals quantize_act_mx of the bf16 output of the same launch plan, bit for
    bit (same accumulation, the bf16 value is what gets quantized), for per-token and MX activations."""
    K, N = 1024, 256
    w = _weights(2 * N, K, 5)
    n_cfg = 0
    for cfg in range(len(ops.mgemm_configs())):
        mode = 3 if act_mx else 1
        if not ops.mgemm_valid(cfg, 64, N, K, ops.EPI_SWIGLU, mode, 1, mx_out=True):
            continue
        n_cfg += 1
        for M in (19, 64):
            x = _act(M, K, cfg + M, spread=False).to(DEV)
            act = ops.quantize_act_mx(x) if act_mx else ops.quantize_act_fp8(x)
            for grid in (1, 4, -256):
                if not ops.mgemm_valid(cfg, M, N, K, ops.EPI_SWIGLU, mode, grid, mx_out=True):
                    continue
                y = ops.mgemm(x, w, ops.EPI_SWIGLU, cfg=cfg, grid=grid, act=act)
                mx = ops.mgemm(x, w, ops.EPI_SWIGLU, cfg=cfg, grid=grid, act=act, mx_out=True)
                q, e = ref.quantize_mx(y.cpu())
                assert torch.equal(mx.blocks().cpu(), e), f"cfg {cfg} grid {grid} M {M}"
                assert torch.equal(mx.q.cpu(), q), f"cfg {cfg} grid {grid} M {M}"
    assert n_cfg >= 2


@pytest.mark.parametrize("epi", [ops.EPI_BF16, ops.EPI_F32, ops.EPI_SWIGLU])
def test_pgemm_mx_every_config(epi):
    """pgemm's MX mode (prefill rows): every tile configuration, without and with split-K (row slabs + the reduce
    kernel, and the in-launch last-arriver form), partial tiles, the residual epilogue, against the fp32 oracle."""
    K, N = 1024, 320
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, 13)
    keep = ops.native().pgemm_set_row_slabs(-1)
    try:
        for cfg in range(len(ops.pgemm_configs())):
            for M in (200, 300):
                act = ops.quantize_act_mx(_act(M, K, cfg * 10 + M, spread=False).to(DEV))
                exp = _mx_oracle(act, w, epi)
                for splits, slabs in ((1, 1), (3, 1), (3, 0)):
                    ops.native().pgemm_set_row_slabs(slabs)
                    y = ops.pgemm(act, w, epi, cfg=cfg, splits=splits).float().cpu()
                    err = (y - exp).abs().max().item()
                    assert err <= 1e-2 * exp.abs().max().item(), f"cfg {cfg} splits {splits}/{slabs} M {M}: {err}"
                    if epi == ops.EPI_BF16:
                        res = ((torch.rand(M, N, device=DEV) * 2 - 1) * 8).to(torch.bfloat16)
                        want = exp + res.float().cpu()
                        out = ops.pgemm(act, w, epi, cfg=cfg, splits=splits, res=res, out=res)
                        err = (out.float().cpu() - want).abs().max().item()
                        assert err <= 1e-2 * want.abs().max().item(), f"res cfg {cfg} splits {splits} M {M}: {err}"
    finally:
        ops.native().pgemm_set_row_slabs(keep)


@pytest.mark.parametrize("act_mx", [False, True])
def test_pgemm_swiglu_mx_output_is_the_quantized_bf16_output(act_mx):
    K, N = 1024, 256
    w = _weights(2 * N, K, 17)
    keep = ops.native().pgemm_set_row_slabs(-1)
    try:
        for cfg in range(len(ops.pgemm_configs())):
            M = 300
            x = _act(M, K, cfg, spread=False).to(DEV)
            act = ops.quantize_act_mx(x) if act_mx else ops.quantize_act_fp8(x)
            for splits, slabs in ((1, 1), (3, 1), (3, 0)):
                ops.native().pgemm_set_row_slabs(slabs)
                y = ops.pgemm(x, w, ops.EPI_SWIGLU, cfg=cfg, splits=splits, act=act)
                mx = ops.pgemm(x, w, ops.EPI_SWIGLU, cfg=cfg, splits=splits, act=act, mx_out=True)
                q, e = ref.quantize_mx(y.cpu())
                assert torch.equal(mx.blocks().cpu(), e), f"cfg {cfg} splits {splits}/{slabs}"
                assert torch.equal(mx.q.cpu(), q), f"cfg {cfg} splits {splits}/{slabs}"
    finally:
        ops.native().pgemm_set_row_slabs(keep)


@pytest.mark.parametrize("B,ctx,part", [(24, 300, 1024), (64, 1500, 1024), (40, 700, 512)])
def test_decode_attention_mx_output_is_the_quantized_bf16_output(B, ctx, part, monkeypatch):
    """The one-workgroup decode attention (and its partition merge, ctx > part) writes the O projection's input as
    MX e4m3: bit for bit quantize_act_mx of its bf16 output."""
    from k8s_llm_scheduler_amd.models.config import PRESETS
    from k8s_llm_scheduler_amd.models.llama import LlamaModel
    monkeypatch.setattr(ops, "FUSED_PART_ENV", part)
    monkeypatch.setattr(ops, "SPLIT_MAX_PAIRS", 0)   # the one-workgroup kernel
    m = LlamaModel(PRESETS["tiny"], device="cuda", seed=1, max_model_len=2048)
    nb = (ctx + 15) // 16 + 1
    m.allocate_kv(B * nb + 1, 16)
    kc, vc = m.kv_cache[0, 0], m.kv_cache[0, 1]
    kc.normal_()
    vc.normal_()
    g = torch.Generator(device="cpu").manual_seed(B)
    qkv = (torch.randn(B, (m.nq + 2 * m.nkv) * m.D, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    ctxs = torch.tensor([max(1, ctx - 7 * i) for i in range(B)], dtype=torch.int32, device=DEV)
    bt = torch.arange(B * nb, dtype=torch.int32, device=DEV).view(B, nb)
    args = (qkv, m.cos_sin, kc, vc, bt, ctxs, m.scale, 16, ctx, m.nq, m.nkv, m.D)
    y = ops.decode_attention_fused(*args)
    mx = ops.decode_attention_fused(*args, mx=True)
    assert isinstance(mx, ops.MxAct)
    q, e = ref.quantize_mx(y.cpu())
    assert torch.equal(mx.blocks().cpu(), e)
    assert torch.equal(mx.q.cpu(), q)


def test_mgemm_residual_mx_copy_and_mx_rms_prologue():
    """The residual epilogue's MX copy equals quantize_act_mx of the bf16 residual stream it wrote (bit for bit),
    and an MX-mode GEMM with the RMS prologue matches the oracle on the dequantized rows (RMS of the dequantized
    values), with bf16 and SwiGLU (+ MX output) epilogues."""
    K, N, eps = 1024, 256, 1e-5
    wo = _weights(N, K, 21)
    n_cfg = 0
    for cfg in range(len(ops.mgemm_configs())):
        if not ops.mgemm_valid(cfg, 64, N, K, ops.EPI_BF16, 3, 1, mx_out=True):
            continue
        n_cfg += 1
        for M in (19, 64):
            act = ops.quantize_act_mx(_act(M, K, cfg + 3 * M, spread=False).to(DEV))
            for grid in (1, 4, -256):
                if not ops.mgemm_valid(cfg, M, N, K, ops.EPI_BF16, 3, grid, mx_out=True):
                    continue
                res = ((torch.rand(M, N, device=DEV) * 2 - 1) * 8).to(torch.bfloat16)
                want = ops.mgemm(act, wo, ops.EPI_BF16, cfg=cfg, grid=grid, res=res.clone(), out=None)
                out, mx = ops.mgemm(act, wo, ops.EPI_BF16, cfg=cfg, grid=grid, res=res.clone(), out=None,
                                    mx_out=True)
                # (the two epilogues may contract acc * scale + res differently: 1 bf16 ulp at most)
                torch.testing.assert_close(out.float(), want.float(), rtol=2 ** -7, atol=1e-6)
                q, e = ref.quantize_mx(out.cpu())
                assert torch.equal(mx.blocks().cpu(), e) and torch.equal(mx.q.cpu(), q), f"cfg {cfg} grid {grid}"
    assert n_cfg >= 4
    # MX rows + RMS prologue
    M = 48
    x = (_act(M, K, 5, spread=False).float() * 3).to(torch.bfloat16).to(DEV)
    act = ops.quantize_act_mx(x)
    xa = ref.dequant_mx(act.q.cpu(), act.e.cpu())
    inv = torch.rsqrt(xa.pow(2).mean(-1, keepdim=True) + eps)
    wq = _weights(N, K, 23)
    gu = _weights(2 * N, K, 24)
    n_cfg = 0
    for cfg in range(len(ops.mgemm_configs())):
        if not ops.mgemm_valid(cfg, M, N, K, ops.EPI_BF16, 3):
            continue
        n_cfg += 1
        y = ops.mgemm(act, wq, ops.EPI_BF16, cfg=cfg, grid=1, rms_eps=eps).float().cpu()
        exp = (xa * inv) @ ref.dequant_fp8(wq.q.cpu(), wq.scale.cpu()).t()
        assert (y - exp).abs().max().item() <= 1e-2 * exp.abs().max().item(), f"rms cfg {cfg}"
        if ops.mgemm_valid(cfg, M, N, K, ops.EPI_SWIGLU, 3, 1, mx_out=True):
            ys = ops.mgemm(act, gu, ops.EPI_SWIGLU, cfg=cfg, grid=1, rms_eps=eps)
            mx = ops.mgemm(act, gu, ops.EPI_SWIGLU, cfg=cfg, grid=1, rms_eps=eps, mx_out=True)
            q, e = ref.quantize_mx(ys.cpu())
            assert torch.equal(mx.blocks().cpu(), e) and torch.equal(mx.q.cpu(), q), f"rms swiglu cfg {cfg}"
            expg = (xa * inv) @ ref.dequant_fp8(gu.q.cpu(), gu.scale.cpu()).t()
            expg = torch.nn.functional.silu(expg[:, :N]) * expg[:, N:]
            assert (ys.float().cpu() - expg).abs().max().item() <= 1e-2 * expg.abs().max().item(), f"swiglu {cfg}"
    assert n_cfg >= 6


def test_embedding_mx_copy_is_the_quantized_rows():
    g = torch.Generator(device="cpu").manual_seed(9)
    table = (torch.randn(1000, 1024, generator=g) * 0.3).to(torch.bfloat16).to(DEV)
    ids = torch.randint(0, 1000, (37,), generator=g, dtype=torch.int32).to(DEV)
    out, mx = ops.embedding(ids, table, mx=True)
    assert torch.equal(out, ops.embedding(ids, table))
    q, e = ref.quantize_mx(out.cpu())
    assert torch.equal(mx.blocks().cpu(), e) and torch.equal(mx.q.cpu(), q)


@pytest.mark.parametrize("N", [4096, 8192])
def test_mgemm_bf16_rms_prologue_both_forms(N):
    """The bf16 RMS prologue: v_dot2 squares below 8192 output features, the x . x^T MFMA diagonal from 8192 on
    (mgemm.hip rms_mfma) -- every configuration against the fp32 oracle."""
    K, eps = 1024, 1e-5
    g = torch.Generator(device="cpu").manual_seed(N)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16).to(DEV)
    n_cfg = 0
    for cfg in range(len(ops.mgemm_configs())):
        if not ops.mgemm_valid(cfg, 64, N, K, ops.EPI_BF16, 0):
            continue
        n_cfg += 1
        for M in (24, 64):
            r = (torch.randn(M, K, generator=g) * 3).to(torch.bfloat16).to(DEV)
            y = ops.mgemm(r, w, ops.EPI_BF16, cfg=cfg, grid=1, rms_eps=eps).float().cpu()
            rf = r.float().cpu()
            exp = (rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + eps)) @ w.float().cpu().t()
            assert (y - exp).abs().max().item() <= 1e-2 * exp.abs().max().item(), f"cfg {cfg} M {M}"
    assert n_cfg >= 6
