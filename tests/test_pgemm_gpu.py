"""pgemm.hip (big-tile MFMA GEMM for prefill-size row counts) against the fp32 PyTorch oracle: every tile
configuration x epilogue (bf16 / fp32 / SwiGLU / residual) x weight dtype (bf16 / row-scaled e4m3 on the
f8f6f4 MFMA) x split-K, partial tiles in M and N, the RMS prologue, exact small-integer data (fragment layout
and k-permutation errors show as exact mismatches), and the Llama-3.3-70B prefill shapes."""

import pytest
import torch

from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _oracle(x, w, epi):
    """fp32 oracle, computed on the operands' device (fp32 GEMM, no reduced-precision path on gfx950)."""
    if ops._is_fp8(w):
        xq, sx = ref.quantize_fp8(x)
        xr = ref.dequant_fp8(xq, sx, torch.float32)
        wr = ref.dequant_fp8(w.q, w.scale, torch.float32)
    else:
        xr, wr = x.float(), w.float()
    y = xr @ wr.t()
    if epi == ops.EPI_SWIGLU:
        n = wr.shape[0] // 2
        y = torch.nn.functional.silu(y[:, :n]) * y[:, n:]
    return y


def _check(y, x, w, epi, tol=2e-2, what=""):
    exp = _oracle(x, w, epi)
    got = y.float()
    assert got.shape == exp.shape
    err = (got - exp).abs().max().item()
    scale = exp.abs().max().item() + 1e-6
    assert err <= tol * scale, f"{what}: max err {err:.4g} vs scale {scale:.4g}"


def _weights(rows, K, fp8, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    w = (torch.rand(rows, K, generator=g, device=DEV) * 2 - 1).to(torch.bfloat16)
    return ops.quantize_fp8(w) if fp8 else w


def test_exact_small_integers_every_config():
    """Integer operands with an asymmetric weight matrix: bf16 products and fp32 sums are exact, so any
    fragment-layout, swizzle or k-permutation error is an exact mismatch, not a tolerance miss."""
    K = 512
    for cfg, (bp, bq, _lds) in enumerate(ops.pgemm_configs()):
        M, N = bq + 40, bp + 36
        x = torch.randint(-3, 4, (M, K), device=DEV).to(torch.bfloat16)
        w = (torch.arange(N * K, device=DEV).view(N, K) % 7 - 3).to(torch.bfloat16)
        w[:, 5] += torch.arange(N, device=DEV).to(torch.bfloat16) % 5   # break row symmetry
        exp = x.float() @ w.float().t()
        for splits in (1, 3):
            y = ops.pgemm(x, w, ops.EPI_F32, cfg=cfg, splits=splits)
            torch.cuda.synchronize()
            assert torch.equal(y, exp), f"cfg {cfg} splits {splits}: {(y - exp).abs().max().item()}"


def test_exact_short_k_every_ring_depth():
    """1-5 k-tiles per slice: fewer k-tiles than weight-ring stages (configs 4-7 keep 3-4 weight stages), so the
    prologue, the tail waits and the ring slots all run their short-loop paths; exact integer data."""
    for cfg, (bp, bq, _lds) in enumerate(ops.pgemm_configs()):
        M, N = bq + 8, bp + 20
        for K in (64, 192, 320):
            x = torch.randint(-3, 4, (M, K), device=DEV).to(torch.bfloat16)
            w = (torch.arange(N * K, device=DEV).view(N, K) % 5 - 2).to(torch.bfloat16)
            w[:, 3] += torch.arange(N, device=DEV).to(torch.bfloat16) % 3
            exp = x.float() @ w.float().t()
            for splits in (1, 2):
                if splits > K * 2 // 128:
                    continue
                y = ops.pgemm(x, w, ops.EPI_F32, cfg=cfg, splits=splits)
                torch.cuda.synchronize()
                assert torch.equal(y, exp), f"cfg {cfg} K {K} splits {splits}: {(y - exp).abs().max().item()}"


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("epi", [ops.EPI_BF16, ops.EPI_F32, ops.EPI_SWIGLU])
def test_every_config(epi, fp8):
    torch.manual_seed(0)
    K = 1024
    N = 200  # partial n tiles
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, fp8, 1)
    for cfg, (bp, bq, _lds) in enumerate(ops.pgemm_configs()):
        for M in (13, bq + 7):
            x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
            for splits in (1, 2, 5):
                for gm in (1, 4):
                    y = ops.pgemm(x, w, epi, cfg=cfg, splits=splits, group_m=gm)
                    torch.cuda.synchronize()
                    _check(y, x, w, epi, what=f"cfg {cfg} M {M} splits {splits} gm {gm}")


@pytest.mark.parametrize("epi", [ops.EPI_BF16, ops.EPI_SWIGLU, ops.EPI_F32])
def test_rms_prologue_and_residual_epilogue(epi):
    torch.manual_seed(1)
    K, N, eps = 1024, 200, 1e-5
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, False, 5)
    for cfg, (bp, bq, _lds) in enumerate(ops.pgemm_configs()):
        for M in (13, bq + 7):
            r = ((torch.rand(M, K, device=DEV) * 2 - 1) * 3).to(torch.bfloat16)
            rf = r.float().cpu()
            xn = rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + eps)
            exp = xn @ w.float().cpu().t()
            if epi == ops.EPI_SWIGLU:
                exp = torch.nn.functional.silu(exp[:, :N]) * exp[:, N:]
            for splits in (1, 4):
                y = ops.pgemm(r, w, epi, cfg=cfg, splits=splits, rms_eps=eps).float().cpu()
                err = (y - exp).abs().max().item()
                assert err <= 2e-2 * exp.abs().max().item(), f"rms cfg {cfg} splits {splits} M {M}: {err}"
                if epi == ops.EPI_BF16:
                    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
                    res = ((torch.rand(M, N, device=DEV) * 2 - 1) * 8).to(torch.bfloat16)
                    want = (x.float() @ w.float().t() + res.float()).cpu()
                    out = ops.pgemm(x, w, epi, cfg=cfg, splits=splits, res=res, out=res)   # in place
                    assert out.data_ptr() == res.data_ptr()
                    err = (out.float().cpu() - want).abs().max().item()
                    assert err <= 2e-2 * want.abs().max().item(), f"res cfg {cfg} splits {splits} M {M}: {err}"


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("epi", [ops.EPI_BF16, ops.EPI_F32, ops.EPI_SWIGLU])
def test_row_slab_reduce_is_bit_identical_to_last_arriver(epi, fp8):
    """Split-K combine by the separate reduce kernel (row-major slabs) against the in-launch last-arriver
    reduction: same slice order, same epilogue arithmetic -> the same bits (RMS prologue, residual, fp8 scales)."""
    torch.manual_seed(2)
    K, N, eps = 2048, 200, 1e-5
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, fp8, 7)
    old = ops.native().pgemm_set_row_slabs(0)
    try:
        for cfg, (bp, bq, _lds) in enumerate(ops.pgemm_configs()):
            for M in (13, bq + 7):
                x = ((torch.rand(M, K, device=DEV) * 2 - 1) * 3).to(torch.bfloat16)
                res = ((torch.rand(M, N, device=DEV) * 2 - 1) * 8).to(torch.bfloat16) \
                    if epi == ops.EPI_BF16 else None
                rms = None if fp8 else eps
                for splits in (2, 5):
                    got = []
                    for mode in (0, 1):
                        ops.native().pgemm_set_row_slabs(mode)
                        r = None if res is None else res.clone()
                        got.append(ops.pgemm(x, w, epi, cfg=cfg, splits=splits, rms_eps=rms, res=r))
                    torch.cuda.synchronize()
                    assert torch.equal(got[0], got[1]), f"cfg {cfg} M {M} splits {splits}"
                    if rms is None and res is None:
                        _check(got[1], x, w, epi, what=f"row slabs cfg {cfg} M {M} splits {splits}")
    finally:
        ops.native().pgemm_set_row_slabs(old)


def test_split_k_tickets_reset_and_graph_replay():
    K, N, M = 4096, 512, 300
    w = _weights(N, K, False, 3)
    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    exp = ops.pgemm(x, w, ops.EPI_F32, cfg=0, splits=8)
    for _ in range(4):
        assert torch.equal(ops.pgemm(x, w, ops.EPI_F32, cfg=0, splits=8), exp)   # fixed slab order: bit-exact
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.pgemm(x, w, ops.EPI_F32, cfg=0, splits=8)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g, stream=s):
        yg = ops.pgemm(x, w, ops.EPI_F32, cfg=0, splits=8)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(yg, exp)
    _check(exp, x, w, ops.EPI_F32, tol=1e-3)


@pytest.mark.parametrize("name,N,K,epi", [
    ("qkv", 10240, 8192, ops.EPI_BF16),
    ("o_proj", 8192, 8192, ops.EPI_BF16),
    ("gate_up", 28672, 8192, ops.EPI_SWIGLU),
    ("down", 8192, 28672, ops.EPI_BF16),
    ("lm_head", 128256, 8192, ops.EPI_F32),
])
@pytest.mark.parametrize("fp8", [False, True])
def test_tp1_prefill_shapes(name, N, K, epi, fp8):
    """Llama-3.3-70B TP=1 projections at a 245-token prefill (the headline decision) through the planner."""
    M = 245
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, fp8, 7)
    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    for cfg, splits in ((0, 1), (0, 4), (2, 2)):
        y = ops.pgemm(x, w, epi, cfg=cfg, splits=splits)
        torch.cuda.synchronize()
        _check(y, x, w, epi, what=f"{name} cfg {cfg} splits {splits}")


# ----------------------------------------------------------------------------- pgemm4.hip (4-wave big tiles, bf16)
def test_pgemm4_exact_small_integers_every_config():
    K = 512
    for cfg, (bp, bq, _lds) in enumerate(ops.pgemm4_configs()):
        M, N = bq + 40, bp + 36
        x = torch.randint(-3, 4, (M, K), device=DEV).to(torch.bfloat16)
        w = (torch.arange(N * K, device=DEV).view(N, K) % 7 - 3).to(torch.bfloat16)
        w[:, 5] += torch.arange(N, device=DEV).to(torch.bfloat16) % 5
        exp = x.float() @ w.float().t()
        for splits in (1, 3):
            y = ops.pgemm4(x, w, ops.EPI_F32, cfg=cfg, splits=splits)
            torch.cuda.synchronize()
            assert torch.equal(y, exp), f"cfg {cfg} splits {splits}: {(y - exp).abs().max().item()}"


def test_pgemm4_exact_short_k_every_config():
    """1-4 k-steps of 64 per slice: the 64-deep-stage configuration's prologue-only, one-loop-iteration and tail paths
    (and the 32-deep ones' short loops); exact integer data."""
    for cfg, (bp, bq, _lds) in enumerate(ops.pgemm4_configs()):
        M, N = bq + 8, bp + 20
        for K in (64, 128, 256):
            x = torch.randint(-3, 4, (M, K), device=DEV).to(torch.bfloat16)
            w = (torch.arange(N * K, device=DEV).view(N, K) % 5 - 2).to(torch.bfloat16)
            w[:, 3] += torch.arange(N, device=DEV).to(torch.bfloat16) % 3
            exp = x.float() @ w.float().t()
            for splits in (1, 2):
                if splits > K // 64:
                    continue
                y = ops.pgemm4(x, w, ops.EPI_F32, cfg=cfg, splits=splits)
                torch.cuda.synchronize()
                assert torch.equal(y, exp), f"cfg {cfg} K {K} splits {splits}: {(y - exp).abs().max().item()}"


@pytest.mark.parametrize("epi", [ops.EPI_BF16, ops.EPI_F32, ops.EPI_SWIGLU])
def test_pgemm4_every_config(epi):
    torch.manual_seed(0)
    K, N = 1024, 200
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, False, 1)
    for cfg, (bp, bq, _lds) in enumerate(ops.pgemm4_configs()):
        for M in (13, bq + 7):
            x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
            for splits in (1, 2, 5):
                for gm in (1, 4):
                    y = ops.pgemm4(x, w, epi, cfg=cfg, splits=splits, group_m=gm)
                    torch.cuda.synchronize()
                    _check(y, x, w, epi, what=f"cfg {cfg} M {M} splits {splits} gm {gm}")


@pytest.mark.parametrize("epi", [ops.EPI_BF16, ops.EPI_SWIGLU, ops.EPI_F32])
def test_pgemm4_rms_prologue_and_residual_epilogue(epi):
    torch.manual_seed(1)
    K, N, eps = 1024, 200, 1e-5
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, False, 5)
    for cfg, (bp, bq, _lds) in enumerate(ops.pgemm4_configs()):
        for M in (13, bq + 7):
            r = ((torch.rand(M, K, device=DEV) * 2 - 1) * 3).to(torch.bfloat16)
            rf = r.float()
            xn = rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + eps)
            exp = xn @ w.float().t()
            if epi == ops.EPI_SWIGLU:
                exp = torch.nn.functional.silu(exp[:, :N]) * exp[:, N:]
            for splits in (1, 4):
                y = ops.pgemm4(r, w, epi, cfg=cfg, splits=splits, rms_eps=eps).float()
                err = (y - exp).abs().max().item()
                assert err <= 2e-2 * exp.abs().max().item(), f"rms cfg {cfg} splits {splits} M {M}: {err}"
                if epi == ops.EPI_BF16:
                    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
                    res = ((torch.rand(M, N, device=DEV) * 2 - 1) * 8).to(torch.bfloat16)
                    want = x.float() @ w.float().t() + res.float()
                    out = ops.pgemm4(x, w, epi, cfg=cfg, splits=splits, res=res, out=res)   # in place
                    assert out.data_ptr() == res.data_ptr()
                    err = (out.float() - want).abs().max().item()
                    assert err <= 2e-2 * want.abs().max().item(), f"res cfg {cfg} splits {splits} M {M}: {err}"


def test_pgemm4_split_k_deterministic_and_graph_replay():
    K, N, M = 4096, 512, 300
    w = _weights(N, K, False, 3)
    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    exp = ops.pgemm4(x, w, ops.EPI_F32, cfg=0, splits=8)
    for _ in range(4):
        assert torch.equal(ops.pgemm4(x, w, ops.EPI_F32, cfg=0, splits=8), exp)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.pgemm4(x, w, ops.EPI_F32, cfg=0, splits=8)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g, stream=s):
        yg = ops.pgemm4(x, w, ops.EPI_F32, cfg=0, splits=8)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(yg, exp)
    _check(exp, x, w, ops.EPI_F32, tol=1e-3)


@pytest.mark.parametrize("name,N,K,epi", [
    ("qkv", 10240, 8192, ops.EPI_BF16),
    ("o_proj", 8192, 8192, ops.EPI_BF16),
    ("gate_up", 28672, 8192, ops.EPI_SWIGLU),
    ("down", 8192, 28672, ops.EPI_BF16),
    ("lm_head", 128256, 8192, ops.EPI_F32),
])
def test_pgemm4_tp1_prefill_shapes(name, N, K, epi):
    M = 245
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, False, 7)
    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    for cfg, splits in ((0, 1), (0, 4), (1, 3)):
        y = ops.pgemm4(x, w, epi, cfg=cfg, splits=splits)
        torch.cuda.synchronize()
        _check(y, x, w, epi, what=f"{name} cfg {cfg} splits {splits}")
