"""mgemm.hip (hand-written MFMA GEMM for batches of more than 2 rows) against the fp32 PyTorch oracle of ops/reference.py:
every tile configuration x epilogue (bf16 / fp32 / SwiGLU) x weight dtype (bf16 / row-scaled e4m3) x split-K,
partial tiles in M and N, plus the Llama-3.3-70B projection shapes at TP = 8 that the engine routes here."""

import pytest
import torch

from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _oracle(x, w, epi):
    if ops._is_fp8(w):
        xq, sx = ref.quantize_fp8(x.cpu())
        xr = ref.dequant_fp8(xq, sx, torch.float32)
        wr = ref.dequant_fp8(w.q.cpu(), w.scale.cpu(), torch.float32)
    else:
        xr, wr = x.float().cpu(), w.float().cpu()
    y = xr @ wr.t()
    if epi == ops.EPI_SWIGLU:
        n = wr.shape[0] // 2
        y = torch.nn.functional.silu(y[:, :n]) * y[:, n:]
    return y


def _check(y, x, w, epi, tol=2e-2):
    exp = _oracle(x, w, epi)
    got = y.float().cpu()
    err = (got - exp).abs().max().item()
    scale = exp.abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err:.4g} vs scale {scale:.4g}"


def _weights(rows, K, fp8, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    w = (torch.rand(rows, K, generator=g) * 2 - 1).to(torch.bfloat16).to(DEV)
    return ops.quantize_fp8(w) if fp8 else w


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("epi", [ops.EPI_BF16, ops.EPI_F32, ops.EPI_SWIGLU])
def test_every_config(epi, fp8):
    torch.manual_seed(0)
    K = 1024
    N = 200  # not a multiple of any tile width: partial n tiles
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, fp8, 1)
    for cfg, (bm, bn, *_rest) in enumerate(ops.mgemm_configs()):
        for M in (13, bm + 7):
            x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
            # one workgroup per tile, 4-way split-K, and stream-K grids whose shares straddle tiles
            for grid in (1, 4, -7, -256):
                if not ops.mgemm_valid(cfg, M, N, K, epi, fp8, grid):
                    continue
                y = ops.mgemm(x, w, epi, cfg=cfg, grid=grid)
                torch.cuda.synchronize()
                _check(y, x, w, epi)


@pytest.mark.parametrize("name,N,K,epi", [
    ("qkv", 1280, 8192, ops.EPI_BF16),
    ("o_proj", 8192, 1024, ops.EPI_BF16),
    ("gate_up", 3584, 8192, ops.EPI_SWIGLU),
    ("down", 8192, 3584, ops.EPI_BF16),
    ("lm_head", 16032, 8192, ops.EPI_F32),
])
@pytest.mark.parametrize("M", [16, 64, 256])
def test_tp8_projection_shapes_planned(name, N, K, epi, M):
    """The planner's pick (tuned table or heuristic) at one TP=8 rank's Llama-3.3-70B shapes."""
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, False, 2)
    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    y = ops.mgemm(x, w, epi)
    torch.cuda.synchronize()
    _check(y, x, w, epi)


def test_split_k_tickets_reset_between_launches():
    """The last arriving slice resets its tile's ticket: back-to-back launches (and a captured graph
    replayed several times) keep reducing correctly."""
    K, N, M = 4096, 256, 64
    w = _weights(N, K, False, 3)
    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    exp = ops.mgemm(x, w, ops.EPI_F32, cfg=4, grid=16)
    for _ in range(5):
        y = ops.mgemm(x, w, ops.EPI_F32, cfg=4, grid=16)
        assert torch.equal(y, exp)
        y = ops.mgemm(x, w, ops.EPI_F32, cfg=4, grid=-100)   # stream-K shares straddle tiles
        assert (y - exp).abs().max().item() <= 1e-3 * exp.abs().max().item()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.mgemm(x, w, ops.EPI_F32, cfg=4, grid=16)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g, stream=s):
        yg = ops.mgemm(x, w, ops.EPI_F32, cfg=4, grid=16)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(yg, exp)
    _check(exp, x, w, ops.EPI_F32, tol=1e-3)


@pytest.mark.parametrize("epi", [ops.EPI_BF16, ops.EPI_SWIGLU, ops.EPI_F32])
def test_rms_prologue_and_residual_epilogue(epi):
    """ops.linear_rms / linear_residual on the mgemm route: the RMS statistics of the un-normalised rows are
    the GEMM's prologue (1/rms in the epilogue, gamma folded into W) and the residual add is its epilogue
    (in place on the residual stream) -- every tile configuration, one-workgroup-per-tile, split-K and
    stream-K grids (the row sums of squares travel with the partial tiles)."""
    torch.manual_seed(1)
    K, N, eps = 1024, 200, 1e-5
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, False, 5)
    for cfg, (bm, bn, _t, _l, sw, rb) in enumerate(ops.mgemm_configs()):
        for M in (13, bm + 7):
            r = ((torch.rand(M, K, device=DEV) * 2 - 1) * 3).to(torch.bfloat16)
            rf = r.float().cpu()
            xn = (rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + eps))
            exp = xn @ w.float().cpu().t()
            if epi == ops.EPI_SWIGLU:
                exp = torch.nn.functional.silu(exp[:, :N]) * exp[:, N:]
            for grid in (1, 4, -7):
                if not ops.mgemm_valid(cfg, M, N, K, epi, False, grid):
                    continue
                y = ops.mgemm(r, w, epi, cfg=cfg, grid=grid, rms_eps=eps).float().cpu()
                err = (y - exp).abs().max().item()
                assert err <= 2e-2 * exp.abs().max().item(), f"rms cfg {cfg} grid {grid} M {M}: {err}"
                if epi == ops.EPI_BF16:
                    x = ((torch.rand(M, K, device=DEV) * 2 - 1)).to(torch.bfloat16)
                    res = ((torch.rand(M, N, device=DEV) * 2 - 1) * 8).to(torch.bfloat16)
                    want = (x.float() @ w.float().t() + res.float()).cpu()
                    out = ops.mgemm(x, w, epi, cfg=cfg, grid=grid, res=res, out=res)   # in place
                    assert out.data_ptr() == res.data_ptr()
                    err = (out.float().cpu() - want).abs().max().item()
                    assert err <= 2e-2 * want.abs().max().item(), f"res cfg {cfg} grid {grid} M {M}: {err}"


def _w8_oracle(x, w, epi, rms_eps=None):
    """fp32 oracle of the W8 mode: bf16 activations (optionally RMS-normalised, unit gamma) against the
    dequantized e4m3 weights."""
    xr = x.float().cpu()
    if rms_eps is not None:
        xr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + rms_eps)
    y = xr @ ref.dequant_fp8(w.q.cpu(), w.scale.cpu(), torch.float32).t()
    if epi == ops.EPI_SWIGLU:
        n = y.shape[1] // 2
        y = torch.nn.functional.silu(y[:, :n]) * y[:, n:]
    return y


@pytest.mark.parametrize("epi", [ops.EPI_BF16, ops.EPI_F32, ops.EPI_SWIGLU])
def test_w8_every_config(epi):
    """W8 mode (fp8 weights, bf16 activations, no activation quantization): every configuration built for it x
    epilogue x one-workgroup-per-tile / split-K / stream-K grids, partial M and N tiles, RMS prologue and the
    residual epilogue, against the fp32 oracle."""
    torch.manual_seed(2)
    K, N, eps = 1024, 200, 1e-5
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, True, 7)
    n_cfg = 0
    for cfg, (bm, *_rest) in enumerate(ops.mgemm_configs()):
        if not ops.mgemm_valid(cfg, 64, N, K, epi, 2):
            continue
        n_cfg += 1
        for M in (17, bm + 7):
            x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
            for grid in (1, 4, -7, -256):
                if not ops.mgemm_valid(cfg, M, N, K, epi, 2, grid):
                    continue
                y = ops.mgemm(x, w, epi, cfg=cfg, grid=grid, w8=True).float().cpu()
                exp = _w8_oracle(x, w, epi)
                err = (y - exp).abs().max().item()
                assert err <= 1e-2 * exp.abs().max().item(), f"cfg {cfg} grid {grid} M {M}: {err}"
                r = (x.float() * 3).to(torch.bfloat16)
                y = ops.mgemm(r, w, epi, cfg=cfg, grid=grid, rms_eps=eps, w8=True).float().cpu()
                exp = _w8_oracle(r, w, epi, eps)
                err = (y - exp).abs().max().item()
                assert err <= 1e-2 * exp.abs().max().item(), f"rms cfg {cfg} grid {grid} M {M}: {err}"
                if epi == ops.EPI_BF16:
                    res = ((torch.rand(M, N, device=DEV) * 2 - 1) * 8).to(torch.bfloat16)
                    want = _w8_oracle(x, w, epi) + res.float().cpu()
                    out = ops.mgemm(x, w, epi, cfg=cfg, grid=grid, res=res, out=res, w8=True)
                    err = (out.float().cpu() - want).abs().max().item()
                    assert err <= 1e-2 * want.abs().max().item(), f"res cfg {cfg} grid {grid} M {M}: {err}"
    assert n_cfg >= 6


@pytest.mark.parametrize("M", [17, 64, 128])
def test_w8_decode_projections_launch_no_activation_quantization(M, monkeypatch):
    """The fp8 projections of a 17-128-row decode step (one TP=4 rank's 70B shapes) run mgemm's W8 mode: no
    quantize_act_fp8 call on any of the four, and each matches the bf16-activation oracle."""
    if not ops.W8_ON:
        pytest.skip("K8S_MGEMM_W8=0")

    def no_quant(*a, **k):
        raise AssertionError("quantize_act_fp8 called on a W8 row count")

    monkeypatch.setattr(ops, "quantize_act_fp8", no_quant)
    eps, H, I, nqkv, no = 1e-5, 8192, 28672 // 4, (64 + 16) * 128 // 4, 64 * 128 // 4
    r = ((torch.rand(M, H, device=DEV) * 2 - 1) * 2).to(torch.bfloat16)
    wqkv = _weights(nqkv, H, True, 11)
    y = ops.linear_rms(r, wqkv, eps)
    exp = _w8_oracle(r, wqkv, ops.EPI_BF16, eps)
    assert (y.float().cpu() - exp).abs().max().item() <= 1e-2 * exp.abs().max().item()
    wgu = _weights(2 * I, H, True, 12)
    h = ops.linear_rms(r, wgu, eps, ops.EPI_SWIGLU)
    exp = _w8_oracle(r, wgu, ops.EPI_SWIGLU, eps)
    assert (h.float().cpu() - exp).abs().max().item() <= 1e-2 * exp.abs().max().item()
    wdown = _weights(H, I, True, 13)
    res = r.clone()
    want = _w8_oracle(h, wdown, ops.EPI_BF16) + res.float().cpu()
    out = ops.linear_residual(h, wdown, res)
    assert (out.float().cpu() - want).abs().max().item() <= 1e-2 * want.abs().max().item()
    wo = _weights(H, no, True, 14)
    a = (torch.rand(M, no, device=DEV) * 2 - 1).to(torch.bfloat16)
    y = ops.linear(a, wo)
    exp = _w8_oracle(a, wo, ops.EPI_BF16)
    assert (y.float().cpu() - exp).abs().max().item() <= 1e-2 * exp.abs().max().item()
