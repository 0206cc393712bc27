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
def test_fence_free_split_k_publish_equals_fenced(epi):
    """the default split-K publish (write-through slab stores, s_waitcnt, a relaxed ticket, sc1 loads by the
    reducer) relies on gfx950's cache behaviour; the fenced form (agent-scope release / acquire) is the memory
    model's.  Both sum the slices in the same order, so they must agree BITWISE -- over many-slice split-K and
    stream-K grids whose slices land on different XCDs, 40 launches back to back (a rare cross-XCD visibility race
    would show as one differing launch), and replayed from a graph."""
    torch.manual_seed(3)
    K, N, M = 8192, 1280, 64          # one TP = 8 rank's QKV at batch 64: the split-K decode shape
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, False, 9)
    x = ((torch.rand(M, K, device=DEV) * 2 - 1) * 2).to(torch.bfloat16)
    for cfg, grid in ((11, 16), (11, -600), (4, 32), (12, 8)):
        if not ops.mgemm_valid(cfg, M, N, K, epi, False, grid):
            continue
        want = ops.mgemm(x, w, epi, cfg=cfg, grid=grid, fenced=True)
        outs = [ops.mgemm(x, w, epi, cfg=cfg, grid=grid, fenced=False) for _ in range(40)]
        torch.cuda.synchronize()
        bad = [i for i, y in enumerate(outs) if not torch.equal(y, want)]
        assert not bad, f"cfg {cfg} grid {grid}: fence-free launches {bad} differ from the fenced result"
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ops.mgemm(x, w, epi, cfg=cfg, grid=grid, fenced=False)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            yg = [ops.mgemm(x, w, epi, cfg=cfg, grid=grid, fenced=False) for _ in range(8)]
        for _ in range(3):
            g.replay()
            torch.cuda.synchronize()
            assert all(torch.equal(y, want) for y in yg), f"cfg {cfg} grid {grid}: graph replay differs"
        _check(want, x, w, epi)


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


