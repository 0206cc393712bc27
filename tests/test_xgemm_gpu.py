"""xgemm.hip (activation-resident GEMM for 17-64 decode rows) against the fp32 PyTorch oracle: every epilogue (bf16,
fp32 logits, SwiGLU, + residual in place, x 1/rms), ragged row counts, K split into 2048-wide slabs (one, several, a
short last one), the 70B TP = 1 / TP = 8 decode shapes, determinism, and the routing of batched decode onto it."""

import pytest
import torch

from k8s_llm_scheduler_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.native()


def _rand(*shape, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.rand(*shape, generator=g, device=DEV) * 2 - 1).mul_(scale).to(torch.bfloat16)


def _ref(x, w, epi, res=None, rms_eps=None):
    xf = x.float()
    y = xf @ w.float().T
    if rms_eps is not None:
        y = y * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + rms_eps)
    if epi == ops.EPI_SWIGLU:
        n = w.shape[0] // 2
        return torch.nn.functional.silu(y[:, :n]) * y[:, n:]
    if res is not None:
        y = y + res.float()
    return y


def _close(got, want, rel=1e-2):
    err = (got.float() - want).abs().max().item()
    assert err <= rel * want.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("M", [17, 24, 32, 33, 48, 64])
@pytest.mark.parametrize("N,K", [(1280, 8192), (1024, 1024), (512, 2560), (2048, 4224)])
def test_xgemm_plain_matches_fp32(M, N, K):
    _setup()
    x, w = _rand(M, K, seed=M), _rand(N, K, scale=0.05, seed=N + K)
    y = ops.xgemm(x, w)
    assert y is not None and y.shape == (M, N) and y.dtype == torch.bfloat16
    _close(y, _ref(x, w, ops.EPI_BF16))


@pytest.mark.parametrize("M", [20, 64])
def test_xgemm_epilogues(M):
    _setup()
    N, K = 1024, 4096
    x, w = _rand(M, K, seed=1), _rand(N, K, scale=0.05, seed=2)
    f = ops.xgemm(x, w, ops.EPI_F32)
    assert f.dtype == torch.float32
    _close(f, _ref(x, w, ops.EPI_F32), 2e-3)
    wgu = _rand(2 * N, K, scale=0.05, seed=3)
    _close(ops.xgemm(x, wgu, ops.EPI_SWIGLU), _ref(x, wgu, ops.EPI_SWIGLU))
    res = _rand(M, N, seed=4)
    want = _ref(x, w, ops.EPI_BF16, res=res)
    out = ops.xgemm(x, w, res=res, out=res)      # in place into the residual stream
    assert out.data_ptr() == res.data_ptr()
    _close(out, want)
    for epi in (ops.EPI_BF16, ops.EPI_SWIGLU, ops.EPI_F32):
        ww = wgu if epi == ops.EPI_SWIGLU else w
        _close(ops.xgemm(x, ww, epi, rms_eps=1e-5), _ref(x, ww, epi, rms_eps=1e-5))


@pytest.mark.parametrize("tp", [1, 8])
def test_xgemm_70b_decode_shapes_and_determinism(tp):
    """Llama-3.3-70B projections at 64 rows (one TP rank's shapes) -- QKV with the RMS epilogue, O with the residual,
    gate/up with SwiGLU, down (K = 28672 / tp: 14 or 2 slabs) -- and bit-identical repeated launches."""
    _setup()
    H, I, M = 8192, 28672 // tp, 64
    r = _rand(M, H, seed=5)
    cases = [((10240 // tp, H), ops.EPI_BF16, "rms"), ((H, H // tp), ops.EPI_BF16, "res"),
             ((2 * I, H), ops.EPI_SWIGLU, "rms"), ((H, I), ops.EPI_BF16, "res")]
    for (n, k), epi, kind in cases:
        w = _rand(n, k, scale=0.02, seed=n + k)
        x = r if k == H else _rand(M, k, seed=k)
        if kind == "rms":
            a = ops.xgemm(x, w, epi, rms_eps=1e-5)
            b = ops.xgemm(x, w, epi, rms_eps=1e-5)
            _close(a, _ref(x, w, epi, rms_eps=1e-5))
        else:
            res = _rand(M, n, seed=9)
            a = ops.xgemm(x, w, res=res)
            b = ops.xgemm(x, w, res=res)
            _close(a, _ref(x, w, epi, res=res))
        assert torch.equal(a, b)


def test_batched_decode_projections_route_to_xgemm(monkeypatch):
    """33-64 bf16 rows: linear / linear_rms / linear_residual / linear_swiglu take xgemm (no RMSNorm kernel, no mgemm)
    and match the K8S_XGEMM=0 route."""
    _setup()
    M, H, N = 40, 2048, 1536
    r, w, wgu = _rand(M, H, seed=11), _rand(N, H, scale=0.05, seed=12), _rand(2 * N, H, scale=0.05, seed=13)
    monkeypatch.setattr(ops, "XGEMM_ON", True)
    calls = []
    orig = ops.xgemm
    monkeypatch.setattr(ops, "xgemm", lambda *a, **k: calls.append(1) or orig(*a, **k))
    got = [ops.linear_rms(r, w, 1e-5), ops.linear_rms(r, wgu, 1e-5, ops.EPI_SWIGLU), ops.linear(r, w[:, :H])]
    assert len(calls) >= 3
    monkeypatch.setattr(ops, "XGEMM_ON", False)
    want = [ops.linear_rms(r, w, 1e-5), ops.linear_rms(r, wgu, 1e-5, ops.EPI_SWIGLU), ops.linear(r, w[:, :H])]
    for a, b in zip(got, want):
        _close(a, b.float(), 2e-2)
