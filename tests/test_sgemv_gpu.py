"""sgemv.hip (small decode batches: 3..4 rows on v_dot2, 5..16 rows on the matrix cores; x in registers) against the fp32 PyTorch oracle: every epilogue
(bf16, fp32 logits, SwiGLU, residual add in place) with and without the folded-norm 1/rms prologue, bf16 and row-scaled
e4m3 weights (bf16 activations: sgemv never quantizes them), ragged N / K, every launch plan (1024-element slices,
2048-element slices split 2 or 4 ways, k-groups with partial slabs + finalize), the Llama-3.3-70B projection shapes at
TP = 1 and TP = 8, determinism, and the routing of ops.linear_rms / linear_residual / linear at 3..8 rows."""

import pytest
import torch

from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _weights(rows, K, fp8, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    w = (torch.rand(rows, K, generator=g) * 2 - 1).to(torch.bfloat16).to(DEV)
    return ops.quantize_fp8(w) if fp8 else w


def _oracle(x, w, epi, norm, res, eps=1e-5):
    """fp32: (x / rms(x)) @ W^T (fp8: dequantized W, bf16 x), then the epilogue."""
    xf = x.float()
    if norm:
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    wf = ref.dequant_fp8(w.q, w.scale, torch.float32) if ops._is_fp8(w) else w.float()
    y = xf @ wf.t()
    if epi == ops.EPI_SWIGLU:
        n = wf.shape[0] // 2
        y = torch.nn.functional.silu(y[:, :n]) * y[:, n:]
    if res is not None:
        y = y + res.float()
    return y


def _run(M, N, K, epi, fp8, norm=False, with_res=False, seed=0):
    rows = 2 * N if epi == ops.EPI_SWIGLU else N
    w = _weights(rows, K, fp8, seed + 1)
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = ((torch.rand(M, K, generator=g) * 2 - 1) * (4.0 if norm else 1.0)).to(torch.bfloat16).to(DEV)
    res = (torch.rand(M, N, generator=g) * 2 - 1).to(torch.bfloat16).to(DEV) if with_res else None
    exp = _oracle(x, w, epi, norm, res)
    out = res.clone() if with_res else None
    y = ops._sgemv(x, w, epi, res=out, rms_eps=1e-5 if norm else None, out=out)
    torch.cuda.synchronize()
    assert y is not None, "sgemv declined"
    err = (y.float() - exp).abs().max().item()
    scale = exp.abs().max().item() + 1e-6
    assert err <= 1e-2 * scale, f"M={M} N={N} K={K} epi={epi} fp8={fp8} norm={norm} res={with_res}: " \
                                f"max err {err:.4g} vs scale {scale:.4g}"
    return y


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("epi,norm,with_res", [(ops.EPI_BF16, False, False), (ops.EPI_BF16, True, False),
                                               (ops.EPI_BF16, False, True), (ops.EPI_F32, True, False),
                                               (ops.EPI_F32, False, False), (ops.EPI_SWIGLU, True, False),
                                               (ops.EPI_SWIGLU, False, False)])
@pytest.mark.parametrize("M", [3, 4, 5, 8])
def test_every_epilogue_ragged(M, epi, norm, with_res, fp8):
    # N = 200: bands of 64 rows with a partial last band; K = 1008 (not a multiple of a 1024-element slice)
    _run(M, 200, 1008, epi, fp8, norm, with_res, seed=M)


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("epi,norm,with_res", [(ops.EPI_BF16, False, False), (ops.EPI_BF16, True, False),
                                               (ops.EPI_BF16, False, True), (ops.EPI_F32, True, False),
                                               (ops.EPI_SWIGLU, True, False), (ops.EPI_SWIGLU, False, False)])
@pytest.mark.parametrize("M,K", [(5, 1024), (8, 3584), (9, 8192), (16, 1024), (12, 12288), (16, 28672)])
def test_matrix_core_rows(M, K, epi, norm, with_res, fp8):
    """5..16 rows on the matrix-core form: both x layouts (<= 8 rows: odd steps parked in lanes 8..15; 9..16 rows),
    8 / 16 / 32 register steps, a ragged band (N = 300), masked steps of the last wave (K = 3584) and k-groups with
    partial slabs (12288, 28672; the norm prologue needs one k-group)."""
    if norm and (K > 8192 or (fp8 and K > 8192)):
        pytest.skip("the norm prologue needs one k-group")
    _run(M, 300, K, epi, fp8, norm, with_res, seed=M + K)


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("K", [1024, 3584, 4096, 6144, 8192, 14336, 28672])
def test_every_plan(K, fp8):
    """1024-element slices (K <= 1024), 2048-element slices split 2 / 4 ways with idle slices (3584, 6144), and the
    k-group splits with partial slabs (14336: 2 x 4 slices, 28672: 7 x 2 slices) -- plain and residual epilogues."""
    _run(8, 136, K, ops.EPI_BF16, fp8, seed=K)
    _run(5, 72, K, ops.EPI_BF16, fp8, with_res=True, seed=K + 1)


@pytest.mark.parametrize("name,N,K,epi,norm,with_res", [
    ("tp1_qkv", 10240, 8192, ops.EPI_BF16, True, False),
    ("tp1_o", 8192, 8192, ops.EPI_BF16, False, True),
    ("tp1_gate_up", 28672, 8192, ops.EPI_SWIGLU, True, False),
    ("tp1_down", 8192, 28672, ops.EPI_BF16, False, True),
    ("tp8_qkv", 1280, 8192, ops.EPI_BF16, True, False),
    ("tp8_o", 8192, 1024, ops.EPI_BF16, False, False),
    ("tp8_gate_up", 3584, 8192, ops.EPI_SWIGLU, True, False),
    ("tp8_down", 8192, 3584, ops.EPI_BF16, False, False),
    ("tp8_lm_head", 16032, 8192, ops.EPI_F32, True, False),
])
@pytest.mark.parametrize("fp8", [False, True])
def test_llama70b_shapes(name, N, K, epi, norm, with_res, fp8):
    for M in (4, 8, 16):
        _run(M, N, K, epi, fp8, norm, with_res, seed=M)


def test_deterministic():
    w = _weights(8192, 28672, False, 3)
    x = (torch.rand(6, 28672, device=DEV) * 2 - 1).to(torch.bfloat16)
    a = ops._sgemv(x, w, ops.EPI_BF16)
    b = ops._sgemv(x, w, ops.EPI_BF16)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_ops_route_small_batches_to_sgemv(monkeypatch):
    """3..16 rows: linear_rms (norm prologue; fp8 too, bf16 activations), linear_residual and linear go to sgemv;
    2 rows stay on the GEMV, 17 rows go to mgemm."""
    nat = ops.native()
    calls = []
    orig = nat.sgemv

    def spy(*a):
        calls.append(a[6])   # M
        return orig(*a)

    monkeypatch.setattr(nat, "sgemv", spy)
    K, N = 2048, 512
    for fp8 in (False, True):
        w = _weights(N, K, fp8, 5)
        for M in (2, 3, 8, 16, 17):
            x = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
            ops.linear_rms(x, w, 1e-5)
            ops.linear(x, w)
            r = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
            ops.linear_residual(x, w, r)
    torch.cuda.synchronize()
    assert sorted(set(calls)) == [3, 8, 16] and len(calls) == 2 * 3 * 3


def test_k_group_tickets_return_to_zero():
    """K-group launches reduce their partial slabs in the kernel (the last workgroup of a band sums them, a ticket
    per band): 600 launches cycle every ticket range twice and stay bitwise equal, also under graph replay."""
    w = _weights(2 * 1024, 28672, True, 7)
    x = (torch.rand(8, 28672, device=DEV) * 2 - 1).to(torch.bfloat16)
    ref0 = ops._sgemv(x, w, ops.EPI_SWIGLU)
    outs = [ops._sgemv(x, w, ops.EPI_SWIGLU) for _ in range(600)]
    torch.cuda.synchronize()
    assert all(torch.equal(o, ref0) for o in outs)
    exp = _oracle(x, w, ops.EPI_SWIGLU, False, None)
    assert (ref0.float() - exp).abs().max().item() <= 1e-2 * exp.abs().max().item()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops._sgemv(x, w, ops.EPI_SWIGLU)
        with torch.cuda.graph(g, stream=s):
            y = ops._sgemv(x, w, ops.EPI_SWIGLU)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(5):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, ref0)
