"""FP8 (row-scaled OCP e4m3) weights on CPU: quantization error bound, the fp8 linear ops against
dequantized fp32 math, and the tiny Llama with fp8 projections tracking its bf16 twin."""

import torch

from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine
from k8s_llm_scheduler_amd.models.config import PRESETS
from k8s_llm_scheduler_amd.models.llama import LlamaModel
from k8s_llm_scheduler_amd.ops import reference as ref

from test_engine_cpu import _prefill  # noqa: E402


def test_quantize_roundtrip_error_bound():
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(64, 512, generator=g) * torch.logspace(-3, 1, 64)[:, None]).bfloat16()
    fw = ops.quantize_fp8(w)
    assert fw.q.dtype == torch.uint8 and fw.scale.shape == (64,)
    back = fw.dequant(torch.float32)
    wf = w.float()
    # e4m3: 3 mantissa bits -> relative error <= 2^-4 for normal values; row max maps to 448
    rel = ((back - wf).abs() / wf.abs().clamp_min(1e-30))[wf.abs() > fw.scale[:, None] * 2 ** -6]
    assert float(rel.max()) <= 2 ** -4 + 1e-6
    assert torch.allclose(back.abs().amax(1), wf.abs().amax(1), rtol=1e-6)


def test_fp8_linear_ops_match_dequantized_math():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(ops.GEMV_MAX_M, 256, generator=g).bfloat16()   # GEMV rows: bf16 activations
    w = ops.quantize_fp8((torch.randn(96, 256, generator=g) * 0.05).bfloat16())
    wd = w.dequant(torch.float32)
    torch.testing.assert_close(ops.linear(x, w).float(), (x.float() @ wd.T).bfloat16().float())
    xs = torch.randn(5, 256, generator=g).bfloat16()   # small-batch sgemv rows (3..8): bf16 activations too
    torch.testing.assert_close(ops.linear(xs, w).float(), (xs.float() @ wd.T).bfloat16().float())
    gu = ops.quantize_fp8((torch.randn(2 * 48, 256, generator=g) * 0.05).bfloat16())
    # GEMM rows (above the sgemv rows): per-token e4m3 activations
    xb = torch.randn(131, 256, generator=g).bfloat16()
    q, sc = ref.quantize_fp8(xb)
    xq = ref.dequant_fp8(q, sc, torch.float32)
    torch.testing.assert_close(ops.linear(xb, w).float(), (xq.bfloat16().float() @ wd.T).bfloat16().float())
    y = ops.linear_swiglu(xb, gu)
    want = ref.linear_swiglu(xq.bfloat16(), gu.dequant(torch.float32))
    torch.testing.assert_close(y.float(), want.float())


def test_tiny_model_fp8_tracks_bf16():
    ids = [7, 100, 2000, 31, 32, 33, 900, 12]
    m16 = LlamaModel(PRESETS["tiny"], device="cpu", seed=3, max_model_len=256)
    m8 = LlamaModel(PRESETS["tiny"], device="cpu", seed=3, max_model_len=256, weight_dtype="fp8")
    assert isinstance(m8.layers[0].wqkv, ops.Fp8Weight)
    proj = lambda m: m.weight_bytes() - sum(t.numel() * 2 for t in (m.embed, m.norm, m.lm_head))
    assert proj(m8) < 0.52 * proj(m16)   # 1 byte per weight + one fp32 scale per row
    a, _ = _prefill(m16, ids)
    b, _ = _prefill(m8, ids)
    a, b = a.flatten().float(), b.flatten().float()
    cos = torch.nn.functional.cosine_similarity(a, b, dim=0)
    assert float(cos) > 0.99
    eng = build_engine("tiny", device="cpu", max_batch=2, max_model_len=256, num_blocks=32, seed=1,
                       weight_dtype="fp8")
    out = eng.generate(["fp8 weights"], SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))[0]
    assert len(out.token_ids) == 4


def test_fp8_lm_head_option_tracks_bf16_head(monkeypatch):
    """K8S_FP8_LM_HEAD=1 quantizes the (norm-folded) LM head too; prefill and decode logits stay close to the
    bf16-head fp8 model's."""
    ids = [7, 100, 2000, 31, 32, 33, 900, 12]
    m8 = LlamaModel(PRESETS["tiny"], device="cpu", seed=3, max_model_len=256, weight_dtype="fp8")
    monkeypatch.setenv("K8S_FP8_LM_HEAD", "1")
    mh = LlamaModel(PRESETS["tiny"], device="cpu", seed=3, max_model_len=256, weight_dtype="fp8")
    assert isinstance(mh.lm_head, ops.Fp8Weight) and not isinstance(m8.lm_head, ops.Fp8Weight)
    assert mh.weight_bytes() < m8.weight_bytes() - 0.9 * m8.lm_head.numel()   # ~1 byte per head weight saved
    a, bt_a = _prefill(m8, ids)
    b, bt_b = _prefill(mh, ids)
    cos = torch.nn.functional.cosine_similarity(a.flatten().float(), b.flatten().float(), dim=0)
    assert float(cos) > 0.995
    ctx = torch.tensor([len(ids) + 1], dtype=torch.int32)
    da = m8.forward_decode(torch.tensor([77], dtype=torch.int32), ctx, bt_a, 256)
    db = mh.forward_decode(torch.tensor([77], dtype=torch.int32), ctx, bt_b, 256)
    assert float(torch.nn.functional.cosine_similarity(da.flatten().float(), db.flatten().float(), dim=0)) > 0.995


def test_fp8_linear_rms_quantizes_the_unnormalised_rows():
    """Above the sgemv rows, fp8 pre-norm projections quantize the residual rows themselves and fold 1/rms into
    the per-token scales (no normalised copy): the same bytes as quantizing x, the result within e4m3 rounding of
    quantize(RMSNorm(x)) @ W."""
    g = torch.Generator().manual_seed(3)
    M = max(ops.GEMV_MAX_M, ops.SGEMV_MAX_M) + 4
    r = (torch.randn(M, 256, generator=g) * 3).bfloat16()
    w = ops.quantize_fp8((torch.randn(64, 256, generator=g) * 0.05).bfloat16())
    q, s = ops.quantize_act_fp8(r, rms_eps=1e-5)
    q0, s0 = ops.quantize_act_fp8(r)
    assert torch.equal(q, q0)
    inv = torch.rsqrt(r.float().pow(2).mean(-1) + 1e-5)
    torch.testing.assert_close(s, s0 * inv)
    got = ops.linear_rms(r, w, 1e-5)
    xn = r.float() * inv[:, None]
    want = xn @ w.dequant(torch.float32).T
    assert float((got.float() - want).abs().max() / want.abs().max()) < 0.06
    gu = ops.quantize_fp8((torch.randn(2 * 32, 256, generator=g) * 0.05).bfloat16())
    y = ops.linear_rms(r, gu, 1e-5, ops.EPI_SWIGLU)
    assert y.shape == (M, 32) and y.dtype == torch.bfloat16


def test_mx_rows_route_o_and_down_inputs_through_mx_e4m3():
    """K16 block-scaled: above the sgemv rows the fp8 SwiGLU output is produced as MX e4m3 (one E8M0 scale per 32
    values) and the O / down projections consume MX rows; the CPU path rounds exactly as the GPU kernels do."""
    g = torch.Generator().manual_seed(4)
    M = max(ops.GEMV_MAX_M, ops.SGEMV_MAX_M) + 5
    r = (torch.randn(M, 256, generator=g) * 3).bfloat16()
    gu = ops.quantize_fp8((torch.randn(2 * 128, 256, generator=g) * 0.05).bfloat16())
    wd = ops.quantize_fp8((torch.randn(256, 128, generator=g) * 0.05).bfloat16())
    y = ops.linear_rms(r, gu, 1e-5, ops.EPI_SWIGLU, mx_consumer=wd)
    if not ops.mx_rows(M, wd):
        assert isinstance(y, torch.Tensor)
        return
    assert isinstance(y, ops.MxAct) and y.q.shape == (M, 128) and y.blocks().shape == (M, 4)
    bf = ops.linear_rms(r, gu, 1e-5, ops.EPI_SWIGLU)
    q, e = ref.quantize_mx(bf)
    assert torch.equal(y.q, q) and torch.equal(y.blocks(), e)
    res = torch.randn(M, 256, generator=g).bfloat16()
    want = (res.float() + (ref.dequant_mx(q, e) @ wd.dequant(torch.float32).T).bfloat16().float()).bfloat16()
    out = ops.linear_residual(y, wd, res.clone())
    torch.testing.assert_close(out.float(), want.float())
    # bf16 rows of the MX range are quantized to MX before the fp8 GEMM (the attention output's path)
    out2 = ops.linear_residual(bf, wd, res.clone())
    torch.testing.assert_close(out2.float(), want.float())


def _fp8_tp_worker(rank, world, port, q, ids):
    import os

    import torch.distributed as dist

    from k8s_llm_scheduler_amd.parallel import TPGroup

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tp = TPGroup(rank, world, dist.group.WORLD, "gloo")
        m = LlamaModel(PRESETS["tiny"], tp, device="cpu", seed=3, max_model_len=256, weight_dtype="fp8")
        lg, _ = _prefill(m, ids)
        if rank == 0:
            q.put(lg.float().flatten())
    finally:
        dist.destroy_process_group()


def test_fp8_mx_rows_under_tensor_parallel_track_tp1():
    """A 24-token fp8 prefill (GEMM rows: the O / down inputs travel as MX e4m3, the SwiGLU output is produced in MX)
    on TP = 2 gloo ranks tracks TP = 1: the 32-value blocks never straddle a shard boundary, so each rank's MX rows
    are the TP = 1 rows' own slices."""
    import socket

    import torch.multiprocessing as mp

    ids = [(37 * i + 11) % 16000 for i in range(24)]
    m1 = LlamaModel(PRESETS["tiny"], device="cpu", seed=3, max_model_len=256, weight_dtype="fp8")
    assert ops.mx_rows(24, m1.layers[0].wo) == ops.MX_ON
    lg1, _ = _prefill(m1, ids)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fp8_tp_worker, args=(r, 2, port, q, ids)) for r in range(2)]
    for p in procs:
        p.start()
    lg2 = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    cos = torch.nn.functional.cosine_similarity(lg1.float().flatten(), lg2, dim=0)
    assert float(cos) > 0.995, float(cos)


def test_mx_prologue_statistics_track_the_bf16_rms():
    """fp8 GEMM rows at TP = 1 take their RMS statistics from the dequantized MX copy of the residual stream
    (x_mx) instead of the bf16 rows.  Pin that parity: the MX-prologue result stays within e4m3 activation rounding of
    rmsnorm(r) (bf16 statistics) followed by the GEMM on the same e4m3 weights, and the RMS statistic itself within
    0.5 % (block-scaled e4m3 errors average out over a row of 8192)."""
    g = torch.Generator().manual_seed(5)
    M, K, N, eps = 24, 8192, 256, 1e-5
    r = (torch.randn(M, K, generator=g) * torch.linspace(0.2, 4.0, M).view(-1, 1)).bfloat16()
    w = ops.quantize_fp8((torch.randn(N, K, generator=g) * 0.02).bfloat16())
    x_mx = ops.quantize_act_mx(r)
    got = ops.linear_rms(r, w, eps, x_mx=x_mx).float()
    xn = (r.float() * torch.rsqrt(r.float().pow(2).mean(-1, keepdim=True) + eps)).bfloat16()
    want = (xn.float() @ w.dequant(torch.float32).T)
    rel = float((got - want).norm() / want.norm())
    assert rel < 0.05, rel                                       # e4m3 activations: a few % at most
    rms_mx = x_mx.dequant(torch.float32).pow(2).mean(-1).sqrt()
    rms_bf = r.float().pow(2).mean(-1).sqrt()
    assert float(((rms_mx - rms_bf) / rms_bf).abs().max()) < 5e-3
