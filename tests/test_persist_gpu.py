"""Layer-persistent decode (decode_persist.hip, ops/persist.py): one launch for every decoder layer of a decode step.

Checked against the four-launch decode path (norm+GEMV, fused RoPE/KV/attention, GEMV, ...) and against the CPU fp32
reference model with the same weights, at TP = 1 and at one simulated TP rank of the 70B head layout (GQA 8:1, one kv
head, 1024-wide O input, 3584-wide down input); multi-chunk contexts (in-launch merge), padded rows, determinism and
epochs across launches, graph replay, and the bounded-wait drain when every in-kernel wait times out."""

import math

import pytest
import torch

from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.models.config import LlamaConfig
from k8s_llm_scheduler_amd.models.llama import LlamaModel
from k8s_llm_scheduler_amd.parallel import TPGroup

pytestmark = pytest.mark.gpu

# TP = 1 model with the tiny-tp8 head layout (16 q / 8 kv heads), and the 70B layout at one TP = 8 rank's shapes
CFG_TP1 = LlamaConfig("p-tp1", 2, 2048, 16, 8, 128, 4096, 16384, bos_id=16128, eos_ids=(16137,), max_position=4096)
CFG_70B = LlamaConfig("p-70b-2l", 2, 8192, 64, 8, 128, 28672, 16384, bos_id=16128, eos_ids=(16137,),
                      max_position=4096)


def _models(cfg, tp_sim: int):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.native()
    tp = (lambda: TPGroup(0, tp_sim, None, "none", simulate=True)) if tp_sim > 1 else (lambda: None)
    g = LlamaModel(cfg, tp=tp(), device="cuda", seed=5, max_model_len=4096)
    c = LlamaModel(cfg, tp=tp(), device="cpu", seed=5, max_model_len=4096)
    return g, c


@pytest.fixture(scope="module")
def tp1():
    return _models(CFG_TP1, 1)


@pytest.fixture(scope="module")
def tp8sim():
    return _models(CFG_70B, 8)


def _state(g, c, ctxs, nblocks=160, seed=0):
    """Random KV cache (the same on both models), block tables and context lengths (new token included)."""
    gen = torch.Generator().manual_seed(seed)
    g.allocate_kv(nblocks, 16)
    c.allocate_kv(nblocks, 16)
    kv = (torch.rand(c.kv_cache.shape, generator=gen) - 0.5).to(torch.bfloat16)
    c.kv_cache.copy_(kv)
    g.kv_cache.copy_(kv.cuda())
    B = len(ctxs)
    per = nblocks // B
    bt = torch.zeros(B, per, dtype=torch.int32)
    for b in range(B):
        bt[b] = torch.arange(b * per, (b + 1) * per, dtype=torch.int32).flip(0)   # scattered, descending block ids
    ctx = torch.tensor(ctxs, dtype=torch.int32)
    tok = torch.tensor([(97 * (b + 3)) % 16000 for b in range(B)], dtype=torch.int32)
    return tok, ctx, bt


def _decode(m, tok, ctx, bt, persist, max_context=4096):
    m.persist_decode = persist
    dev = m.device
    out = m.forward_decode(tok.to(dev), ctx.to(dev), bt.to(dev), max_context)
    m.persist_decode = None
    return out


def _check(g, c, ctxs, seed=0):
    tok, ctx, bt = _state(g, c, ctxs, seed=seed)
    kv0 = g.kv_cache.clone()
    four = _decode(g, tok, ctx, bt, False)
    kv_four = g.kv_cache.clone()
    g.kv_cache.copy_(kv0)
    g.persist_decode = True
    assert g.persist_decode_ok(len(ctxs), 4096), g._persist.rc if g._persist else None
    pers = _decode(g, tok, ctx, bt, True)
    torch.cuda.synchronize()
    cpu = _decode(c, tok, ctx, bt, False)
    # logits [tp, B, V] of the live rows: persistent vs four launches vs the fp32 reference (bf16 roundings differ
    # between the paths)
    live = [b for b, n in enumerate(ctxs) if n > 0]
    pc, fc, cc = (t.float().cpu()[:, live] for t in (pers, four, cpu))
    scale = cc.abs().max().item()
    assert (pc - cc).abs().max().item() < 0.05 * scale
    if not g.tp.simulate:     # (a simulated rank's four-launch path skips the all-reduce and its residual add)
        assert (pc - fc).abs().max().item() < 0.05 * scale
    cos = torch.nn.functional.cosine_similarity(pc.flatten(), cc.flatten(), dim=0).item()
    assert cos > 0.999, cos
    assert torch.isfinite(pers.float()).all()
    # the new token's K/V were written at its slot (and nothing else changed)
    diff = (g.kv_cache.float()[:1] - kv_four.float()[:1]).abs()    # layer 0: the same input on both paths
    assert diff.max().item() < 0.05
    changed = (g.kv_cache != kv0).flatten(3).any(-1)   # [L, 2, slots]
    for b, n in enumerate(ctxs):
        if n <= 0:
            continue
        pos = n - 1
        slot = int(bt[b, pos // 16]) * 16 + pos % 16
        assert changed[:, :, slot].all()
        changed[:, :, slot] = False
    assert not changed.any()
    return pers


def _handoff(g, l, b, B, off, n):
    """Values [off, off + n) (granule units: 2 values each) of layer l's hand-off buffer of row b, as float32."""
    gl = g._persist.gl
    w = g._persist.gran.view(torch.int32).view(-1, 2)[(l * B + b) * gl + off:(l * B + b) * gl + off + n // 2, 0]
    return w.contiguous().view(torch.bfloat16).float()


def test_persist_layer0_handoffs_match_the_kernels(tp1):
    """Stage by stage (layer 0, one row): the QKV, attention, O (+ residual), SwiGLU and down (+ residual) vectors the
    persistent kernel hands from CU to CU equal the four-launch kernels' outputs up to bf16 rounding."""
    g, c = tp1
    tok, ctx, bt = _state(g, c, [70], seed=7)
    kv0 = g.kv_cache.clone()
    dev = torch.device("cuda")
    t, cx, b_ = tok.to(dev), ctx.to(dev), bt.to(dev)
    _decode(g, tok, ctx, bt, True)
    torch.cuda.synchronize()
    g.kv_cache.copy_(kv0)
    w = g.layers[0]
    eps, D = g.cfg.rms_eps, g.D
    x0 = ops.embedding(t, g.embed)
    qkv = ops.linear_norm(x0, w.wqkv, None, eps, None, None)
    a = ops.decode_attention_fused(qkv, g.cos_sin, g.kv_cache[0, 0], g.kv_cache[0, 1], b_, cx, g.scale, 16, 4096,
                                   g.nq, g.nkv, D)
    o = (x0.float() + ops.linear(a, w.wo).float()).to(torch.bfloat16)
    gg = ops.linear_norm(o, w.wgu, None, eps, None, None, epi=ops.EPI_SWIGLU)
    x1 = (o.float() + ops.linear(gg, w.wdown).float()).to(torch.bfloat16)
    nqkv, nqD, H, I = qkv.shape[1], g.nq * D, g.cfg.hidden, g.I
    offs = {"qkv": (0, nqkv, qkv), "attn": (nqkv // 2, nqD, a), "o": ((nqkv + nqD) // 2, H, o),
            "g": ((nqkv + nqD + H) // 2, I, gg), "x": ((nqkv + nqD + H + I) // 2, H, x1)}
    for name, (off, n, ref) in offs.items():
        got = _handoff(g, 0, 0, 1, off, n)
        r = ref.float().flatten().cpu()
        err = (got.cpu() - r).abs().max().item()
        assert err <= 0.02 * r.abs().max().item() + 1e-3, (name, err, got[:8], r[:8])


@pytest.mark.parametrize("ctxs", [[1], [64], [65], [300], [300, 7], [700, 129]])
def test_persist_tp1_matches_four_launch_and_cpu(tp1, ctxs):
    g, c = tp1
    _check(g, c, ctxs)


@pytest.mark.parametrize("ctxs", [[1], [528], [528, 40]])
def test_persist_tp8_shapes_match_four_launch_and_cpu(tp8sim, ctxs):
    """One TP = 8 rank of the 70B layout (collectives skipped): G = 8 q heads per kv head, O K = 1024, down K = 3584
    (7 pieces per row), 5 QKV rows per CU (uneven row-pair split)."""
    g, c = tp8sim
    _check(g, c, ctxs)


def test_persist_padded_row_and_plan_limits(tp1):
    """A padded graph row (context 0) gets zero attention and leaves the cache alone; shapes the kernel does not plan
    (O input not a multiple of 512 at one TP = 8 rank of tiny-tp8) fall back to the four-launch path."""
    g, c = tp1
    _check(g, c, [90, 0])
    from k8s_llm_scheduler_amd.models.config import PRESETS

    small = LlamaModel(PRESETS["tiny-tp8"], tp=TPGroup(0, 8, None, "none", simulate=True), device="cuda", seed=1,
                       max_model_len=512)
    small.allocate_kv(32, 16)
    small.persist_decode = True
    assert not small.persist_decode_ok(1, 512) and small._persist.rc < 0


def test_persist_deterministic_epochs_and_graph(tp1):
    """The fixed-order reduction makes repeated launches bit-identical; each launch advances the epoch by one; a
    captured graph replays the same result without host involvement."""
    g, c = tp1
    tok, ctx, bt = _state(g, c, [333, 77], seed=3)
    kv0 = g.kv_cache.clone()
    dev = torch.device("cuda")
    args = (tok.to(dev), ctx.to(dev), bt.to(dev), 4096)
    g.persist_decode = True
    outs = []
    e0 = None
    for _ in range(3):
        g.kv_cache.copy_(kv0)
        outs.append(g.forward_decode(*args).clone())
        torch.cuda.synchronize()
        e = int(g._persist.sync[0])
        assert e0 is None or e == e0 + 1
        e0 = e
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        g.kv_cache.copy_(kv0)
        with torch.cuda.graph(graph, stream=s):
            out_g = g.forward_decode(*args)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(2):
        g.kv_cache.copy_(kv0)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out_g, outs[0])
    g.snapshot_decode_health()
    torch.cuda.synchronize()
    g.check_decode_health()
    g.persist_decode = None


def test_persist_timeout_drains_and_reports(tp1, monkeypatch):
    """With every in-kernel wait bounded by ~10 ns, the waits time out at once: the grid still drains (no hang), the
    error bits reach check_decode_health (CollectiveError for the decision service's retries), and the next launch
    with the normal bound is correct again."""
    from k8s_llm_scheduler_amd.ops import persist
    from k8s_llm_scheduler_amd.parallel.comm import CollectiveError

    g, c = tp1
    tok, ctx, bt = _state(g, c, [200], seed=4)
    kv0 = g.kv_cache.clone()
    monkeypatch.setattr(persist, "TIMEOUT_S", 1e-8)
    _decode(g, tok, ctx, bt, True)
    g.snapshot_decode_health()
    torch.cuda.synchronize()
    with pytest.raises(CollectiveError):
        g.check_decode_health()
    monkeypatch.setattr(persist, "TIMEOUT_S", 0.25)
    g.kv_cache.copy_(kv0)
    good = _decode(g, tok, ctx, bt, True)
    g.kv_cache.copy_(kv0)
    ref = _decode(g, tok, ctx, bt, False)
    assert (good.float() - ref.float()).abs().max().item() < 0.05 * ref.float().abs().max().item()
    g.snapshot_decode_health()
    torch.cuda.synchronize()
    g.check_decode_health()
