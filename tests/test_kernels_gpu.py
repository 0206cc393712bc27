"""T3: every HIP kernel vs its plain-PyTorch fp32 reference (ops/reference.py) on an MI355X,
at Llama-3 shapes per TP slice."""

import math
import os

import pytest
import torch

from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.native()  # loud failure if the extension is missing on a GPU box


def rnd(*shape, scale=1.0, dtype=torch.bfloat16, gen=None):
    return (torch.randn(*shape, generator=gen, device=DEV) * scale).to(dtype)


def close(a, b, atol, rtol=2e-2):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), atol=atol, rtol=rtol)


@pytest.mark.parametrize("H,rows", [(8192, 1), (8192, 5), (4096, 33), (512, 3)])
def test_rmsnorm(H, rows):
    x, w = rnd(rows, H), rnd(H, scale=0.5) + 1
    r = rnd(rows, H)
    got = ops.rmsnorm(x, w, 1e-5)
    want, _ = ref.rmsnorm(x.cpu(), w.cpu(), 1e-5)
    close(got, want, 2e-2)
    r_gpu, r_cpu = r.clone(), r.cpu().clone()
    got = ops.rmsnorm(x, w, 1e-5, residual=r_gpu)
    want, _ = ref.rmsnorm(x.cpu(), w.cpu(), 1e-5, residual=r_cpu)
    close(r_gpu, r_cpu, 0, 0)
    close(got, want, 2e-2)


@pytest.mark.parametrize("nq,nkv", [(8, 1), (64, 8), (16, 2)])
def test_rope_kv_write_prefill_and_decode(nq, nkv):
    D, T, bs = 128, 37, 16
    scaling = dict(rope_type="llama3", factor=8.0, low_freq_factor=1.0, high_freq_factor=4.0,
                   original_max_position_embeddings=8192)
    cs = ref.rope_table(D, 4096, 500000.0, scaling).to(DEV)
    qkv = rnd(T, (nq + 2 * nkv) * D)
    nslots = 64 * bs
    kc = torch.zeros(nslots, nkv, D, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(nslots, device=DEV)[:T].int()
    slots[3] = -1
    q = ops.rope_kv_write(qkv, cs, kc, vc, nq, nkv, D, positions=pos, slot_mapping=slots)
    kr, vr = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    qr = ref.rope_kv_write(qkv.cpu(), cs.cpu(), pos.cpu(), slots.cpu(), kr, vr, nq, nkv, D)
    close(q, qr.view(T, nq, D), 2e-2)
    close(kc, kr, 2e-2)
    close(vc, vr, 0, 0)
    # decode addressing: ctx lens + block tables
    B = 4
    bt = torch.randperm(64, device=DEV)[: B * 8].view(B, 8).int()
    ctx = torch.tensor([1, 17, 128, 0], device=DEV, dtype=torch.int32)
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    q2 = ops.rope_kv_write(qkv[:B], cs, kc2, vc2, nq, nkv, D, context_lens=ctx, block_tables=bt, block_size=bs)
    p, s = ref.decode_positions(ctx.cpu(), bt.cpu(), bs)
    kr2, vr2 = torch.zeros_like(kc2).cpu(), torch.zeros_like(vc2).cpu()
    qr2 = ref.rope_kv_write(qkv[:B].cpu(), cs.cpu(), p, s, kr2, vr2, nq, nkv, D)
    close(q2[:3], qr2.view(B, nq, D)[:3], 2e-2)
    close(kc2, kr2, 2e-2)


def _paged_cache(nkv, D, bs, nblocks, gen=None):
    kc = rnd(nblocks * bs, nkv, D, gen=gen)
    vc = rnd(nblocks * bs, nkv, D, gen=gen)
    return kc, vc


@pytest.mark.parametrize("nq,nkv", [(8, 1), (64, 8), (32, 8), (16, 16)])
@pytest.mark.parametrize("ctxs", [[1, 5, 300], [1000, 2, 513], [4097]])
def test_paged_decode_attention(nq, nkv, ctxs):
    D, bs = 128, 16
    B = len(ctxs)
    maxb = (max(ctxs) + bs - 1) // bs
    nblocks = B * maxb + 3
    kc, vc = _paged_cache(nkv, D, bs, nblocks)
    bt = torch.randperm(nblocks, device=DEV)[: B * maxb].view(B, maxb).int()
    ctx = torch.tensor(ctxs, device=DEV, dtype=torch.int32)
    q = rnd(B, nq, D)
    scale = 1 / math.sqrt(D)
    for max_context in (max(ctxs), 8192):
        got = ops.paged_decode_attention(q, kc, vc, bt, ctx, scale, bs, max_context)
        want = ref.paged_decode_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), ctx.cpu(), scale, bs)
        close(got, want, 2e-2)


@pytest.mark.parametrize("nq,nkv", [(8, 1), (64, 8), (4, 2)])
@pytest.mark.parametrize("qlens,cached", [([37], [0]), ([130, 1, 64], [0, 5, 17]), ([200], [160])])
def test_paged_prefill_attention(nq, nkv, qlens, cached):
    _prefill_attention_case(nq, nkv, qlens, cached)


@pytest.mark.parametrize("nq,nkv,qlens,cached", [(64, 8, [600, 45], [1200, 30]), (8, 1, [4100], [0]),
                                                 (64, 8, [513], [3000]), (64, 8, [2100], [500])])
def test_paged_prefill_attention_wide_workgroups(nq, nkv, qlens, cached):
    """Grids of >= 256 eight-wave workgroups (16 queries x 8 heads at 8:1 GQA) take the 8-wave form: long contexts,
    several sequences, a chunk after a long cached prefix."""
    G = nq // nkv
    assert -(-max(qlens) // (128 // G)) * nkv * len(qlens) >= 256
    _prefill_attention_case(nq, nkv, qlens, cached)


def test_paged_prefill_attention_sixteen_wave_subprocess():
    """The opt-in 16-wave form (32 queries x 8 heads per workgroup) against the fp32 oracle, in a child process
    (the wave count is read from K8S_PREFILL_ATTN_WAVES once per process)."""
    import subprocess
    import sys

    code = (f"import sys; sys.path.insert(0, {os.path.dirname(os.path.abspath(__file__))!r}); import test_kernels_gpu as t; "
            "t._prefill_attention_case(64, 8, [600, 45], [1200, 30]); t._prefill_attention_case(8, 1, [300], [20])")
    r = subprocess.run([sys.executable, "-c", code], env={**os.environ, "K8S_PREFILL_ATTN_WAVES": "16"},
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]


def _prefill_attention_case(nq, nkv, qlens, cached):
    D, bs = 128, 16
    S = len(qlens)
    ctxs = [q + c for q, c in zip(qlens, cached)]
    maxb = (max(ctxs) + bs - 1) // bs
    nblocks = S * maxb + 2
    kc, vc = _paged_cache(nkv, D, bs, nblocks)
    bt = torch.randperm(nblocks, device=DEV)[: S * maxb].view(S, maxb).int()
    cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), device=DEV, dtype=torch.int32)
    ctx = torch.tensor(ctxs, device=DEV, dtype=torch.int32)
    q = rnd(sum(qlens), nq, D)
    scale = 1 / math.sqrt(D)
    got = ops.paged_prefill_attention(q, kc, vc, cu, ctx, bt, scale, bs, max(qlens))
    want = ref.paged_prefill_attention(q.cpu(), kc.cpu(), vc.cpu(), cu.cpu(), ctx.cpu(), bt.cpu(), scale, bs)
    close(got, want, 2e-2)


def test_prefill_attention_spike_forces_rescale():
    """T13-style: a late key with a huge score forces the online-softmax rescale branch."""
    nq, nkv, D, bs = 8, 1, 128, 16
    L = 300
    kc, vc = _paged_cache(nkv, D, bs, 32)
    bt = torch.arange(32, device=DEV, dtype=torch.int32).view(1, 32)
    q = rnd(L, nq, D)
    kc[250, 0] = q[280, 3] * 4  # key 250 dominates query 280 / head 3
    cu = torch.tensor([0, L], device=DEV, dtype=torch.int32)
    ctx = torch.tensor([L], device=DEV, dtype=torch.int32)
    got = ops.paged_prefill_attention(q, kc, vc, cu, ctx, bt, 1 / math.sqrt(D), bs, L)
    want = ref.paged_prefill_attention(q.cpu(), kc.cpu(), vc.cpu(), cu.cpu(), ctx.cpu(), bt.cpu(), 1 / math.sqrt(D), bs)
    close(got, want, 2e-2)


@pytest.mark.parametrize("M", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("N,K", [(1280, 8192), (8192, 1024), (16032, 8192), (8192, 3584), (96, 512)])
def test_gemv(M, N, K):
    """The GEMV kernel at every row count it accepts, and ops.linear's routing (GEMV up to GEMV_MAX_M rows,
    mgemm above) at the same shapes."""
    x, w = rnd(M, K), rnd(N, K, scale=0.05)
    want = ref.linear(x.cpu(), w.cpu())
    want32 = ref.linear(x.cpu(), w.cpu(), torch.float32)
    close(ops._gemv(x, w, ops.EPI_BF16, torch.bfloat16), want, 3e-2)
    close(ops._gemv(x, w, ops.EPI_F32, torch.float32), want32, 1e-2, 1e-3)
    close(ops.linear(x, w), want, 3e-2)
    close(ops.linear(x, w, out_dtype=torch.float32), want32, 1e-2, 1e-3)


@pytest.mark.parametrize("M", [1, 4, 8])
@pytest.mark.parametrize("I,K", [(3584, 8192), (128, 512)])
def test_gemv_swiglu(M, I, K):
    x, w = rnd(M, K), rnd(2 * I, K, scale=0.05)
    want = ref.linear_swiglu(x.cpu(), w.cpu())
    close(ops._gemv(x, w, ops.EPI_SWIGLU, torch.bfloat16), want, 3e-2)
    close(ops.linear_swiglu(x, w), want, 3e-2)


def test_prefill_linear_and_silu_mul():
    x, w = rnd(300, 1024), rnd(2 * 512, 1024, scale=0.05)
    close(ops.linear_swiglu(x, w), ref.linear_swiglu(x.cpu(), w.cpu()), 3e-2)


def test_embedding():
    table = rnd(1000, 512)
    ids = torch.tensor([0, 999, 5, 5, 17], device=DEV, dtype=torch.int32)
    close(ops.embedding(ids, table), ref.embedding(ids.cpu(), table.cpu()), 0, 0)


def test_sampler_greedy_and_state_update():
    B, V = 3, 128256
    logits = torch.randn(B, V, device=DEV)
    logits[1, 77777] = 50.0
    t = torch.zeros(B, device=DEV)
    p = torch.ones(B, device=DEV)
    seeds = torch.arange(B, device=DEV, dtype=torch.int32)
    ctx = torch.tensor([5, 9, 0], device=DEV, dtype=torch.int32)
    hist = torch.full((B, 4), -1, device=DEV, dtype=torch.int32)
    steps = torch.zeros(B, device=DEV, dtype=torch.int32)
    toks = torch.zeros(B, device=DEV, dtype=torch.int32)
    ops.sample(logits, t, p, seeds, ctx, tokens_out=toks, ctx_inc=ctx, hist=hist, steps=steps)
    want = logits.argmax(-1).int()
    assert toks[:2].tolist() == want[:2].tolist() and toks[1].item() == 77777
    assert ctx.tolist() == [6, 10, 0] and steps.tolist() == [1, 1, 0] and hist[:, 0].tolist()[:2] == want[:2].tolist()


def test_sampler_sharded_layout_matches_flat():
    S, B, Vs = 8, 2, 16032
    logits = torch.randn(S, B, Vs, device=DEV)
    flat = logits.permute(1, 0, 2).reshape(B, S * Vs).contiguous()
    t = torch.full((B,), 0.7, device=DEV)
    p = torch.tensor([1.0, 0.9], device=DEV)
    seeds = torch.tensor([11, 12], device=DEV, dtype=torch.int32)
    ctr = torch.tensor([3, 4], device=DEV, dtype=torch.int32)
    a = ops.sample(logits, t, p, seeds, ctr, shards=S)
    b = ops.sample(flat, t, p, seeds, ctr)
    assert a.tolist() == b.tolist()


def test_sampler_matches_reference_and_distribution():
    V = 64
    logits = torch.randn(1, V, device=DEV, generator=torch.Generator(DEV).manual_seed(0)) * 2
    t = torch.tensor([0.8], device=DEV)
    for top_p in (1.0, 0.5):
        p = torch.tensor([top_p], device=DEV)
        agree = 0
        counts = torch.zeros(V)
        N = 4000
        for c in range(N):
            ctr = torch.tensor([c], device=DEV, dtype=torch.int32)
            seeds = torch.tensor([1234], device=DEV, dtype=torch.int32)
            tok = int(ops.sample(logits, t, p, seeds, ctr)[0])
            if c < 200:
                agree += tok == int(ref.sample(logits.cpu(), t.cpu(), p.cpu(), seeds.cpu(), ctr.cpu())[0])
            counts[tok] += 1
        assert agree >= 195
        probs = torch.softmax(logits[0].cpu() / 0.8, -1)
        if top_p < 1:
            keep = ref.nucleus_mask(logits[0].cpu(), 0.8, top_p).nonzero().flatten()
            order = torch.argsort(probs, descending=True)
            exact = order[: int((probs[order].cumsum(0) < top_p).sum()) + 1]
            assert set(exact.tolist()) <= set(keep.tolist()) and len(keep) <= len(exact) + 1   # bin ties only
            assert counts[keep].sum() == N            # never samples outside the nucleus
            probs = torch.zeros_like(probs).index_put_((keep,), probs[keep])
            probs /= probs.sum()
        emp = counts / N
        assert (emp - probs).abs().sum() < 0.12       # L1 distance (expected ~0.05 at N=4000)


@pytest.mark.parametrize("shards", [1, 8])
def test_nucleus_full_vocab_matches_reference(shards):
    """Multi-workgroup nucleus passes on a Llama-3 sized vocabulary (sharded like the TP=8 LM head),
    rows of different temperature / top_p mixed with a Gumbel and a greedy row, eager and replayed from
    a hipGraph: the token matches the CPU reference and lies in its nucleus."""
    V, B = 128256, 4
    g = torch.Generator(DEV).manual_seed(5)
    flat = torch.randn(B, V, device=DEV, generator=g) * torch.tensor([[3.0], [1.0], [2.0], [2.0]], device=DEV)
    logits = flat.reshape(B, shards, V // shards).permute(1, 0, 2).contiguous() if shards > 1 else flat
    t = torch.tensor([0.3, 1.0, 0.7, 0.0], device=DEV)
    p = torch.tensor([0.9, 0.5, 1.0, 0.9], device=DEV)
    seeds = torch.tensor([1, 2, 3, 4], device=DEV, dtype=torch.int32)
    agree = 0
    for c in range(12):
        ctr = torch.full((B,), c, device=DEV, dtype=torch.int32)
        got = ops.sample(logits, t, p, seeds, ctr, shards=shards).cpu()
        want = ref.sample(flat.cpu(), t.cpu(), p.cpu(), seeds.cpu(), ctr.cpu())
        agree += int((got == want).sum())
        for b in (0, 1):
            assert bool(ref.nucleus_mask(flat[b].cpu(), float(t[b]), float(p[b]))[int(got[b])])
        assert int(got[3]) == int(flat[3].argmax())
    assert agree >= 12 * B - 2
    # graph replay: the memset node re-arms the row state every replay
    ctr = torch.full((B,), 3, device=DEV, dtype=torch.int32)
    out = torch.zeros(B, device=DEV, dtype=torch.int32)
    exp = ops.sample(logits, t, p, seeds, ctr, shards=shards, nucleus=True).clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.sample(logits, t, p, seeds, ctr, shards=shards, tokens_out=out, nucleus=True)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        ops.sample(logits, t, p, seeds, ctr, shards=shards, tokens_out=out, nucleus=True)
    for _ in range(3):
        out.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert out.tolist() == exp.tolist()


def test_nucleus_scratch_shared_across_batch_sizes():
    """One nucleus scratch buffer serves every batch size: top_p < 1 at B=1, then B=8, then B=3 on the same
    buffer give the tokens of a run on a fresh buffer, and the row state is zero again afterwards (the
    histograms of a small batch must never land in a larger batch's row state)."""
    V = 128256
    g = torch.Generator(DEV).manual_seed(11)
    flat = torch.randn(8, V, device=DEV, generator=g) * 2.0
    t = torch.full((8,), 0.7, device=DEV)
    p = torch.tensor([0.9, 0.5, 0.8, 0.95, 0.6, 0.9, 0.7, 0.85], device=DEV)
    seeds = torch.arange(1, 9, device=DEV, dtype=torch.int32)
    ctr = torch.full((8,), 5, device=DEV, dtype=torch.int32)
    fresh = {}
    for B in (1, 8, 3):
        ops._SCRATCH.pop(("sample_nucleus", torch.cuda.current_device()), None)   # a fresh zeroed buffer
        fresh[B] = ops.sample(flat[:B].contiguous(), t[:B], p[:B], seeds[:B], ctr[:B], nucleus=True).cpu()
    ops._SCRATCH.pop(("sample_nucleus", torch.cuda.current_device()), None)
    ops.sample(flat[:8].contiguous(), t, p, seeds, ctr, nucleus=True)       # size the shared buffer for B=8
    for B in (1, 8, 3, 8, 1):
        got = ops.sample(flat[:B].contiguous(), t[:B], p[:B], seeds[:B], ctr[:B], nucleus=True).cpu()
        assert got.tolist() == fresh[B].tolist(), f"B={B}"
        torch.cuda.synchronize()
        buf = ops._SCRATCH[("sample_nucleus", torch.cuda.current_device())]
        rows = buf[: 4096 * 64].view(torch.int32).view(4096, 16)
        # NucRow words 4 (maxkey), 7 (cnt0), 8 (cnt1) are re-armed to zero by every launch
        assert int(rows[:, [4, 7, 8]].abs().sum()) == 0, f"row state not re-armed after B={B}"


def test_hash_init_matches_reference():
    out = torch.empty(300, 257, dtype=torch.bfloat16, device=DEV)
    ops.hash_init_(out, gcols=1000, row0=7, col0=11, seed=3, tensor_id=9, scale=0.02)
    want = ref.hash_init(300, 257, 1000, 7, 11, 3, 9, 0.02, 0.0)
    close(out, want, 0, 0)


@pytest.mark.parametrize("M", [1, 3, 8])
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("with_res", [False, True])
def test_linear_norm_fused(M, epi, with_res):
    K, N = 8192, 1280
    x = rnd(M, K)
    res_in = rnd(M, K) if with_res else None
    nw = rnd(K, scale=0.1) + 1
    w = rnd(2 * N if epi == 2 else N, K, scale=0.05)
    res_out = torch.zeros(M, K, dtype=torch.bfloat16, device=DEV)
    got = ops.linear_norm(x, w, nw, 1e-5, res_in, res_out, epi=epi)
    ro_cpu = torch.zeros(M, K, dtype=torch.bfloat16)
    want = ops.linear_norm(x.cpu(), w.cpu(), nw.cpu(), 1e-5, res_in.cpu() if with_res else None, ro_cpu, epi=epi)
    close(res_out, ro_cpu, 0, 0)
    close(got, want, 3e-2 if epi != 1 else 2e-2)


@pytest.mark.parametrize("variant", ["one-wg-1024", "one-wg-512", "small-grid-split"])
@pytest.mark.parametrize("nq,nkv", [(8, 1), (64, 8), (32, 8), (4, 2), (16, 1)])
@pytest.mark.parametrize("ctxs", [[1, 37, 600], [1024, 1025], [3000], [64, 65, 128]])
def test_decode_attention_fused(nq, nkv, ctxs, variant, monkeypatch):
    """The one-workgroup-per-pair kernel at both partition sizes (16 waves x 1024 tokens, 8 waves x 512 tokens with
    the merge kernel from 513 tokens on) and the small-grid split kernel."""
    monkeypatch.setattr(ops, "SPLIT_MAX_PAIRS", 64 if variant == "small-grid-split" else 0)
    monkeypatch.setattr(ops, "FUSED_PART_ENV", 512 if variant == "one-wg-512" else 1024)
    D, bs = 128, 16
    B = len(ctxs)
    maxb = (max(ctxs) + bs - 1) // bs
    nblocks = B * maxb + 3
    kc, vc = _paged_cache(nkv, D, bs, nblocks)
    bt = torch.randperm(nblocks, device=DEV)[: B * maxb].view(B, maxb).int()
    ctx = torch.tensor(ctxs, device=DEV, dtype=torch.int32)
    qkv = rnd(B, (nq + 2 * nkv) * D)
    scaling = dict(rope_type="llama3", factor=8.0, low_freq_factor=1.0, high_freq_factor=4.0,
                   original_max_position_embeddings=8192)
    cs = ref.rope_table(D, 4096, 500000.0, scaling).to(DEV)
    kc_ref, vc_ref = kc.cpu().clone(), vc.cpu().clone()
    for max_context in (max(ctxs), 4096):
        kc2, vc2 = kc.clone(), vc.clone()
        got = ops.decode_attention_fused(qkv, cs, kc2, vc2, bt, ctx, 1 / math.sqrt(D), bs, max_context, nq, nkv, D)
        kr, vr = kc_ref.clone(), vc_ref.clone()
        want = ops.decode_attention_fused(qkv.cpu(), cs.cpu(), kr, vr, bt.cpu(), ctx.cpu(), 1 / math.sqrt(D), bs,
                                          max_context, nq, nkv, D)
        close(got, want, 2e-2)
        close(kc2, kr, 2e-2)
        close(vc2, vr, 0, 0)


@pytest.mark.parametrize("variant", ["one-wg-1024", "one-wg-512", "small-grid-split"])
def test_decode_attention_stale_slots_do_not_leak(variant, monkeypatch):
    """The new token's cache slot and the unused slots after it hold NaN before the call: the V rows the kernels
    stage for padding keys (P = 0) must not carry them into the output (0 * NaN)."""
    monkeypatch.setattr(ops, "SPLIT_MAX_PAIRS", 64 if variant == "small-grid-split" else 0)
    monkeypatch.setattr(ops, "FUSED_PART_ENV", 512 if variant == "one-wg-512" else 1024)
    nq, nkv, D, bs = 64, 8, 128, 16
    ctxs = [1, 37, 600, 64, 65, 33]
    B = len(ctxs)
    maxb = (max(ctxs) + bs - 1) // bs + 1
    nblocks = B * maxb + 3
    kc, vc = _paged_cache(nkv, D, bs, nblocks)
    bt = torch.randperm(nblocks, device=DEV)[: B * maxb].view(B, maxb).int()
    btc = bt.cpu()
    for b, c in enumerate(ctxs):
        for t in range(c - 1, (c + bs - 1) // bs * bs):
            slot = int(btc[b, t // bs]) * bs + t % bs
            kc[slot] = float("nan")
            vc[slot] = float("nan")
    ctx = torch.tensor(ctxs, device=DEV, dtype=torch.int32)
    qkv = rnd(B, (nq + 2 * nkv) * D)
    cs = ref.rope_table(D, 4096, 500000.0, None).to(DEV)
    kr, vr = kc.cpu().clone(), vc.cpu().clone()
    got = ops.decode_attention_fused(qkv, cs, kc, vc, bt, ctx, 1 / math.sqrt(D), bs, 1024, nq, nkv, D)
    want = ops.decode_attention_fused(qkv.cpu(), cs.cpu(), kr, vr, btc, ctx.cpu(), 1 / math.sqrt(D), bs, 1024, nq,
                                      nkv, D)
    assert torch.isfinite(got).all()
    close(got, want, 2e-2)


def test_fp8_decode_matches_torch_e4m3():
    """v_cvt_pk_f32_fp8 on gfx950 decodes OCP e4m3 (torch.float8_e4m3fn) for every finite byte."""
    codes = torch.tensor([c if c not in (0x7F, 0xFF) else 0 for c in range(256)], dtype=torch.uint8)
    q = codes.repeat(16, 1).contiguous()  # 16 rows x 256
    w = ops.Fp8Weight(q.to(DEV), torch.ones(16, device=DEV))
    got = w.dequant(torch.float32).cpu()
    want = q.view(torch.float8_e4m3fn).float().bfloat16().float()
    assert torch.equal(got, want)


def test_fp8_quantize_matches_reference():
    w = rnd(256, 1024, scale=0.03)
    fw = ops.quantize_fp8(w)
    q_ref, s_ref = ref.quantize_fp8(w.cpu())
    torch.testing.assert_close(fw.scale.cpu(), s_ref, rtol=1e-6, atol=0)
    a = fw.q.cpu().view(torch.float8_e4m3fn).float()
    b = q_ref.view(torch.float8_e4m3fn).float()
    # w * (1/s) vs w / s may round differently at a tie: at most one e4m3 step, on a tiny fraction
    diff = (a - b).abs()
    assert float((diff > 0).float().mean()) < 1e-3
    assert float((diff / b.abs().clamp_min(2 ** -6)).max()) <= 0.125 + 1e-6


@pytest.mark.parametrize("M", [1, 3, 8])
@pytest.mark.parametrize("N,K", [(1280, 8192), (8192, 1024), (8192, 3584), (96, 512)])
def test_gemv_fp8(M, N, K):
    x = rnd(M, K)
    w = ops.quantize_fp8(rnd(N, K, scale=0.05))
    want = x.float().cpu() @ ref.dequant_fp8(w.q.cpu(), w.scale.cpu()).T   # exact fp32 dequant
    # the GEMV kernel itself at every row count it accepts (ops.linear routes M > GEMV_MAX_M to mgemm)
    close(ops._gemv(x, w, ops.EPI_BF16, torch.bfloat16), want.bfloat16(), 3e-2)
    close(ops._gemv(x, w, ops.EPI_F32, torch.float32), want, 1e-2, 1e-3)


@pytest.mark.parametrize("M", [1, 4])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_linear_norm_fp8(M, epi):
    K, N = 4096, 1024
    x, res = rnd(M, K), rnd(M, K)
    nw = (torch.rand(K, device=DEV) + 0.5).bfloat16()
    w = ops.quantize_fp8(rnd(2 * N if epi == 2 else N, K, scale=0.05))
    ro = torch.empty_like(x)
    got = ops.linear_norm(x, w, nw, 1e-5, res, ro, epi=epi)
    r = (x.float() + res.float()).bfloat16()
    h, _ = ref.rmsnorm(r.cpu(), nw.cpu(), 1e-5)
    wd = ref.dequant_fp8(w.q.cpu(), w.scale.cpu())
    if epi == 2:
        want = ref.linear_swiglu(h, wd)
    else:
        want = ref.linear(h, wd, torch.float32 if epi == 1 else None)
    close(got, want, 3e-2)
    close(ro, r, 1e-2)


def test_decode_attention_split_graph_replay_rearms_counters(monkeypatch):
    """The small-grid kernel's last-arriver merge must leave its arrival counters at zero: many
    captured launches in a row (as in 80 decode layers) give the same answer every time."""
    monkeypatch.setattr(ops, "SPLIT_MAX_PAIRS", 64)
    nq, nkv, D, bs, B = 8, 1, 128, 16, 2
    ctxs = [700, 129]
    maxb = 64
    kc, vc = _paged_cache(nkv, D, bs, B * maxb)
    bt = torch.arange(B * maxb, device=DEV, dtype=torch.int32).view(B, maxb)
    ctx = torch.tensor(ctxs, device=DEV, dtype=torch.int32)
    qkv = rnd(B, (nq + 2 * nkv) * D)
    cs = ref.rope_table(D, 4096, 500000.0, None).to(DEV)
    want = ops.decode_attention_fused(qkv.cpu(), cs.cpu(), kc.cpu().clone(), vc.cpu().clone(), bt.cpu(), ctx.cpu(),
                                      1 / math.sqrt(D), bs, 1024, nq, nkv, D)
    outs = []
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.decode_attention_fused(qkv, cs, kc, vc, bt, ctx, 1 / math.sqrt(D), bs, 1024, nq, nkv, D)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(6):
            outs.append(ops.decode_attention_fused(qkv, cs, kc, vc, bt, ctx, 1 / math.sqrt(D), bs, 1024, nq, nkv, D))
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    for o in outs:
        close(o, want, 2e-2)


@pytest.mark.parametrize("T,K", [(1, 8192), (300, 1024), (37, 3584), (5, 28672)])
def test_quantize_act_fp8_matches_reference(T, K):
    x = rnd(T, K, scale=2.0)
    q, s = ops.quantize_act_fp8(x)
    q_ref, s_ref = ref.quantize_fp8(x.cpu())
    torch.testing.assert_close(s.cpu(), s_ref, rtol=1e-6, atol=0)
    a = q.cpu().view(torch.float8_e4m3fn).float()
    b = q_ref.view(torch.float8_e4m3fn).float()
    diff = (a - b).abs()
    assert float((diff > 0).float().mean()) < 1e-3          # rounding ties only
    assert float((diff / b.abs().clamp_min(2 ** -6)).max()) <= 0.125 + 1e-6


@pytest.mark.parametrize("T,K", [(1, 8192), (300, 1024), (37, 3584), (64, 8192)])
def test_quantize_act_fp8_rms_folds_the_norm_into_the_scale(T, K):
    """K2 fused into K16: the RMSNorm of a row only rescales it, so the quantized bytes are x's own and the scale
    carries 1/rms -- the dequantized result equals the per-token quantization of RMSNorm(x) (CPU reference)."""
    x = rnd(T, K, scale=3.0)
    q, s = ops.quantize_act_fp8(x, rms_eps=1e-5)
    q0, s0 = ops.quantize_act_fp8(x)
    assert torch.equal(q, q0)                                  # same bytes
    inv = torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5)
    torch.testing.assert_close(s, s0 * inv, rtol=2e-6, atol=0)
    xn = (x.float() * inv[:, None]).cpu()
    back = ref.dequant_fp8(q.cpu(), s.cpu())
    assert float(((back - xn).abs() / xn.abs().amax(-1, keepdim=True)).max()) <= 2 ** -4


def test_fp8_linear_rms_runs_no_rmsnorm_kernel(monkeypatch):
    """fp8 pre-norm projections above the sgemv rows: one quantize (with the norm folded in) + the fp8 GEMM, no
    rmsnorm kernel; the result tracks quantize(RMSNorm(x)) @ W."""
    calls = []
    nat = ops.native()
    orig = nat.rmsnorm
    monkeypatch.setattr(nat, "rmsnorm", lambda *a: calls.append("rmsnorm") or orig(*a))
    M, N, K = 64, 2560, 8192
    r = rnd(M, K, scale=3.0)
    w = ops.quantize_fp8(rnd(N, K, scale=0.05))
    got = ops.linear_rms(r, w, 1e-5)
    torch.cuda.synchronize()
    assert not calls
    xn = r.float() * torch.rsqrt(r.float().pow(2).mean(-1, keepdim=True) + 1e-5)
    want = xn.cpu() @ ref.dequant_fp8(w.q.cpu(), w.scale.cpu()).T
    rel = float((got.float().cpu() - want).abs().max() / want.abs().max())
    assert rel < 0.06, rel


@pytest.mark.parametrize("M", [9, 64, 300])
@pytest.mark.parametrize("N,K", [(2560, 8192), (8192, 2048), (96, 512)])
def test_fp8_prefill_gemm(M, N, K):
    """Prefill / batched decode with fp8 weights: per-token e4m3 activations x row-scaled e4m3
    weights (fp8 MFMA GEMM) against the fp32 product of the dequantized weights."""
    x = rnd(M, K)
    w = ops.quantize_fp8(rnd(N, K, scale=0.05))
    want = x.float().cpu() @ ref.dequant_fp8(w.q.cpu(), w.scale.cpu()).T
    got = ops.linear(x, w)
    rel = float((got.float().cpu() - want).abs().max() / want.abs().max())
    assert rel < 0.06, rel                                   # e4m3 activations: ~2^-4 relative
    gu = ops.quantize_fp8(rnd(2 * N, K, scale=0.05))
    want_gu = ref.linear_swiglu(x.cpu().float(), ref.dequant_fp8(gu.q.cpu(), gu.scale.cpu()))
    got_gu = ops.linear_swiglu(x, gu)
    rel = float((got_gu.float().cpu() - want_gu.float()).abs().max() / want_gu.float().abs().max())
    assert rel < 0.08, rel


@pytest.mark.parametrize("M", [1, 3, 4, 8])
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("N", [1280, 96])
def test_linear_norm_folded(M, epi, N):
    """Decode pre-norm projection with the norm weight folded into W (the model's layout):
    y = epi((r @ (W * g).T) / rms(r)), bf16 and fp8 weights, against exact fp32 products (the
    kernel never rounds the normalised activations), and loosely against the unfolded layer."""
    K = 8192
    torch.manual_seed(1000 * M + 10 * epi + N)
    x, res = rnd(M, K), rnd(M, K)
    g = rnd(K, scale=0.1) + 1
    w = rnd(2 * N if epi == 2 else N, K, scale=0.05)
    wf = (w.float() * g.float()).bfloat16()
    ro = torch.zeros(M, K, dtype=torch.bfloat16, device=DEV)
    got = ops.linear_norm(x, wf, None, 1e-5, res, ro, epi=epi)
    r = (x.float() + res.float()).bfloat16()
    rf = r.cpu().float()
    h32 = rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + 1e-5)

    def exact(wt):
        y32 = h32 @ wt.float().T
        return torch.nn.functional.silu(y32[:, :N]) * y32[:, N:] if epi == 2 else y32

    close(ro, r, 0, 0)
    close(got, exact(wf.cpu()), 3e-2)
    # the unfolded layer it stands for: that reference rounds the normalised activations to bf16,
    # which SwiGLU's gate x up product amplifies to ~0.2-0.8 absolute at these output magnitudes (|y| up
    # to ~30); the exact check above is the numerics test, this one only guards the layout
    h, _ = ref.rmsnorm(r.cpu(), g.cpu(), 1e-5)
    unf = ref.linear_swiglu(h, w.cpu()) if epi == 2 else ref.linear(h, w.cpu(), torch.float32 if epi == 1 else None)
    close(got, unf, 1.0 if epi == 2 else 6e-2, 4e-2)
    wq = ops.quantize_fp8(wf)          # fp8 weights, folded the same way
    got8 = ops.linear_norm(x, wq, None, 1e-5, res, ro, epi=epi)
    close(got8, exact(ref.dequant_fp8(wq.q.cpu(), wq.scale.cpu())), 3e-2)


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("epi,folded", [(0, False), (1, True), (2, True), (2, False), (0, True)])
@pytest.mark.parametrize("fp8", [False, True])
def test_gemv_row_set_loop_matches_single(M, epi, folded, fp8):
    """The row-set loop (several row sets per wave, x staged once, the next set's weights in flight) gives the
    one-row-set GEMV's bits, and both match the fp32 oracle.  N is large enough for the loop to engage at 1-2
    workgroups per CU; 1283 rows leave a ragged last row set."""
    K = 8192
    torch.manual_seed(7 * M + epi + 100 * fp8)
    N = 4099 if epi != 2 else 2051
    x, res = rnd(M, K), rnd(M, K)
    w = rnd(2 * N if epi == 2 else N, K, scale=0.05)
    ww = ops.quantize_fp8(w) if fp8 else w
    wd = ref.dequant_fp8(ww.q.cpu(), ww.scale.cpu()) if fp8 else w.cpu().float()
    ro = torch.zeros(M, K, dtype=torch.bfloat16, device=DEV)
    out_dtype = torch.float32 if epi == 1 else torch.bfloat16

    def run():
        if folded:
            return ops.linear_norm(x, ww, None, 1e-5, res, ro, epi=epi)
        return ops._gemv(x, ww, epi, out_dtype)

    old = ops.native().gemv_set_loop(0)
    try:
        base = run()
        outs = []
        for lp in (1, 2):
            ops.native().gemv_set_loop(lp)
            outs.append(run())
    finally:
        ops.native().gemv_set_loop(old)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, base)
    h = x.cpu().float()
    if folded:
        rf = (x.float() + res.float()).bfloat16().cpu().float()
        h = rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + 1e-5)
    y32 = h @ wd.T
    want = torch.nn.functional.silu(y32[:, :N]) * y32[:, N:] if epi == 2 else y32
    close(base, want, 3e-2)


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("fp8", [False, True])
def test_gemv_wide_loop_large_k_matches_single(M, fp8):
    """The 8-wave row-set loop of the large-K plain projections (down: x takes >= 32 KiB of LDS) gives the bits of
    the 4-wave loop and of one row set per wave, and matches the fp32 oracle."""
    K, N = 28672, 4103
    torch.manual_seed(11 * M + fp8)
    x = rnd(M, K)
    w = rnd(N, K, scale=0.05)
    ww = ops.quantize_fp8(w) if fp8 else w
    wd = ref.dequant_fp8(ww.q.cpu(), ww.scale.cpu()) if fp8 else w.cpu().float()
    old_loop, old_wide = ops.native().gemv_set_loop(0), ops.native().gemv_set_wide(1)
    try:
        base = ops._gemv(x, ww, ops.EPI_BF16, torch.bfloat16)
        outs = []
        for lp, wide in ((1, 1), (2, 1), (2, 0)):
            ops.native().gemv_set_loop(lp)
            ops.native().gemv_set_wide(wide)
            outs.append(ops._gemv(x, ww, ops.EPI_BF16, torch.bfloat16))
    finally:
        ops.native().gemv_set_loop(old_loop)
        ops.native().gemv_set_wide(old_wide)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, base)
    close(base, x.cpu().float() @ wd.T, 3e-2)
