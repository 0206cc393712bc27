"""Cascade (shared-prefix) decode attention: decode_prefix_kernel attends the batch's shared prefix once for every
row and the per-row kernel merges its partials (attn_decode_fused.hip).  Checked against the per-row kernel on the
same inputs and against the fp32 PyTorch oracle (ops/reference.py): every GQA group size, 2 / 16 / 64 rows, one
partition (<= 1024 tokens) and several (the merge kernel), an idle row, no shared spans (bit-identical to the plain
kernel), the MX output (bit-equal to quantizing the bf16 output) and graph replay with the shared length changed
between replays."""

import math

import pytest
import torch

from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
D, BS = 128, 16


def _rnd(*shape, gen=None):
    return torch.randn(*shape, generator=gen, device=DEV).to(torch.bfloat16)


def _batch(B, nq, nkv, prefix, suffixes, seed=0, idle=()):
    """B rows whose block tables start with the same prefix // 16 blocks, then blocks of their own."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    pb = prefix // BS
    own = [(prefix + s + BS - 1) // BS - pb + 1 for s in suffixes]
    maxb = pb + max(own)
    nblocks = pb + sum(own) + 2
    kc, vc = _rnd(nblocks * BS, nkv, D, gen=g), _rnd(nblocks * BS, nkv, D, gen=g)
    perm = torch.randperm(nblocks, generator=torch.Generator().manual_seed(seed)).tolist()
    shared, rest = perm[:pb], perm[pb:]
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    for b in range(B):
        mine, rest = rest[:own[b]], rest[own[b]:]
        row = shared + mine
        bt[b, :len(row)] = torch.tensor(row, dtype=torch.int32)
    ctx = torch.tensor([0 if b in idle else prefix + suffixes[b] for b in range(B)], dtype=torch.int32)
    qkv = _rnd(B, (nq + 2 * nkv) * D, gen=g)
    cs = ref.rope_table(D, 8192, 500000.0, None).to(DEV)
    return qkv, cs, kc, vc, bt.to(DEV), ctx.to(DEV)


def _run(qkv, cs, kc, vc, bt, ctx, mc, nq, nkv, cascade=None, mx=False):
    return ops.decode_attention_fused(qkv, cs, kc, vc, bt, ctx, 1 / math.sqrt(D), BS, mc, nq, nkv, D, mx=mx,
                                      cascade=cascade)


def _close(a, b, tol=2e-2):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), atol=tol, rtol=tol)


@pytest.mark.parametrize("nq,nkv", [(64, 8), (8, 1), (32, 8), (16, 1), (4, 2), (4, 4)])
@pytest.mark.parametrize("B", [2, 16, 64])
@pytest.mark.parametrize("mc", [1024, 4096])
def test_cascade_equals_per_row_attention(nq, nkv, B, mc):
    prefix = 640 if mc == 1024 else 2560
    gen = torch.Generator().manual_seed(B)
    suffixes = torch.randint(1, 300 if mc == 1024 else 1000, (B,), generator=gen).tolist()
    suffixes[0] = 1                                   # a row whose new token directly follows the prefix
    idle = (B - 1,) if B > 2 else ()                  # an idle slot (context 0) inside the batch
    qkv, cs, kc, vc, bt, ctx = _batch(B, nq, nkv, prefix, suffixes, seed=B + nq, idle=idle)
    assert int(ctx.max()) <= mc
    cas = torch.tensor([prefix // 64, 0], dtype=torch.int32, device=DEV)
    ngm = ops.cascade_groups_max(B, nq, nkv)
    kc1, vc1, kc2, vc2 = kc.clone(), vc.clone(), kc.clone(), vc.clone()
    got = _run(qkv, cs, kc1, vc1, bt, ctx, mc, nq, nkv, cascade=(cas, ngm))
    base = _run(qkv, cs, kc2, vc2, bt, ctx, mc, nq, nkv)
    torch.cuda.synchronize()
    live = [b for b in range(B) if b not in idle]
    _close(got[live], base[live])
    assert torch.equal(kc1, kc2) and torch.equal(vc1, vc2), "the new tokens' K/V writes differ"
    if mc > 1024 and max(suffixes) < 1024:   # the engine's suffix context class: one partition past the prefix
        short = _run(qkv, cs, kc.clone(), vc.clone(), bt, ctx, 1024, nq, nkv, cascade=(cas, ngm))
        _close(short[live], base[live])
    if B <= 16:   # the fp32 oracle too
        kr, vr = kc.cpu().clone(), vc.cpu().clone()
        want = _run(qkv.cpu(), cs.cpu(), kr, vr, bt.cpu(), ctx.cpu(), mc, nq, nkv)
        _close(got[live], want[live])


def test_cascade_without_shared_spans_is_the_plain_kernel():
    nq, nkv, B = 64, 8, 16
    qkv, cs, kc, vc, bt, ctx = _batch(B, nq, nkv, 320, [5 + 7 * b for b in range(B)], seed=3)
    assert int(ctx.max()) <= 1024
    cas = torch.zeros(2, dtype=torch.int32, device=DEV)
    got = _run(qkv, cs, kc.clone(), vc.clone(), bt, ctx, 1024, nq, nkv, cascade=(cas, 8))
    base = _run(qkv, cs, kc.clone(), vc.clone(), bt, ctx, 1024, nq, nkv)
    assert torch.equal(got, base)


@pytest.mark.parametrize("mc", [1024, 4096])
def test_cascade_mx_output_is_the_quantized_bf16_output(mc):
    nq, nkv, B = 64, 8, 16
    prefix = 512 if mc == 1024 else 2048
    step = 29 if mc == 1024 else 37     # (every context within max_context)
    qkv, cs, kc, vc, bt, ctx = _batch(B, nq, nkv, prefix, [1 + step * b for b in range(B)], seed=5)
    assert int(ctx.max()) <= mc
    cas = torch.tensor([prefix // 64, 3], dtype=torch.int32, device=DEV)
    ngm = ops.cascade_groups_max(B, nq, nkv)
    bf = _run(qkv, cs, kc.clone(), vc.clone(), bt, ctx, mc, nq, nkv, cascade=(cas, ngm))
    mx = _run(qkv, cs, kc.clone(), vc.clone(), bt, ctx, mc, nq, nkv, cascade=(cas, ngm), mx=True)
    want = ops.quantize_act_mx(bf)
    assert torch.equal(mx.q, want.q) and torch.equal(mx.e, want.e)


@pytest.mark.parametrize("mc", [1024, 4096])
def test_cascade_graph_replay_follows_the_shared_length(mc):
    """The shared length is device state the engine writes before a replay: one graph serves every length (mc 1024:
    one partition past the prefix, 4096: several and the merge kernel)."""
    nq, nkv, B = 64, 8, 16
    prefix = 1536
    qkv, cs, kc, vc, bt, ctx = _batch(B, nq, nkv, prefix, [3 + 50 * b for b in range(B)], seed=7)
    shs = (prefix // 64, 7, 0, 1, prefix // 64) if mc > 1024 else (prefix // 64, 20, 22, prefix // 64)
    assert int(ctx.max()) - 64 * min(shs) <= mc            # every row's suffix fits max_context
    cas = torch.tensor([prefix // 64, 0], dtype=torch.int32, device=DEV)
    ngm = ops.cascade_groups_max(B, nq, nkv)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _run(qkv, cs, kc, vc, bt, ctx, mc, nq, nkv, cascade=(cas, ngm))
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = _run(qkv, cs, kc, vc, bt, ctx, mc, nq, nkv, cascade=(cas, ngm))
    base = _run(qkv, cs, kc.clone(), vc.clone(), bt, ctx, 4096, nq, nkv)
    for sh in shs:
        cas[0] = sh
        g.replay()
        torch.cuda.synchronize()
        _close(out, base)


def test_engine_batched_decode_takes_the_cascade_and_decides_the_same():
    """Pods decided against one cluster snapshot with the cluster-first layout share their prompt up to the pod
    block: the engine's decode chunks take the cascade graphs, and the greedy answers match per-row attention (up
    to near-ties of the random-weight logits: the summation order differs)."""
    from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine

    eng = build_engine("tiny", device="cuda:0", max_batch=8, num_blocks=2048, max_model_len=2048, seed=3)
    shared = " ".join(f"node-{i} cpu {i % 7} cores free, memory {i % 5} GiB free;" for i in range(60))
    p = SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True)
    eng.generate([shared + " warm-up pod"], p)            # the shared prefix is now in the prefix cache
    prompts = [shared + f" pod-{i} requests {i + 1} cores" for i in range(6)]
    assert len(eng.tok.encode(prompts[0])) > eng.cascade_min + 64
    a = eng.generate(prompts, p)
    assert eng.stats["cascade_chunks"] > 0 and eng.stats["graph_replays"] > 0
    eng.cascade = False
    b = eng.generate(prompts, p)
    same = sum(x == y for oa, ob in zip(a, b) for x, y in zip(oa.token_ids, ob.token_ids))
    assert same >= 0.9 * sum(len(o.token_ids) for o in a), (same, [o.token_ids for o in a], [o.token_ids for o in b])
