"""T5 engine tests on CPU (reference ops): model correctness vs a dense un-paged Llama forward,
prefill/decode consistency, prefix caching, stops, aborts, deadlines, checkpoint round trip,
tokenizer and the native block allocator."""

import math
import time

import pytest
import torch

from k8s_llm_scheduler_amd import ops
from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine
from k8s_llm_scheduler_amd.engine.tokenizer import Tokenizer
from k8s_llm_scheduler_amd.models.config import PRESETS
from k8s_llm_scheduler_amd.models.llama import LlamaModel, save_hf_checkpoint
from k8s_llm_scheduler_amd.ops import reference as ref


def dense_llama_logits(m: LlamaModel, ids):
    """Independent textbook forward (no paging, no fused ops) for the LAST position."""
    c = m.cfg
    x = m.embed[torch.tensor(ids)].float()
    T = len(ids)
    cs = ref.rope_table(c.head_dim, T, c.rope_theta, c.rope_scaling)
    mask = torch.full((T, T), float("-inf")).triu(1)

    def norm(v, w):
        v = v.to(torch.bfloat16).float()
        return (v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + c.rms_eps) * w.float()).to(torch.bfloat16).float()

    def rot(v):
        h = v.shape[-1] // 2
        cc, ss = cs[:, None, :h], cs[:, None, h:]
        return torch.cat([v[..., :h] * cc - v[..., h:] * ss, v[..., h:] * cc + v[..., :h] * ss], -1)

    D, nq, nkv = c.head_dim, c.num_heads, c.num_kv_heads
    for w in m.layers:
        h = norm(x, w.ln1)
        qkv = (h @ w.wqkv.float().T).to(torch.bfloat16).float()
        q = rot(qkv[:, :nq * D].view(T, nq, D)).to(torch.bfloat16).float()
        k = rot(qkv[:, nq * D:(nq + nkv) * D].view(T, nkv, D)).to(torch.bfloat16).float()
        v = qkv[:, (nq + nkv) * D:].view(T, nkv, D)
        k = k.repeat_interleave(nq // nkv, 1)
        v = v.repeat_interleave(nq // nkv, 1)
        att = torch.softmax(torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(D) + mask, -1)
        a = torch.einsum("hqk,khd->qhd", att, v).reshape(T, nq * D).to(torch.bfloat16).float()
        x = (x + (a @ w.wo.float().T).to(torch.bfloat16).float()).to(torch.bfloat16).float()
        h = norm(x, w.ln2)
        gu = h @ w.wgu.float().T
        g = (torch.nn.functional.silu(gu[:, :m.I]) * gu[:, m.I:]).to(torch.bfloat16).float()
        x = (x + (g @ w.wdown.float().T).to(torch.bfloat16).float()).to(torch.bfloat16).float()
    h = norm(x[-1:], m.norm)
    return (h @ m.lm_head.float().T)[0]


@pytest.fixture(scope="module")
def tiny():
    return LlamaModel(PRESETS["tiny"], device="cpu", seed=3, max_model_len=512)


def _prefill(m, ids, bs=16, nblocks=64):
    m.allocate_kv(nblocks, bs)
    T = len(ids)
    blocks = list(range(math.ceil((T + 4) / bs)))
    bt = torch.zeros(1, 32, dtype=torch.int32)
    bt[0, :len(blocks)] = torch.tensor(blocks)
    i32 = lambda x: torch.tensor(x, dtype=torch.int32)
    slots = [blocks[p // bs] * bs + p % bs for p in range(T)]
    lg = m.forward_prefill(i32(ids), i32(list(range(T))), i32(slots), i32([0, T]), i32([T]), bt, T, i32([T - 1]))
    return lg, bt


def test_prefill_matches_dense_reference(tiny):
    ids = [5, 17, 200, 3, 3000, 42, 7, 9, 11, 1000, 15, 16, 300, 301, 302, 303, 12, 13]
    lg, _ = _prefill(tiny, ids)
    want = dense_llama_logits(tiny, ids)
    assert lg.shape == (1, 1, tiny.cfg.vocab)
    torch.testing.assert_close(lg[0, 0], want, atol=5e-2, rtol=5e-2)
    assert int(lg[0, 0].argmax()) == int(want.argmax())


def test_decode_step_matches_prefill(tiny):
    ids = list(range(100, 140))
    lg_full, _ = _prefill(tiny, ids + [777])
    _, bt = _prefill(tiny, ids)
    ctx = torch.tensor([len(ids) + 1], dtype=torch.int32)
    lg_dec = tiny.forward_decode(torch.tensor([777], dtype=torch.int32), ctx, bt, 512)
    torch.testing.assert_close(lg_dec, lg_full, atol=5e-2, rtol=5e-2)


def test_random_init_is_device_and_tp_independent():
    c = PRESETS["tiny"]
    a = ref.hash_init(64, 32, 256, 64, 0, 1, 2, 0.1, 0.0)
    b = ref.hash_init(128, 32, 256, 0, 0, 1, 2, 0.1, 0.0)[64:]
    assert torch.equal(a, b)
    assert c.params > 0


def test_checkpoint_roundtrip(tmp_path, tiny):
    save_hf_checkpoint(tiny, tmp_path / "ckpt")
    m2 = LlamaModel(tiny.cfg, device="cpu", weights=str(tmp_path / "ckpt"), max_model_len=512)
    for a, b in zip(tiny.layers, m2.layers):
        assert torch.equal(a.wqkv, b.wqkv) and torch.equal(a.wgu, b.wgu) and torch.equal(a.wdown, b.wdown)
    assert torch.equal(tiny.lm_head, m2.lm_head)


@pytest.fixture(scope="module")
def engine():
    return build_engine("tiny", device="cpu", max_batch=4, max_model_len=512, num_blocks=200, seed=1)


def test_generate_deterministic_with_seed(engine):
    p = SamplingParams(max_tokens=6, temperature=0.7, seed=5, ignore_eos=True)
    a = engine.generate(["hello kubernetes"], p)[0]
    b = engine.generate(["hello kubernetes"], p)[0]
    assert a.token_ids == b.token_ids and len(a.token_ids) == 6 and a.finish_reason == "length"


def test_batched_equals_single(engine):
    p = SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True)
    prompts = ["pod one needs cpu", "a much longer prompt about node kind-worker2 and memory", "x"]
    singles = [engine.generate([q], p)[0].token_ids for q in prompts]
    batched = [o.token_ids for o in engine.generate(prompts, p)]
    assert singles == batched


def test_prefix_cache_hit(engine):
    sys_msg = "You are an intelligent Kubernetes scheduler. " * 8
    p = SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True)
    a = engine.generate([engine.render_chat(sys_msg, "pod A")], p)[0]
    b = engine.generate([engine.render_chat(sys_msg, "pod B")], p)[0]
    assert a.cached_tokens == 0 and b.cached_tokens >= 48
    # cached result equals an uncached computation of the same prompt
    engine.allocator.reset_prefix_cache()
    c = engine.generate([engine.render_chat(sys_msg, "pod B")], p)[0]
    assert c.cached_tokens == 0 and c.token_ids == b.token_ids


def test_eos_stop(engine):
    eos = engine.tok.eot_id
    saved = engine.model.lm_head[eos].clone()
    engine.model.lm_head[eos] = 1.0  # make EOS win the greedy choice
    try:
        o = engine.generate(["anything"], SamplingParams(max_tokens=10, temperature=0.0))[0]
    finally:
        engine.model.lm_head[eos] = saved
    assert o.finish_reason == "stop" and o.token_ids == []


def test_deadline_and_abort(engine):
    with pytest.raises(TimeoutError):
        engine.generate(["slow"], SamplingParams(max_tokens=50, ignore_eos=True), deadline=time.monotonic() - 1)
    assert not engine.has_work() and engine.allocator.num_free == engine.allocator.num_blocks - engine.allocator.num_cached \
        or engine.allocator.num_free > 0


def test_tokenizer_roundtrip_and_template():
    tok = Tokenizer(model_vocab=128256)
    text = 'Select the best node from [kind-worker, kind-worker2] and respond with JSON only: {"a": 1}'
    assert tok.decode(tok.encode(text)) == text
    ids = tok.chat_ids("sys", "user msg")
    assert ids[0] == 128000 and ids.count(128009) == 2 and ids[-1] != 128009
    assert tok.decode([128000, *tok.encode("hi"), 128009]) == "hi"


def test_block_allocator_prefix_and_eviction():
    A = ops.native().BlockAllocator(6, 4, True)
    t = list(range(13))
    a = A.allocate(t, 14)                         # 4 blocks
    assert a.cached_tokens == 0 and A.num_free == 2
    A.commit_prefix(a.blocks, t, 13)              # 3 full blocks published
    b = A.allocate(t, 14)                         # shares 3 blocks (last token recomputed)
    assert b.cached_tokens == 12 and b.blocks[:3] == a.blocks[:3] and A.num_free == 1
    assert A.refcount(a.blocks[0]) == 2
    A.release(a.blocks)
    A.release(b.blocks)
    assert A.num_free == 6 and A.num_cached == 3  # cached blocks stay (evictable)
    c = A.allocate(list(range(100, 124)), 24)     # needs all 6 -> evicts the cached ones
    assert len(c.blocks) == 6 and A.num_cached == 0
    with pytest.raises(RuntimeError):
        A.allocate([1], 4)
    with pytest.raises(Exception):
        A.release([c.blocks[0], c.blocks[0]])


def test_block_allocator_sub_block_prefix():
    """Sub-block prefix hits: after the full-block hits, the longest run of leading tokens shared with a cached block
    under the same parent chain is reported for copying (never the last prompt token); evicted blocks leave the
    index."""
    A = ops.native().BlockAllocator(8, 4, True)
    t = list(range(10))                           # [0-3] [4-7] [8 9]
    a = A.allocate(t, 12)
    A.commit_prefix(a.blocks, t, 10)              # 2 full blocks published
    u = [0, 1, 2, 3, 4, 5, 9, 9, 1]
    b = A.allocate(u, 12)                         # block 0 shared, then tokens 4, 5 of block 1
    assert (b.cached_tokens, b.copy_src, b.copy_tokens) == (6, a.blocks[1], 2)
    assert b.blocks[0] == a.blocks[0] and b.blocks[1] != a.blocks[1]
    c = A.allocate([0, 1, 2, 3, 4, 5], 8)         # the last prompt token (5) is recomputed
    assert (c.cached_tokens, c.copy_tokens) == (5, 1)
    d = A.allocate([7, 1, 2], 4)                  # nothing shared
    assert (d.cached_tokens, d.copy_src, d.copy_tokens) == (0, -1, 0)
    for x in (a, b, c, d):
        A.release(x.blocks)
    e = A.allocate(list(range(100, 132)), 32)     # takes every block: the cached ones are evicted
    A.release(e.blocks)
    f = A.allocate(u, 12)
    assert (f.cached_tokens, f.copy_tokens) == (0, 0)


def test_forced_decode_emits_script_and_stops_on_json(engine):
    ans = '{"selected_node": "kind-worker2", "confidence": 0.9, "reasoning": "r"}'
    ids = engine.tok.encode(ans)
    o = engine.generate(["pick a node"], SamplingParams(max_tokens=200, temperature=0.3, forced_output_ids=ids))[0]
    assert o.text == ans and o.finish_reason == "json"


def test_in_batch_prefix_sharing(engine):
    """Requests submitted together that share a long prompt prefix: the first prefills it, the
    others are admitted one step later and read it from the prefix cache; results are unchanged."""
    engine.allocator.reset_prefix_cache()
    shared = "AVAILABLE NODES: kind-worker cpu 20% mem 30% pods 4/110; kind-worker2 cpu 35% mem 10% " * 6
    prompts = [engine.render_chat("system", shared + f" POD pod-{i}") for i in range(3)]
    p = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True)
    outs = engine.generate(prompts, p)
    assert outs[0].cached_tokens == 0
    assert all(o.cached_tokens >= 2 * engine.block_size for o in outs[1:])
    engine.allocator.reset_prefix_cache()
    alone = [engine.generate([q], p)[0].token_ids for q in prompts[1:]]
    assert [o.token_ids for o in outs[1:]] == alone


def test_background_loop_batches_concurrent_callers_and_matches_sync():
    """start_background(): generate() from several threads joins one running batch; outputs equal the
    synchronous engine's (sampling is deterministic per (seed, position))."""
    import threading

    prompts = [[5, 6, 7, 8 + i] * 6 for i in range(4)]
    params = [SamplingParams(max_tokens=6, temperature=0.7, seed=11 + i, ignore_eos=True) for i in range(4)]
    sync = build_engine("tiny", device="cpu", max_batch=4, max_model_len=256, num_blocks=128, seed=1)
    want = [o.token_ids for o in sync.generate(prompts, params)]

    eng = build_engine("tiny", device="cpu", max_batch=4, max_model_len=256, num_blocks=128, seed=1)
    eng.start_background()
    got = [None] * 4

    def call(i):
        got[i] = eng.generate([prompts[i]], [params[i]])[0].token_ids

    ts = [threading.Thread(target=call, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    eng.stop_background()
    assert got == want
    assert not eng.requests and not eng.has_work()


def test_background_loop_deadline_and_engine_failure_raise():
    eng = build_engine("tiny", device="cpu", max_batch=2, max_model_len=256, num_blocks=128, seed=1)
    eng.start_background()
    try:
        with pytest.raises(TimeoutError):
            eng.generate([[1, 2, 3]], SamplingParams(max_tokens=200, ignore_eos=True), deadline=time.monotonic() + 0.01)
        real = eng.model.forward_decode

        def boom(*a, **k):
            raise RuntimeError("xGMI peer timeout (injected)")

        eng.model.forward_decode = boom
        with pytest.raises(RuntimeError, match="xGMI peer timeout"):
            eng.generate([[1, 2, 3]], SamplingParams(max_tokens=4, ignore_eos=True))
        eng.model.forward_decode = real
        out = eng.generate([[1, 2, 3]], SamplingParams(max_tokens=3, ignore_eos=True))   # still serving
        assert len(out[0].token_ids) == 3
    finally:
        eng.stop_background()


def test_checkpoint_without_tokenizer_is_rejected(tmp_path, tiny):
    """real weights are never paired with the synthetic vocabulary by accident."""
    import shutil

    from k8s_llm_scheduler_amd.engine import resolve_tokenizer
    from k8s_llm_scheduler_amd.engine.tokenizer import ASSET

    save_hf_checkpoint(tiny, tmp_path / "ckpt")
    with pytest.raises(FileNotFoundError, match="tokenizer"):
        resolve_tokenizer(str(tmp_path / "ckpt"), None)
    shutil.copy(ASSET, tmp_path / "ckpt" / "tokenizer.json")
    assert resolve_tokenizer(str(tmp_path / "ckpt"), None) == str(tmp_path / "ckpt" / "tokenizer.json")
    assert resolve_tokenizer(str(tmp_path / "ckpt"), "/x/tok.json") == "/x/tok.json"
    assert resolve_tokenizer(None, None) is None


def test_nucleus_bins_cover_exact_nucleus():
    """ref.nucleus_mask (the sampler.hip top-p rule) keeps the exact sorted-cumsum nucleus, plus at most
    the rest of its boundary bin (28/65536 of log-probability wide), for peaked and flat rows."""
    from k8s_llm_scheduler_amd.ops import reference as ref

    g = torch.Generator().manual_seed(3)
    for scale, T, P in ((3.0, 0.3, 0.9), (1.0, 1.0, 0.5), (0.2, 0.7, 0.95), (2.0, 0.5, 0.0)):
        l = torch.randn(20000, generator=g) * scale
        keep = ref.nucleus_mask(l, T, P)
        probs = torch.softmax(l.double() / T, -1)
        order = torch.argsort(probs, descending=True)
        n = int((probs[order].cumsum(0) < P).sum()) + 1
        exact = set(order[:n].tolist())
        kept = set(keep.nonzero().flatten().tolist())
        assert exact <= kept
        extra = kept - exact
        if extra:   # only boundary-bin ties: within 28/65536 in (M - l) / T of the last exact token
            lo = float(l[order[n - 1]])
            assert max((lo - float(l[i])) / T for i in extra) <= 28.0 / 65536 * 1.01


@pytest.mark.parametrize("tp,slot_kib,expect_spec", [(2, 512, False), (4, 512, False), (8, 512, True),
                                                       (4, 4096, True)])
def test_spec_verify_graph_capture_gated_on_gather_size(tp, slot_kib, expect_spec):
    """The speculative verify graph all-gathers SPEC_GRAPH_T rows of fp32 logits: at Llama-3.3-70B shapes
    (vocab 128256) that is ~2 MB at TP=2 and ~1 MB at TP=4, above a 512 KiB xGMI slot, so that graph must not
    be captured (eager verify) while one-row prefill buckets still are."""
    from types import SimpleNamespace

    from k8s_llm_scheduler_amd.engine.engine import SPEC_GRAPH_T, LLMEngine

    vocab, hidden = 128256, 8192
    xg = SimpleNamespace(slot_bytes=slot_kib << 10, max_allreduce_bytes=8 << 20)
    fake = SimpleNamespace(model=SimpleNamespace(
        tp=SimpleNamespace(world=tp, simulate=False, xgmi=xg, xgmi_max_ar=None),
        cfg=SimpleNamespace(hidden=hidden),
        lm_head=torch.empty(vocab // tp, 1)))
    assert LLMEngine._prefill_bucket_capturable(fake, 16) is True        # one logits row: 257 KB at TP=2
    got = LLMEngine._prefill_bucket_capturable(fake, SPEC_GRAPH_T, logits_rows=SPEC_GRAPH_T)
    assert got is expect_spec


@pytest.mark.parametrize("k", [1, 5, 9])
def test_forced_json_close_runs_exactly_k_decode_steps(k):
    """Device-side stop detection (sampler StopArgs): an answer whose JSON object closes at token k (token 0
    comes from the prefill) costs exactly k decode steps, whatever decode_chunk is; without it the chunk
    runs to its end."""
    eng = build_engine("tiny", device="cpu", max_batch=2, max_model_len=256, num_blocks=64, seed=1, decode_chunk=4)
    (lb,), (fill,), (rb,) = eng.tok.encode("{"), eng.tok.encode("a"), eng.tok.encode("}")
    ids = [lb] + [fill] * (k - 1) + [rb]      # the closing brace is answer token k
    p = SamplingParams(max_tokens=64, temperature=0.0, forced_output_ids=ids)
    o = eng.generate(["pick a node"], p)[0]
    assert o.finish_reason == "json" and o.token_ids == ids
    assert eng.stats["decode_steps"] == k
    eng.device_stop = False
    eng.stats["decode_steps"] = 0
    o = eng.generate(["pick a node"], p)[0]
    assert o.token_ids == ids and eng.stats["decode_steps"] == 4 * math.ceil(k / 4)


def test_device_stop_on_eos_and_max_tokens():
    eng = build_engine("tiny", device="cpu", max_batch=2, max_model_len=256, num_blocks=64, seed=1, decode_chunk=4)
    o = eng.generate(["a"], SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True))[0]
    assert len(o.token_ids) == 6 and o.finish_reason == "length" and eng.stats["decode_steps"] == 5
    eos = eng.tok.eot_id
    eng.stats["decode_steps"] = 0
    o = eng.generate(["a"], SamplingParams(max_tokens=30, temperature=0.0, forced_output_ids=[11, 12, eos, 13]))[0]
    assert o.token_ids == [11, 12] and o.finish_reason == "stop" and eng.stats["decode_steps"] == 2


def test_mixed_prefill_decode_steps_match_split_path():
    """A request arriving while others decode is prefilled in one varlen forward together with the decode rows
    (mixed step); tokens equal the split path (prefill, then decode)."""
    prompts = [[5, 6, 7, 8 + i] * (3 + 2 * i) for i in range(3)]
    params = [SamplingParams(max_tokens=20, temperature=0.6, seed=3 + i, ignore_eos=True) for i in range(3)]

    def run(mixed):
        eng = build_engine("tiny", device="cpu", max_batch=4, max_model_len=256, num_blocks=128, seed=1)
        eng.mixed_steps = mixed
        reqs = [eng.add_request(prompts[0], params[0])]
        eng.step()                      # request 0: prefill + decode
        eng.step()
        reqs.append(eng.add_request(prompts[1], params[1]))
        eng.step()                      # request 1 prefills while 0 decodes
        reqs.append(eng.add_request(prompts[2], params[2]))
        while eng.has_work():
            eng.step()
        return [r.output_ids for r in reqs], eng.stats["mixed_steps"]

    mixed, n_mixed = run(True)
    split, n_split = run(False)
    assert n_mixed >= 2 and n_split == 0
    assert mixed == split and all(len(t) == 20 for t in mixed)


def test_mixed_step_leaves_a_device_finished_rows_prefix_block_alone():
    """a decode row the device has already finished (context 0, not yet reaped by the host) can ride
    a mixed step.  Its leftover token's K/V must go nowhere: position 0 of its first block is the shared, published
    prefix block (BOS / attention sink) that other sequences and later prefix hits read."""
    eng = build_engine("tiny", device="cpu", max_batch=4, max_model_len=256, num_blocks=128, seed=1)
    eng.mixed_steps = True
    shared = [(i * 13) % 500 + 20 for i in range(40)]        # 2 full (published) blocks + 8 tokens
    p = SamplingParams(max_tokens=30, temperature=0.0, ignore_eos=True)
    a = eng.add_request(shared + [7, 8], p)
    eng.step()
    eng.step()
    assert a.slot is not None and a in eng.running.values()
    kv = eng.model.kv_cache
    slot0 = a.blocks[0] * eng.block_size
    before = kv[:, :, slot0].clone()
    eng.s_ctx[a.slot:a.slot + 1].fill_(0)                    # the device finished row a (stop detected on device)
    eng.add_request(shared + [9, 10, 11], p)                 # arrives: the next step is a mixed step with row a
    n0 = eng.stats["mixed_steps"]
    eng._admit()
    eng._prefill()
    assert eng.stats["mixed_steps"] == n0 + 1
    assert torch.equal(kv[:, :, slot0], before)


@pytest.mark.parametrize("tp", [2, 4, 8])
def test_decision_prefill_buckets_stay_on_captured_xgmi(tp):
    """with the default slot size every decision-sized prefill bucket (<= 512 tokens, 8 MiB
    all-reduces at 70B) fits the xGMI transports at TP = 2 / 4 / 8 and is captured -- also when the autotune found
    RCCL faster for large messages eagerly (xgmi_max_ar below the chunk's size): while capturing, the all-reduces
    that fit run on xGMI (TPGroup.capture_on_xgmi), so RCCL never enters a graph."""
    from types import SimpleNamespace

    from k8s_llm_scheduler_amd.engine.engine import PREFILL_GRAPH_BUCKETS, LLMEngine
    from k8s_llm_scheduler_amd.parallel.comm import TPGroup, default_slot_bytes

    slot = default_slot_bytes(tp)
    xg = SimpleNamespace(slot_bytes=slot, max_allreduce_bytes=tp * slot)
    group = TPGroup(0, tp, None, "nccl", xgmi=xg)
    group.xgmi_max_ar = 1 << 20                     # autotune: RCCL faster from 1 MiB on (eager chunks)
    fake = SimpleNamespace(model=SimpleNamespace(tp=group, cfg=SimpleNamespace(hidden=8192),
                                                 lm_head=torch.empty(128256 // tp, 1)))
    for Tb in PREFILL_GRAPH_BUCKETS:
        assert LLMEngine._prefill_bucket_capturable(fake, Tb), (tp, Tb)
    chunk = SimpleNamespace(numel=lambda: 512 * 8192, element_size=lambda: 2, is_cuda=True)
    assert not group._xgmi_ok(chunk, reduce=True)     # eager: the autotune's RCCL threshold
    group.capture_on_xgmi = True
    assert group._xgmi_ok(chunk, reduce=True)         # captured: xGMI
    assert 10 * tp * slot <= 320 << 20                # the whole peer region stays small next to 288 GB
    assert 64 * (128256 // 8) * 4 <= default_slot_bytes(8)   # TP=8 decode logits gather at batch 64 fits a slot


def test_mixed_step_rows_stay_within_the_cap():
    """engine.mixed_step_rows: a mixed step that would land just past the cap (up to twice it) keeps its rows (prompt
    tokens + one per running decode) within it, the prompt tokens over it go into the next step; a larger backlog keeps
    its big chunk; the tokens equal the uncapped engine's."""
    prompt_long = [9, 10, 11, 12] * 12             # 48 prompt tokens
    params = [SamplingParams(max_tokens=n, temperature=0.0, ignore_eos=True) for n in (60, 60, 12)]

    def run(cap):
        eng = build_engine("tiny", device="cpu", max_batch=4, max_model_len=256, num_blocks=128, seed=1)
        eng.mixed_step_rows = cap
        rows = []
        orig = eng.model.forward_prefill

        def spy(ids, *a, **k):
            rows.append(int(ids.shape[0]))
            return orig(ids, *a, **k)

        eng.model.forward_prefill = spy
        reqs = [eng.add_request([5, 6, 7], params[0]), eng.add_request([5, 6, 8], params[1])]
        eng.step()
        eng.step()
        reqs.append(eng.add_request(prompt_long, params[2]))
        while eng.has_work():
            eng.step()
        return [r.output_ids for r in reqs], rows, eng.stats["mixed_steps"]

    capped, rows_c, n_c = run(32)
    free, rows_f, n_f = run(0)
    backlog, rows_b, _ = run(16)                    # 50 rows > 2 x cap: a backlog keeps its big chunk
    assert capped == free == backlog
    assert rows_c[1:3] == [32, 20] and n_c >= 2      # 48 prompt tokens: 30 beside 2 decodes, then 18 (+2)
    assert max(rows_f) == 48 + 2 and n_f == 1
    assert max(rows_b) == 48 + 2


def test_sub_block_prefix_hit_copies_kv_and_matches():
    """A shared prefix that ends inside a block: after the full-block hits, the leading tokens of the next block come
    from a cached block with the same parent chain (K/V copied into the new sequence's own block); the answers equal
    an engine without prefix caching, and only the new tokens are prefilled."""
    shared = [(i * 37) % 9000 + 100 for i in range(37)]          # 2 full blocks + 5 tokens of the third
    pa = shared + list(range(11, 31))                             # its third block is full (published)
    pb = shared + [21, 22, 23, 24, 25, 26, 27]
    params = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)

    def run(cache):
        eng = build_engine("tiny", device="cpu", max_batch=2, max_model_len=256, num_blocks=64, seed=1,
                           prefix_caching=cache)
        a = eng.generate([pa], params)[0].token_ids
        before = eng.stats["prefill_tokens"]
        b = eng.generate([pb], params)[0].token_ids
        return a, b, eng.stats["prefill_tokens"] - before, eng.stats.get("sub_block_tokens", 0)

    a1, b1, pre1, sub1 = run(True)
    a0, b0, pre0, sub0 = run(False)
    assert (a1, b1) == (a0, b0)
    assert sub1 == 5 and sub0 == 0
    assert pre1 == len(pb) - 37 and pre0 == len(pb)
