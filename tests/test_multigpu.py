"""T4 multi-rank tests on GPU.

* ``test_*_rehearsal``: EIGHT real rank processes share the one test GPU (gloo process group + the xGMI
  peer-memory collectives through hipIpc mappings -- the same kernels and protocol as 8 processes on 8
  GPUs, with one HBM standing in for the peers').  World = 8 exercises the 8-peer flag / slot layout
  (XG_MAX_WORLD) and the TP = 8 sharding (one kv head per rank).
* ``test_multi_gpu_*``: run only where >= 2 GPUs are visible (the 8-GPU node): one rank per GPU, RCCL
  communicator + xGMI across physical GPUs, TP = 2 / 4 / 8.

Checks: all-reduce bit-exact against the fixed-order fp32 sum at every message size class (LL and
flagged protocols, fused residual, hipGraph replays), all-gather, RCCL all-reduce against a reference
sum, TP = k logits == TP = 1 logits (prefill and decode), and identical greedy / sampled tokens on every
rank from an engine with captured decode graphs."""

import os

import pytest
import torch

from mp_harness import run_ranks

pytestmark = pytest.mark.gpu

IDS = [7, 100, 2000, 31, 32, 33, 900, 12, 5, 5, 5, 6000, 42, 43]


def _data(rank, n, seed):
    g = torch.Generator().manual_seed(1000 * seed + rank)
    return (torch.randn(n, generator=g) * 4).to(torch.bfloat16)


def _check_collectives(tp, res):
    world = tp.world
    xg = tp.xgmi
    if xg is not None:
        for path, ll in (("ll", xg.ll_max_bytes), ("flagged", 0)):
            keep = xg.ll_max_bytes
            xg.ll_max_bytes = ll
            for seed, n in enumerate([8, 520, 8192, 32768, xg.slot_bytes // 2]):
                x = _data(tp.rank, n, seed).cuda()
                want32 = sum(_data(r, n, seed).float() for r in range(world))   # fixed rank order, fp32
                tp.all_reduce_(x)
                torch.cuda.synchronize()
                assert torch.equal(x.cpu(), want32.to(torch.bfloat16)), f"xgmi {path} all_reduce n={n}"
                r = _data(99, n, seed).cuda()
                x = _data(tp.rank, n, seed).cuda()
                tp.all_reduce_(x, residual=r)
                torch.cuda.synchronize()
                assert torch.equal(x.cpu(), (want32 + r.cpu().float()).to(torch.bfloat16)), \
                    f"xgmi {path} all_reduce+residual n={n}"
            xg.ll_max_bytes = keep
        _check_twoshot(tp, res)
        _check_fused_gemv_ar(tp, res)
        for n in (4, 4096, 2048 * 4):
            src = torch.arange(n, dtype=torch.float32, device="cuda") + 1e6 * tp.rank
            out = tp.all_gather_shards(src)
            torch.cuda.synchronize()
            want = torch.stack([torch.arange(n, dtype=torch.float32) + 1e6 * r for r in range(world)])
            assert torch.equal(out.cpu(), want), f"xgmi all_gather n={n}"
        # captured + replayed: device-side epochs / slots advance across replays
        buf = torch.zeros(8192, dtype=torch.bfloat16, device="cuda")

        def step():
            buf.mul_(0).add_(tp.rank + 1)
            tp.all_reduce_(buf)
            buf.add_(1)

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(4):
                step()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        assert float(buf[0]) == world * (world + 1) / 2 + 1
        res["xgmi_err"] = xg.error()
    if tp.rccl is not None:
        for dt, code in ((torch.float32, 1), (torch.bfloat16, 0)):
            for n in (16, 8192, 1 << 20):
                x = _data(tp.rank, n, 7).to(dt).cuda()
                want = sum(_data(r, n, 7).to(dt).float() for r in range(world))
                tp.rccl.all_reduce(x.data_ptr(), x.data_ptr(), n, code, 0, -1)
                torch.cuda.synchronize()
                tol = 0 if dt == torch.float32 else 0.02 * float(want.abs().max())
                assert float((x.float().cpu() - want).abs().max()) <= tol + 1e-3, f"rccl all_reduce {dt} n={n}"


def _check_fused_gemv_ar(tp, res):
    """Row-parallel GEMV with the all-reduce in its epilogue (gemv.hip GemvAr): bit-exact against
    GEMV + separate xGMI all-reduce where both GEMVs take one K slice, within bf16 rounding of the fp32 oracle
    (sum over ranks of x_r . W_r^T, + residual) everywhere; bf16 and fp8 weights; graph replays."""
    from k8s_llm_scheduler_amd import ops

    world = tp.world
    shapes = [(1, 2048, 256), (2, 2048, 512), (1, 8192, 1024), (4, 1024, 2048), (8, 512, 512), (1, 4096, 3584)]
    done = []
    for i, (M, N, K) in enumerate(shapes):
        xs = [_data(r, M * K, 200 + i).view(M, K) for r in range(world)]
        ws = [(_data(r, N * K, 300 + i) * 0.05).to(torch.bfloat16).view(N, K) for r in range(world)]
        resid = _data(99, M * N, 400 + i).view(M, N)
        x, w, rr = xs[tp.rank].cuda(), ws[tp.rank].cuda(), resid.cuda()
        y = ops.gemv_allreduce(tp.xgmi, x, w, rr)
        assert y is not None, f"fused plan refused {(M, N, K)}"
        base = ops.linear(x, w)
        tp.all_reduce_(base, residual=rr)
        torch.cuda.synchronize()
        ref = sum(xs[r].float() @ ws[r].float().T for r in range(world)) + resid.float()
        err = float((y.float().cpu() - ref).abs().max())
        assert err <= 0.02 * float(ref.abs().max()) + 0.05, f"fused gemv all-reduce {(M, N, K)}: err {err}"
        ks, splits = ops.native().gemv_plan(M, N, K, ops.EPI_BF16, 0)
        same_kernel = splits == 1 and M <= ops.GEMV_MAX_M   # linear() took the one-slice GEMV too (not mgemm)
        if same_kernel:
            assert torch.equal(y.cpu(), base.cpu()), f"fused != GEMV + all-reduce {(M, N, K)}"
        # fp8 weights (per-row scales applied before the bf16 partial rounding, as the unfused GEMV does); above
        # GEMV_MAX_M rows linear() quantizes the activations too (fp8 GEMM), so only the weight error is shared
        wq = ops.quantize_fp8(w)
        y8 = ops.gemv_allreduce(tp.xgmi, x, wq, rr)
        torch.cuda.synchronize()
        assert y8 is not None
        assert float((y8.float().cpu() - ref).abs().max()) <= 0.1 * float(ref.abs().max()) + 0.05, \
            f"fp8 fused gemv all-reduce {(M, N, K)}"
        if same_kernel:
            b8 = ops.linear(x, wq)
            tp.all_reduce_(b8, residual=rr)
            torch.cuda.synchronize()
            assert torch.equal(y8.cpu(), b8.cpu()), f"fp8 fused != GEMV + all-reduce {(M, N, K)}"
        done.append((M, N, K))
    # captured and replayed, with the separate all-reduce kernels interleaved (their own epochs)
    M, N, K = 1, 2048, 512
    x = _data(tp.rank, M * K, 9).view(M, K).cuda()
    w = (_data(tp.rank, N * K, 10) * 0.05).to(torch.bfloat16).view(N, K).cuda()
    r0 = _data(99, M * N, 11).view(M, N).cuda()
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")

    def step():
        y = ops.gemv_allreduce(tp.xgmi, x, w, r0)
        z = ops.gemv_allreduce(tp.xgmi, x, w, y)
        tp.all_reduce_(z)
        out.copy_(z)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    want = out.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(3):
            step()
    for _ in range(5):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, want), "fused gemv all-reduce graph replay"
    res["fused_gemv_ar_shapes"] = done


def _check_twoshot(tp, res):
    """Two-shot all-reduce (reduce-scatter + all-gather through the peer slots), bit-exact against the fixed-order
    fp32 sum at the MiB sizes the autotune routes to it (a 256-token TP = 8 prefill all-reduces 4 MiB), with and
    without the fused residual, eager and replayed from a graph."""
    xg, world = tp.xgmi, tp.world
    keep = (xg.ll_max_bytes, xg.twoshot_min_bytes)
    xg.ll_max_bytes, xg.twoshot_min_bytes = 0, 16
    cap = xg.max_allreduce_bytes
    # 8 MiB (a 512-token 70B chunk) where the ranks have a GPU each or share one at world <= 4 (eight ranks
    # time-sharing one GPU spin through every two-shot phase: keep their largest message at 4 MiB)
    top = 8 << 20 if world <= 4 or torch.cuda.device_count() >= world else 4 << 20
    sizes = sorted({n for n in (1 << 20, 2 << 20, 4 << 20, 8 << 20) if n <= min(cap, top)})
    try:
        for seed, nbytes in enumerate(sizes):
            n = nbytes // 2
            want32 = sum(_data(r, n, 50 + seed).float() for r in range(world))
            x = _data(tp.rank, n, 50 + seed).cuda()
            tp.all_reduce_(x)
            torch.cuda.synchronize()
            assert torch.equal(x.cpu(), want32.to(torch.bfloat16)), f"two-shot all_reduce {nbytes} B"
            r = _data(99, n, 50 + seed).cuda()
            x = _data(tp.rank, n, 50 + seed).cuda()
            tp.all_reduce_(x, residual=r)
            torch.cuda.synchronize()
            assert torch.equal(x.cpu(), (want32 + r.cpu().float()).to(torch.bfloat16)), f"two-shot + residual {nbytes} B"
        # graph replays of the largest size: the slot / epoch state advances on the device
        n = sizes[-1] // 2
        src = _data(tp.rank, n, 77).cuda()
        want = sum(_data(r, n, 77).float() for r in range(world)).to(torch.bfloat16)
        buf = torch.empty_like(src)

        def step():
            buf.copy_(src)
            tp.all_reduce_(buf)

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(3):
                step()
        for _ in range(4):
            g.replay()
        torch.cuda.synchronize()
        assert torch.equal(buf.cpu(), want), "two-shot graph replay"
    finally:
        xg.ll_max_bytes, xg.twoshot_min_bytes = keep
    res["twoshot_sizes"] = sizes


def _model_and_engine(tp, res, preset="tiny-tp8"):
    from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine
    from k8s_llm_scheduler_amd.models.config import PRESETS
    from k8s_llm_scheduler_amd.models.llama import LlamaModel
    from k8s_llm_scheduler_amd.parallel import TPGroup
    from test_model_gpu import _prefill

    m = LlamaModel(PRESETS[preset], tp, device="cuda", seed=3, max_model_len=512)
    lg, bt = _prefill(m, IDS)
    ctx = torch.tensor([len(IDS) + 1], dtype=torch.int32, device="cuda")
    dec = m.forward_decode(torch.tensor([77], dtype=torch.int32, device="cuda"), ctx, bt, 512)
    full = lambda t: t.permute(1, 0, 2).reshape(t.shape[1], -1) if t.dim() == 3 else t   # noqa: E731
    if tp.rank == 0:
        m1 = LlamaModel(PRESETS[preset], TPGroup(), device="cuda", seed=3, max_model_len=512)
        lg1, bt1 = _prefill(m1, IDS)
        dec1 = m1.forward_decode(torch.tensor([77], dtype=torch.int32, device="cuda"), ctx, bt1, 512)
        res["prefill_err"] = float((full(lg).float() - full(lg1).float()).abs().max())
        res["decode_err"] = float((full(dec).float() - full(dec1).float()).abs().max())
        res["logit_scale"] = float(full(lg1).float().abs().max())
        res["argmax_equal"] = bool(torch.equal(full(lg).argmax(-1).cpu(), full(lg1).argmax(-1).cpu()))
        del m1
    # prefill as two micro-batches whose all-reduces run on the comm stream under the other half's GEMMs
    # (a two-sequence chunk split inside sequence 0) against the same chunk unsplit
    from test_prefill_overlap import _run_chunk

    assert m.prefill_overlap
    lg_a, kv_a = _run_chunk(m, 0)
    lg_b, kv_b = _run_chunk(m, 80)
    res["split_err"] = float((lg_a.float() - lg_b.float()).abs().max())
    res["split_kv_err"] = float((kv_a.float() - kv_b.float()).abs().max())
    res["split_scale"] = float(lg_a.float().abs().max())
    res["split_kv_scale"] = float(kv_a.float().abs().max())
    # the same chunk sequence-parallel: reduce-scatter + all-gather of row shards in place of each all-reduce
    os.environ.update(K8S_SEQ_PARALLEL="1", K8S_SEQ_PARALLEL_MIN="16")
    try:
        assert m.seq_parallel_at(160)
        lg_s, kv_s = _run_chunk(m, 0)
    finally:
        os.environ["K8S_SEQ_PARALLEL"] = "0"
    res["sp_err"] = float((lg_a.float() - lg_s.float()).abs().max())
    res["sp_kv_err"] = float((kv_a.float() - kv_s.float()).abs().max())
    del m
    eng = build_engine(preset, tp=tp, device="cuda", max_batch=4, max_model_len=512, num_blocks=128, seed=1,
                       capture_nucleus=True)   # a top_p < 1 request below: the graphs with the nucleus passes
    outs = eng.generate(["tensor parallel over xgmi", "second request", "third"],
                        [SamplingParams(max_tokens=12, temperature=0.8, seed=9, ignore_eos=True),
                         SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True),
                         SamplingParams(max_tokens=12, temperature=0.3, top_p=0.9, seed=4, ignore_eos=True)])
    # one request alone: its prefill chunk replays a prefill graph (xGMI-only buckets at TP > 1)
    solo = eng.generate(["a single prompt prefilled by a graph"], [SamplingParams(max_tokens=4, temperature=0.0,
                                                                                  ignore_eos=True)])
    # prompts of >= 128 tokens prefill as two overlapped micro-batches: alone (a prefill graph with the
    # fork / join captured) and two at once (the eager varlen split)
    long_p = " ".join(f"node-{i} cpu {i % 7} mem {i % 5}" for i in range(13))
    assert len(eng.tok.encode(long_p)) >= 128
    greedy = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    replays = eng.stats["prefill_graph_replays"]
    lone = eng.generate([long_p], [greedy])
    res["long_graph_replayed"] = eng.stats["prefill_graph_replays"] > replays
    split_chunks = eng.stats["prefill_overlap_chunks"]
    pair = eng.generate([" ".join(f"pod-{i} gpu {i % 3}" for i in range(12)),
                         " ".join(f"rack-{i} disk {i % 9}" for i in range(12))], [greedy, greedy])
    res["tokens"] = [o.token_ids for o in outs] + [solo[0].token_ids] + [lone[0].token_ids] + \
        [o.token_ids for o in pair]
    res["overlap_chunks"] = (split_chunks, eng.stats["prefill_overlap_chunks"])
    res["graph_replays"] = eng.stats["graph_replays"]
    res["prefill_graph_replays"] = eng.stats["prefill_graph_replays"]
    res["prefill_graphs"] = sorted(eng.prefill_graphs)
    del eng
    # speculative decoding at TP > 1: every rank drafts from the same host state, verifies through the captured
    # verify graph (its all-reduces on xGMI) and must accept the same drafts
    from k8s_llm_scheduler_amd.engine.engine import LLMEngine
    from k8s_llm_scheduler_amd.engine.tokenizer import Tokenizer
    from test_speculative_cpu import CycleModel

    cm = CycleModel(PRESETS[preset], tp, device="cuda", seed=1, max_model_len=512)
    seng = LLMEngine(cm, Tokenizer(None, model_vocab=cm.cfg.vocab), max_batch=4, num_blocks=64, max_model_len=512,
                     seed=1, speculative_tokens=4)
    seng.capture_graphs()
    sp = seng.generate([[3, 4, 5, 6, 7]], SamplingParams(max_tokens=30, temperature=0.0, ignore_eos=True))
    res["spec"] = (sp[0].token_ids, seng.stats["spec_graph_replays"], seng.stats["spec_accepted"])


def _rehearsal_rank(rank, world):
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.parallel import init_from_env

    tp = init_from_env("cuda", backend="gloo", comm="xgmi")
    assert tp.xgmi is not None and tp.world == world
    res = {}
    _check_collectives(tp, res)
    if os.environ.get("K8S_TEST_MODEL", "1") == "1":
        _model_and_engine(tp, res)
    dist.barrier()
    dist.destroy_process_group()
    return res


def _assert_model(res, world):
    r0 = res[0]
    assert all(res[r].get("xgmi_err", 0) == 0 for r in range(world))
    assert r0.get("twoshot_sizes"), "two-shot sizes were not checked"
    if "tokens" not in r0:
        return
    assert r0["prefill_err"] < 0.03 * r0["logit_scale"] + 0.03, r0
    assert r0["decode_err"] < 0.03 * r0["logit_scale"] + 0.03, r0
    assert all(res[r]["tokens"] == r0["tokens"] for r in range(world)), "ranks drew different tokens"
    assert r0["graph_replays"] > 0
    assert r0["prefill_graph_replays"] > 0, r0["prefill_graphs"]
    # the halves' GEMMs have other row counts (other tiles / k-split orders): bf16 rounding, not a layout error
    assert r0["split_kv_err"] < 0.02 * r0["split_kv_scale"] + 0.02, r0
    assert r0["split_err"] < 0.02 * r0["split_scale"] + 0.02, r0
    assert r0["sp_kv_err"] < 0.02 * r0["split_kv_scale"] + 0.02, r0
    assert r0["sp_err"] < 0.02 * r0["split_scale"] + 0.02, r0
    assert r0["long_graph_replayed"], r0["prefill_graphs"]
    toks, replays, accepted = r0["spec"]
    assert all(res[r]["spec"] == r0["spec"] for r in range(world)), "ranks diverged under speculative decoding"
    assert toks[:6] == [10, 11, 12, 13, 14, 10] and replays > 0 and accepted >= 15, r0["spec"]
    a, b = r0["overlap_chunks"]
    assert a >= 1 and b >= a + 1, r0["overlap_chunks"]   # the graph chunk and the eager pair chunk were split


@pytest.mark.parametrize("world", [8, 4, 2])
def test_tp_rehearsal_ranks_share_one_gpu(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = run_ranks(_rehearsal_rank, world, env={"K8S_TP_BACKEND": "gloo", "K8S_TP_COMM": "xgmi",
                                                 "K8S_TEST_MODEL": "1" if world == 8 else "0",
                                                 "K8S_PREFILL_OVERLAP_MIN": "128"}, timeout_s=480)
    _assert_model(res, world)
    if world == 8:
        print(f"TP=8 rehearsal (8 ranks, one GPU): max |d logit| prefill {res[0]['prefill_err']:.3g} "
              f"decode {res[0]['decode_err']:.3g} (scale {res[0]['logit_scale']:.3g}), tokens equal on all ranks; "
              f"overlapped prefill vs unsplit: max |d logit| {res[0]['split_err']:.3g}, |d kv| {res[0]['split_kv_err']:.3g} "
              f"(kv scale {res[0]['split_kv_scale']:.3g}), overlapped chunks {res[0]['overlap_chunks']}")


def test_tp_rehearsal_fused_ar_row_set_loop():
    """The fused GEMV all-reduce with the row-set loop (K8S_GEMV_LOOP_AR: each workgroup streams a contiguous band
    of row sets and pushes every set's words as it finishes it): the collective checks, including the fused path's
    bit-exact comparison against GEMV + all-reduce, at 4 ranks on one GPU."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = run_ranks(_rehearsal_rank, 4, env={"K8S_TP_BACKEND": "gloo", "K8S_TP_COMM": "xgmi", "K8S_TEST_MODEL": "0",
                                             "K8S_GEMV_LOOP_AR": "1"}, timeout_s=300)
    _assert_model(res, 4)


def _vocab_parallel_rank(rank, world):
    """Vocab-parallel sampling against the gathered-logits path on the GPU: the same engine
    schedule (captured decode graphs with and without the top-p passes, a mixed prefill + decode step) twice."""
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.engine import SamplingParams, build_engine
    from k8s_llm_scheduler_amd.parallel import init_from_env

    tp = init_from_env("cuda", backend="gloo", comm="xgmi")
    prompts = ["vocab parallel sampling", "a second request", "third", "the fourth prompt about nodes and pods"]
    params = [SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True),
              SamplingParams(max_tokens=16, temperature=0.3, seed=5, ignore_eos=True),
              SamplingParams(max_tokens=16, temperature=0.8, top_p=0.9, seed=7, ignore_eos=True),
              SamplingParams(max_tokens=16, temperature=1.0, top_p=0.5, seed=8, ignore_eos=True)]
    res = {}
    for vp in ("1", "0"):
        os.environ["K8S_VOCAB_PARALLEL"] = vp
        eng = build_engine("tiny-tp8", tp=tp, device="cuda", max_batch=4, max_model_len=512, num_blocks=128, seed=1,
                           capture_nucleus=True)
        out = [o.token_ids for o in eng.generate(prompts, params)]
        long = [SamplingParams(**{**q.__dict__, "max_tokens": 40}) for q in params]
        reqs = [eng.add_request(prompts[0], long[1]), eng.add_request(prompts[1], long[2])]
        eng.step()
        eng.step()
        reqs.append(eng.add_request(prompts[3], long[3]))       # a mixed step: decode rows ride the prefill
        while eng.has_work():
            eng.step()
        res[vp] = {"tokens": out, "mixed": [r.output_ids for r in reqs], "replays": eng.stats["graph_replays"],
                   "mixed_steps": eng.stats["mixed_steps"]}
        del eng
    dist.barrier()
    dist.destroy_process_group()
    return res


@pytest.mark.parametrize("world", [2, 4])
def test_vocab_parallel_sampling_equals_gathered_rehearsal(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # K8S_FUSED_AR=0: this test is about sampling; the fused GEMV + all-reduce (tested on its own above and in
    # test_multigpu_70b.py) launches full grids whose workgroups wait for the peers' partials, and with every rank on
    # ONE device those grids of the ranks that arrived first can hold the CUs the last rank's kernel needs -- the
    # flake this test showed in 3 of 6 full-suite runs of round 6 (the harness's stack dump: the last rank waiting on
    # its own GPU event while the others timed out in the collective).  One process per GPU has no such contention.
    res = run_ranks(_vocab_parallel_rank, world, env={"K8S_TP_BACKEND": "gloo", "K8S_TP_COMM": "xgmi",
                                                      "K8S_FUSED_AR": "0"}, timeout_s=300)
    r0 = res[0]
    assert r0["1"]["replays"] > 0 and r0["1"]["mixed_steps"] >= 1, r0["1"]
    assert (r0["1"]["tokens"], r0["1"]["mixed"]) == (r0["0"]["tokens"], r0["0"]["mixed"]), r0
    assert all(res[r] == r0 for r in range(world)), "ranks drew different tokens"


def _multi_gpu_rank(rank, world):
    import torch.distributed as dist

    from k8s_llm_scheduler_amd.parallel import init_from_env
    from k8s_llm_scheduler_amd.parallel.comm import make_xgmi_comm

    tp = init_from_env("cuda", backend="nccl", comm="rccl")
    assert tp.rccl is not None and torch.cuda.current_device() == rank
    res = {}
    _check_collectives(tp, res)            # RCCL across GPUs
    tp.xgmi = make_xgmi_comm(tp)           # then the xGMI peer-memory path across GPUs
    assert tp.xgmi is not None, "xGMI peer mapping failed across GPUs"
    rc, tp.rccl = tp.rccl, None
    _check_collectives(tp, res)
    tp.rccl = rc
    _model_and_engine(tp, res)             # default transport mix (xGMI small, RCCL large)
    dist.barrier()
    dist.destroy_process_group()
    return res


@pytest.mark.parametrize("world", [2, 4, 8])
def test_multi_gpu_tp_rccl_and_xgmi(world):
    if not torch.cuda.is_available() or torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs (found {torch.cuda.device_count() if torch.cuda.is_available() else 0})")
    res = run_ranks(_multi_gpu_rank, world, env={"K8S_PREFILL_OVERLAP_MIN": "128"}, timeout_s=600)
    _assert_model(res, world)


@pytest.mark.parametrize("world", [2, 4])
def test_bench_self_launch_rehearsal_prefill_on_captured_xgmi(world):
    """VERDICT r3 items 1 + 4: `python bench.py --gpus N` launches its N ranks itself (here time-sharing the one
    GPU), reports n_gpus N, and every decision's prefill chunk replays a captured graph on the xGMI transports --
    no RCCL collective is issued in the timed decisions."""
    import json
    import subprocess
    import sys

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, K8S_TP_BACKEND="gloo", K8S_TP_COMM="xgmi", OMP_NUM_THREADS="2")
    if world == 2:   #  the 2-rank rehearsal runs the all-reduce autotune too
        env["K8S_COMM_AUTOTUNE"] = "force"
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--preset", "tiny-tp8",
                        "--steps", "3", "--warmup", "1", "--gen-tokens", "8"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == world and d["config"]["parallelism"] == f"tp{world}", d
    assert d["prefill_graph_replays"] >= 3 and d["rccl_calls_timed"] == 0, d
    # the self-diagnosing start-up: stage timings of rank 0 and the slowest rank, the transport
    # self-tests, the transport of every timed all-reduce, and (world 2) the autotune table
    want = {"process_group", "xgmi_open", "xgmi_selftest", "fused_ar_selftest", "engine_build", "graph_capture",
            "warmup"} | ({"comm_autotune"} if world == 2 else set())
    assert want <= set(d["init_stages"]["rank0"]) and want <= set(d["init_stages"]["slowest"]), d["init_stages"]
    assert d["tp_comm"]["xgmi"] == "self-test passed", d["tp_comm"]
    assert d["tp_comm"]["fused_gemv_ar_selftest"] == "passed", d["tp_comm"]   # incl. the 70B shard shapes
    assert any(k.startswith(("prefill:xgmi", "decode:xgmi", "decode:fused_gemv_ar")) for k in d["allreduce_transports"]), \
        d["allreduce_transports"]
    if world == 2:
        assert d["tp_comm"].get("allreduce_us"), d["tp_comm"]
