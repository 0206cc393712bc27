"""GEMM routing without a GPU: the mgemm / pgemm plan tables' row buckets and nearest-bucket lookups, the auto policy
(hand-written kernels always; the library only as the K8S_GEMM=library oracle), and the GEMV row threshold."""

import json

import pytest

from k8s_llm_scheduler_amd import ops


def test_row_buckets():
    assert [ops._mg_bucket(m) for m in (1, 2, 3, 4, 5, 8, 9, 16, 17, 1000, 1025, 2000, 5000, 8192)] == \
        [2, 2, 4, 4, 8, 8, 16, 16, 32, 1024, 2048, 2048, 8192, 8192]


def test_mgemm_table_lookup_stays_inside_the_tuned_range():
    table = ops._mg_load_table()
    assert table, "engine/assets/mgemm_gfx950.json is missing or empty"
    fp8_keys = [k for k in table if k[3] == 1]
    assert fp8_keys
    n, k, epi, _ = fp8_keys[0]
    top = max(r[0] for r in table[fp8_keys[0]])
    assert ops._mg_table_row(top, n, k, epi, True) is not None
    assert ops._mg_table_row(4 * top + 1, n, k, epi, True) is None


def test_mgemm_override_replaces_a_table_row(monkeypatch):
    monkeypatch.setenv("K8S_MGEMM_OVERRIDE", "64,10240,8192,0,0=11:1;64,8192,8192,0,0=12:2")
    monkeypatch.setattr(ops, "_MG_TABLE", None)
    try:
        assert ops._mg_table_row(64, 10240, 8192, ops.EPI_BF16, False)[1:3] == (11, 1)
        assert ops._mg_table_row(64, 8192, 8192, ops.EPI_BF16, False)[1:3] == (12, 2)
    finally:
        monkeypatch.delenv("K8S_MGEMM_OVERRIDE")
        ops._MG_TABLE = None   # the next lookup reloads the bundled table


LLAMA_TP1 = [(10240, 8192, ops.EPI_BF16), (8192, 8192, ops.EPI_BF16), (28672, 8192, ops.EPI_SWIGLU),
             (8192, 28672, ops.EPI_BF16)]


@pytest.mark.parametrize("backend", ["auto", "pgemm"])
@pytest.mark.parametrize("fp8", [False, True])
def test_auto_never_routes_to_the_library(monkeypatch, backend, fp8):
    monkeypatch.setattr(ops, "GEMM_BACKEND", backend)
    for M in (3, 8, 64, 128, 129, 245, 256, 1000, 2048, 8192, 20000):
        for N, K, epi in LLAMA_TP1:
            kern, plan = ops.gemm_route(M, N, K, epi, fp8)
            assert kern in ("mgemm", "pgemm", "pgemm4"), (M, N, K, kern)
            if fp8:
                assert kern != "pgemm4"           # the 4-wave kernel is bf16 only
            if backend == "auto" and M < ops.PG_MIN_M:
                assert kern == "mgemm"
            if kern.startswith("pgemm"):
                cfg, sp, gm = plan
                cfgs = ops.pgemm_configs() if kern == "pgemm" else ops.pgemm4_configs()
                assert 0 <= cfg < len(cfgs) and sp >= 1 and gm >= 1


def test_pgemm_table_picks_nearest_bucket_at_or_above(monkeypatch):
    monkeypatch.setattr(ops, "_PG_TABLE", {(100, 256, 0, 0): [(256, "pgemm4", 3, 2, 4, 10.0),
                                                               (2048, "pgemm", 0, 1, 8, 50.0)]})
    assert ops.pgemm_plan_for(200, 100, 256, 0, False) == (("pgemm4", 3, 2, 4), 10.0)
    assert ops.pgemm_plan_for(257, 100, 256, 0, False) == (("pgemm", 0, 1, 8), 50.0)
    assert ops.pgemm_plan_for(9000, 100, 256, 0, False) == (("pgemm", 0, 1, 8), None)   # past the top: its plan
    # fp8 has no 4-wave kernel: a bf16-only plan is not used for it
    monkeypatch.setattr(ops, "_PG_TABLE", {(100, 256, 0, 1): [(256, "pgemm4", 3, 2, 4, 10.0)]})
    assert ops.pgemm_plan_for(200, 100, 256, 0, True)[0][0] == "pgemm"


def test_auto_follows_the_tuned_winner(monkeypatch):
    monkeypatch.setattr(ops, "GEMM_BACKEND", "auto")
    monkeypatch.setattr(ops, "_PG_TABLE", {(1024, 1024, 0, 0): [(256, "mgemm", 0, 0, 0, 25.0),
                                                                 (512, "pgemm", 0, 2, 4, 30.0)]})
    assert ops.gemm_route(256, 1024, 1024, 0, False)[0] == "mgemm"
    assert ops.gemm_route(300, 1024, 1024, 0, False) == ("pgemm", (0, 2, 4))
    monkeypatch.setattr(ops, "GEMM_BACKEND", "pgemm")
    assert ops.gemm_route(256, 1024, 1024, 0, False)[0] == "pgemm"
    monkeypatch.setattr(ops, "GEMM_BACKEND", "library")
    assert ops.gemm_route(256, 1024, 1024, 0, False) == ("library", None)


def test_shipped_pgemm_table_is_consistent():
    if not __import__("os").path.isfile(ops.PG_TABLE_PATH):
        pytest.skip("no tuned pgemm table")
    with open(ops.PG_TABLE_PATH) as f:
        plans = json.load(f)["plans"]
    assert plans
    for key, v in plans.items():
        m, n, k, epi, fp8 = (int(t) for t in key.split(","))
        kern, cfg, sp, gm = v[:4]
        assert kern in ("mgemm", "pgemm", "pgemm4") and not (fp8 and kern == "pgemm4")
        assert ops.pgemm_plan_for(m, n, k, epi, bool(fp8))[0] == (kern, cfg, sp, gm)


def test_gemv_threshold_and_kernel_limit():
    assert 1 <= ops.GEMV_MAX_M <= ops.GEMV_KERNEL_MAX_M == 8


if __name__ == "__main__":
    pytest.main([__file__])


@pytest.mark.parametrize("backend", ["auto", "mgemm", "pgemm"])
def test_unroutable_shape_raises_instead_of_calling_the_library(monkeypatch, backend):
    """a shape no hand-written kernel accepts (N % 4 != 0 here) raises under every hand-written
    route -- linear and linear_swiglu never fall through to hipBLASLt / _scaled_mm silently."""
    import torch

    monkeypatch.setattr(ops, "GEMM_BACKEND", backend)
    monkeypatch.setattr(ops, "_gpu", lambda *a: True)           # route as on the GPU, compute nothing
    called = []
    monkeypatch.setattr(ops, "_lib_linear", lambda x, w: called.append("lib") or x @ w.t())
    x = torch.randn(300, 256, dtype=torch.bfloat16)
    w = torch.randn(130, 256, dtype=torch.bfloat16)              # N = 130: no 4-column output groups
    assert ops.gemm_route(300, 130, 256, ops.EPI_BF16, False)[0] == "library"
    with pytest.raises(ops.NoKernelForShape, match="K8S_GEMM=library"):
        ops.linear(x, w)
    with pytest.raises(ops.NoKernelForShape):
        ops.linear_swiglu(x, torch.randn(2 * 130, 256, dtype=torch.bfloat16))
    assert not called


def test_library_route_only_under_k8s_gemm_library(monkeypatch):
    import torch

    monkeypatch.setattr(ops, "GEMM_BACKEND", "library")
    monkeypatch.setattr(ops, "_gpu", lambda *a: True)
    called = []
    monkeypatch.setattr(ops, "_lib_linear", lambda x, w: called.append("lib") or (x.float() @ w.float().t()).to(x.dtype))
    y = ops.linear(torch.randn(300, 256, dtype=torch.bfloat16), torch.randn(128, 256, dtype=torch.bfloat16))
    assert called == ["lib"] and y.shape == (300, 128)


def _llama70b_decode_shapes(tp):
    hidden, inter, nq, nkv, d = 8192, 28672, 64, 8, 128
    return [((nq + 2 * nkv) * d // tp, hidden, ops.EPI_BF16), (hidden, nq * d // tp, ops.EPI_BF16),
            (inter // tp, hidden, ops.EPI_SWIGLU), (hidden, inter // tp, ops.EPI_BF16)]


@pytest.mark.parametrize("tp", [1, 2, 4, 8])
def test_every_batched_decode_shape_has_a_valid_tuned_plan(tp):
    """The 17-128-row bf16 plans (re-tuned in situ) and the MX plans (keys 3 / 4) cover every projection of a Llama-70B
    decode layer at TP = 1 / 2 / 4 / 8, and each tuned plan is valid for every row count of its bucket -- a shape that
    fell off the table would silently run the heuristic plan."""
    for i, (N, K, epi) in enumerate(_llama70b_decode_shapes(tp)):
        for M in (17, 24, 32, 33, 48, 64, 65, 100, 128):
            row = ops._mg_table_row(M, N, K, epi, False)
            assert row is not None, (tp, M, N, K, epi)
            assert ops.mgemm_valid(row[1], M, N, K, epi, 0, row[2]), (tp, M, N, K, epi, row)
            if K % 128 == 0:
                mx_out = i > 0   # O / down: the residual epilogue's MX copy; gate/up: MX SwiGLU output
                assert ops.mgemm_mx_plan(M, N, K, epi, True, mx_out) is not None, (tp, M, N, K, epi)


def test_mx_plans_are_tuned_for_every_tp_shard():
    """fp8 batched decode at TP = 1 / 2 / 4 / 8: every projection has TUNED MX plans (table keys 3 / 4) for 32-256 rows,
    not only a heuristic one."""
    table = ops._mg_load_table()
    for tp in (1, 2, 4, 8):
        for N, K, epi in _llama70b_decode_shapes(tp):
            key = (N, K, epi, 4 if epi == ops.EPI_SWIGLU else 3)
            assert sorted(r[0] for r in table.get(key, [])) == [32, 64, 128, 256], (tp, key)
