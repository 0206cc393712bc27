"""GEMM routing without a GPU: the mgemm plan table's row buckets, the nearest-bucket lookup and its limit,
the auto policy (library only where the table measured it faster), and the GEMV row threshold."""

import json

import pytest

from k8s_llm_scheduler_amd import ops


def test_row_buckets():
    assert [ops._mg_bucket(m) for m in (1, 2, 3, 4, 5, 8, 9, 16, 17, 1000, 1025, 2000, 5000, 8192)] == \
        [2, 2, 4, 4, 8, 8, 16, 16, 32, 1024, 2048, 2048, 8192, 8192]


def test_table_lookup_stays_inside_the_tuned_range():
    table = ops._mg_load_table()
    assert table, "engine/assets/mgemm_gfx950.json is missing or empty"
    # fp8 shapes are tuned up to 256 rows: an 8192-row prefill chunk is untuned, not a 256-row plan
    fp8_keys = [k for k in table if k[3] == 1]
    assert fp8_keys
    n, k, epi, _ = fp8_keys[0]
    top = max(r[0] for r in table[fp8_keys[0]])
    assert ops._mg_table_row(top, n, k, epi, True) is not None
    assert ops._mg_table_row(4 * top + 1, n, k, epi, True) is None
    assert not ops.mgemm_preferred(4 * top + 1, n, k, epi, True)   # untuned prefill rows: the library


def test_auto_policy_follows_the_table(monkeypatch):
    monkeypatch.setattr(ops, "GEMM_BACKEND", "auto")
    with open(ops.MG_TABLE_PATH) as f:
        plans = json.load(f)["plans"]
    checked = 0
    for key, (cfg, grid, mg_us, lib_us) in list(plans.items())[:200]:
        mb, n, k, epi, fp8 = (int(t) for t in key.split(","))
        row = ops._mg_table_row(mb, n, k, epi, bool(fp8))
        if row is None or row[0] != mb:
            continue
        assert ops.mgemm_preferred(mb, n, k, epi, bool(fp8)) == (row[3] <= 1.03 * row[4])
        checked += 1
    assert checked > 50
    monkeypatch.setattr(ops, "GEMM_BACKEND", "library")
    assert not ops.mgemm_preferred(64, 8192, 8192, ops.EPI_BF16, False)
    monkeypatch.setattr(ops, "GEMM_BACKEND", "mgemm")
    assert ops.mgemm_preferred(8192, 8192, 8192, ops.EPI_BF16, False)


def test_gemv_threshold_and_kernel_limit():
    assert 1 <= ops.GEMV_MAX_M <= ops.GEMV_KERNEL_MAX_M == 8


def test_fused_routing_credit_only_when_asked(monkeypatch):
    monkeypatch.setattr(ops, "GEMM_BACKEND", "auto")
    monkeypatch.setattr(ops, "_mg_table_row", lambda *a: (64, 0, 1, 50.0, 46.0))   # library 8 % faster
    monkeypatch.setattr(ops, "FUSION_CREDIT_US", 0.0)
    assert not ops.mgemm_preferred(64, 1, 1, 0, False, fused=True)
    monkeypatch.setattr(ops, "FUSION_CREDIT_US", 5.0)
    assert ops.mgemm_preferred(64, 1, 1, 0, False, fused=True)
    assert not ops.mgemm_preferred(64, 1, 1, 0, False)


if __name__ == "__main__":
    pytest.main([__file__])
