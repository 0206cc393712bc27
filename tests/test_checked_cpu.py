"""The bounds-checked kernel build on the CPU side: the release extension reports itself unchecked and its check
hooks are no-ops; the checked sources compile for gfx950 (hipcc cross-compiles without a GPU); the build names the
variant ``_C_checked`` (tests/test_checked_gpu.py runs it)."""

import os
import shutil
import subprocess

import pytest

from k8s_llm_scheduler_amd import _build, ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_release_extension_is_unchecked_and_hooks_are_noops():
    if not ops.available():
        pytest.skip("native extension not built")
    assert ops.native().checked is False
    assert ops.check_enable("cpu", 16, 1, 10) is False
    ops.check_raise("cpu")   # no-op without K8S_CHECKED
    assert _build.ext_path(True).name.startswith("_C_checked") and _build.ext_path().name.startswith("_C.")


@pytest.mark.skipif(shutil.which(_build.HIPCC) is None and not os.path.exists(_build.HIPCC), reason="no hipcc")
def test_checked_sources_compile(tmp_path):
    """misc.hip and rope_kv.hip (the cheapest instrumented units) with -DK8S_CHECKED: the macros expand to valid code."""
    for unit in ("misc", "rope_kv"):
        src = os.path.join(ROOT, "k8s_llm_scheduler_amd", "csrc", "kernels", unit + ".hip")
        r = subprocess.run([_build.HIPCC, "-O1", "-fPIC", "-std=c++17", "-x", "hip", f"--offload-arch={_build.ARCH}",
                            f"-I{_build.CSRC}", "-DK8S_CHECKED", "-c", src, "-o", str(tmp_path / (unit + ".o"))],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
