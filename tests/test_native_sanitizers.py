"""Native host code under sanitizers: the C++ paged-KV BlockAllocator is
compiled with -fsanitize=address,undefined (host compiler, no GPU) and driven by a randomized
allocate / commit-prefix / release stress test that checks refcount and free-list invariants."""

import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "k8s_llm_scheduler_amd" / "csrc"


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_block_allocator_asan_ubsan(tmp_path):
    exe = tmp_path / "alloc_stress"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", f"-I{CSRC}", str(ROOT / "tests" / "native" / "block_allocator_stress.cpp"),
           str(CSRC / "runtime" / "block_allocator.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ)
    # the environment may preload its own small library ahead of the ASan runtime: tolerate that
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ")
