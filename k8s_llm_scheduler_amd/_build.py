"""Build the native extension ``k8s_llm_scheduler_amd/ops/_C*.so`` for gfx950.

Plain ``hipcc`` invocations (no hipify, no torch.utils.cpp_extension JIT cache): every ``.hip``
kernel file is compiled with ``--offload-arch=gfx950``, the runtime ``.cpp`` files and the
pybind11 bindings are host code, and only ``torch_stream.cpp`` sees PyTorch headers (to pick up
the current PyTorch HIP stream).  Objects are cached under ``build/`` and rebuilt when a source
or any header is newer.  Cross-compiles without a GPU.

    python -m k8s_llm_scheduler_amd._build [-j N] [--force] [-v] [--checked]

``--checked`` builds the bounds-checked variant ``ops/_C_checked*.so`` (``-DK8S_CHECKED``, objects under
``build/native_checked``; loaded instead of ``_C`` when ``K8S_CHECKED=1``): kernels range-check every index they
derive from data and record violations for the host (csrc/kernels/common.h).
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import List

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
ARCH = os.environ.get("K8S_HIP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path(checked: bool = False) -> Path:
    return PKG / "ops" / (("_C_checked" if checked else "_C") + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_dirs():
    import torch

    root = Path(torch.__file__).resolve().parent
    return root / "include", root / "lib", bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def _headers() -> List[Path]:
    return list(CSRC.rglob("*.h"))


def _stale(obj: Path, src: Path, headers: List[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(h.stat().st_mtime > t for h in headers)


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build(jobs: int = 0, force: bool = False, verbose: bool = False, checked: bool = False) -> Path:
    import pybind11

    tinc, tlib, cxx11 = _torch_dirs()
    bdir = BUILD.parent / "native_checked" if checked else BUILD
    bdir.mkdir(parents=True, exist_ok=True)
    headers = _headers()
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC}", f"-D_GLIBCXX_USE_CXX11_ABI={int(cxx11)}"]
    if checked:
        common += ["-DK8S_CHECKED", "-DK8S_MODULE_NAME=_C_checked"]
    py_inc = sysconfig.get_paths()["include"]
    units = []
    for src in sorted((CSRC / "kernels").glob("*.hip")):
        units.append((src, ["-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]))
    for src in sorted((CSRC / "runtime").glob("*.cpp")):
        units.append((src, []))
    units.append((CSRC / "bindings.cpp", [f"-I{pybind11.get_include()}", f"-I{py_inc}", "-fvisibility=hidden"]))
    units.append((CSRC / "torch_stream.cpp", [f"-I{tinc}", f"-I{tinc / 'torch/csrc/api/include'}",
                                               "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-w"]))
    objs = []
    todo = []
    for src, flags in units:
        obj = bdir / (src.relative_to(CSRC).as_posix().replace("/", "__") + ".o")
        objs.append(obj)
        if force or _stale(obj, src, headers):
            todo.append([HIPCC, *common, *flags, "-c", str(src), "-o", str(obj)])
    n = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        for f in [ex.submit(_run, c, verbose) for c in todo]:
            f.result()
    out = ext_path(checked)
    if todo or force or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        tmp = out.with_suffix(".tmp.so")
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp), *map(str, objs),
              f"-L{tlib}", "-lc10_hip", "-lc10", "-lrccl", f"-Wl,-rpath,{tlib}", "-Wl,--no-as-needed"], verbose)
        os.replace(tmp, out)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--checked", action="store_true", help="bounds-checked kernels: ops/_C_checked*.so")
    a = ap.parse_args(argv)
    p = build(a.jobs, a.force, a.verbose, a.checked)
    print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
