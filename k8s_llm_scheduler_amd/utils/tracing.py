"""Tracing: roctx ranges (visible in ``rocprofv3 --marker-trace`` timelines next to the kernels) and
cheap host-side wall-clock accounting per range name.

The reference's only timing is ``time.time()`` around the API call (``scheduler.py:420,435``).
Here every engine phase (prefill, decode chunk, graph capture, decision) is a named range:

    from k8s_llm_scheduler_amd.utils.tracing import trace
    with trace("prefill"):
        ...

``K8S_TRACE=1`` turns the roctx markers on (libroctx64 via ctypes; silently absent when the
library is missing); the host timers are always on and cost two ``perf_counter`` calls.
"""

from __future__ import annotations

import ctypes
import os
import threading
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, Optional

_lib: Optional[ctypes.CDLL] = None
_enabled = os.environ.get("K8S_TRACE", "0") == "1"
_lock = threading.Lock()
_totals: Dict[str, float] = defaultdict(float)
_counts: Dict[str, int] = defaultdict(int)


def _roctx() -> Optional[ctypes.CDLL]:
    global _lib
    if _lib is None and _enabled:
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so", "libroctx64.so.4"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                break
            except OSError:
                continue
    return _lib


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = on


def enabled() -> bool:
    return _enabled and _roctx() is not None


@contextmanager
def trace(name: str):
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        dt = time.perf_counter() - t0
        if lib is not None:
            lib.roctxRangePop()
        with _lock:
            _totals[name] += dt
            _counts[name] += 1


def mark(name: str) -> None:
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


def summary(reset: bool = False) -> Dict[str, Dict[str, float]]:
    """{range: {"count": n, "total_s": t, "mean_ms": m}} of the host-side timers."""
    with _lock:
        out = {k: {"count": _counts[k], "total_s": round(v, 6), "mean_ms": round(1e3 * v / max(1, _counts[k]), 4)}
               for k, v in _totals.items()}
        if reset:
            _totals.clear()
            _counts.clear()
    return out
