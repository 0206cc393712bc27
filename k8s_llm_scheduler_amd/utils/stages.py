"""Named, bounded start-up stages (VERDICT r4 "next round" item 5: make the first real multi-GPU run self-diagnosing).

Every stage of bringing a TP engine up -- process group, RCCL communicator, xGMI peer mapping, the transports'
self-tests, the all-reduce autotune, the model build, graph capture, warm-up -- runs inside ``stage(name)``.  Each
stage's wall time is recorded (``timings()``; bench.py reports rank 0's and the slowest rank's), and when a watch is
installed a stage that outlives its bound ends the PROCESS with exit code ``EXIT_CODE`` and a line naming the stage
and the rank: a rank parked in a collective or a device wait cannot be interrupted from Python, and waiting for the
driver's own timeout would report nothing.  The reference has no counterpart (its only remote call,
``/root/reference/scheduler.py:425-433``, is an HTTPS request with no timeout passed).

Test hook: ``K8S_STALL_STAGE=<name>`` sleeps inside that stage (the CPU suite forces every stage's timeout with it).
"""

from __future__ import annotations

import contextlib
import os
import sys
import threading
import time
from typing import Dict, Optional

EXIT_CODE = 3

# default bounds (s); K8S_STAGE_TIMEOUT_<NAME> overrides one, K8S_STAGE_TIMEOUT_S all of those not set
DEFAULT_BOUNDS = {
    "process_group": 300.0,
    "rccl_init": 180.0,
    "xgmi_open": 120.0,
    "xgmi_selftest": 120.0,
    "fused_ar_selftest": 120.0,
    "comm_autotune": 300.0,
    "engine_build": 1200.0,
    "graph_capture": 1200.0,
    "warmup": 1200.0,
}

_lock = threading.Lock()
_timings: Dict[str, float] = {}
_watch: Optional["StageWatch"] = None


class StageWatch:
    """Deadline thread: at most one stage is open per process (stages do not nest); past its bound the process exits."""

    def __init__(self, rank: int = 0, bounds: Optional[Dict[str, float]] = None, period_s: float = 0.05):
        self.rank = rank
        self.bounds = dict(DEFAULT_BOUNDS)
        every = os.environ.get("K8S_STAGE_TIMEOUT_S")
        if every:
            self.bounds = {k: float(every) for k in self.bounds}
        for k in list(self.bounds) + list(bounds or {}):
            env = os.environ.get(f"K8S_STAGE_TIMEOUT_{k.upper()}")
            if env:
                self.bounds[k] = float(env)
            elif bounds and k in bounds:
                self.bounds[k] = float(bounds[k])
        self.period_s = period_s
        self._open: Optional[tuple] = None      # (name, deadline)
        self._stop = threading.Event()
        self._thr = threading.Thread(target=self._run, name="stage-watch", daemon=True)
        self._thr.start()

    def bound(self, name: str) -> float:
        return self.bounds.get(name, float(os.environ.get("K8S_STAGE_TIMEOUT_S", "1200")))

    def _run(self) -> None:
        while not self._stop.wait(self.period_s):
            cur = self._open
            if cur is not None and time.monotonic() > cur[1]:
                name, _, t0 = cur
                print(f"[stage] rank {self.rank}: start-up stage '{name}' exceeded its bound of "
                      f"{self.bound(name):.0f}s ({time.monotonic() - t0:.1f}s open); exiting with code {EXIT_CODE}",
                      file=sys.stderr, flush=True)
                os._exit(EXIT_CODE)

    def close(self) -> None:
        self._stop.set()


def install(rank: int = 0, bounds: Optional[Dict[str, float]] = None) -> StageWatch:
    global _watch
    if _watch is None:
        _watch = StageWatch(rank, bounds)
    return _watch


def uninstall() -> None:
    global _watch
    if _watch is not None:
        _watch.close()
        _watch = None


@contextlib.contextmanager
def stage(name: str):
    """Time (and, with a watch installed, bound) one start-up stage."""
    w = _watch
    t0 = time.monotonic()
    if w is not None:
        w._open = (name, t0 + w.bound(name), t0)
    try:
        if os.environ.get("K8S_STALL_STAGE") == name:
            time.sleep(float(os.environ.get("K8S_STALL_S", "3600")))
        yield
    finally:
        if w is not None:
            w._open = None
        with _lock:
            _timings[name] = round(_timings.get(name, 0.0) + time.monotonic() - t0, 3)


def timings() -> Dict[str, float]:
    with _lock:
        return dict(_timings)
