"""Circuit breaker around the decision engine.

State machine of the reference ``CircuitBreaker`` (``scheduler.py:299-332``):

* CLOSED: calls pass; each failure increments ``failures``; reaching ``failure_threshold``
  opens the breaker.  A success in CLOSED does **not** reset the count (quirk 6, preserved when
  ``cumulative_failures`` is True, the default), so 5 *cumulative* failures open it.
* OPEN: calls are rejected with ``CircuitOpenError("Circuit breaker is OPEN")`` until
  ``timeout`` seconds have passed since the last failure, then the breaker goes HALF_OPEN.
* HALF_OPEN: a success closes it and zeroes the count; a failure re-opens it immediately
  (the count is still >= threshold).

``half_open_max_calls`` (``config.yaml:43``, unused in the reference) caps the number of trial
calls that may be *in flight* while HALF_OPEN; extra concurrent callers are rejected as OPEN.
With the reference's one-call-at-a-time loop this never triggers, so behaviour is identical.
The clock is injectable for tests; the breaker is thread-safe.
"""

from __future__ import annotations

import logging
import threading
import time
from typing import Any, Callable, Optional

log = logging.getLogger(__name__)

CLOSED, OPEN, HALF_OPEN = "CLOSED", "OPEN", "HALF_OPEN"


class CircuitOpenError(Exception):
    def __init__(self) -> None:
        super().__init__("Circuit breaker is OPEN")


class CircuitBreaker:
    def __init__(self, failure_threshold: int = 5, timeout: float = 60,
                 half_open_max_calls: int = 3, cumulative_failures: bool = True,
                 clock: Callable[[], float] = time.monotonic):
        self.failure_threshold = int(failure_threshold)
        self.timeout = float(timeout)
        self.half_open_max_calls = max(1, int(half_open_max_calls))
        self.cumulative_failures = cumulative_failures
        self.failures = 0
        self.last_failure_time: Optional[float] = None
        self.state = CLOSED
        self._clock = clock
        self._lock = threading.Lock()
        self._trials = 0

    def _admit(self) -> bool:
        """Returns True if this call is a HALF_OPEN trial."""
        with self._lock:
            if self.state == OPEN:
                if self._clock() - (self.last_failure_time or 0.0) > self.timeout:
                    log.info("Circuit breaker entering HALF_OPEN state")
                    self.state = HALF_OPEN
                else:
                    raise CircuitOpenError()
            if self.state == HALF_OPEN:
                if self._trials >= self.half_open_max_calls:
                    raise CircuitOpenError()
                self._trials += 1
                return True
            return False

    def record_success(self, trial: bool) -> None:
        with self._lock:
            if trial:
                self._trials -= 1
            if self.state == HALF_OPEN:
                log.info("Circuit breaker closing")
                self.state = CLOSED
                self.failures = 0
            elif not self.cumulative_failures:
                self.failures = 0

    def record_failure(self, trial: bool) -> None:
        with self._lock:
            if trial:
                self._trials -= 1
            self.failures += 1
            self.last_failure_time = self._clock()
            if self.failures >= self.failure_threshold:
                if self.state != OPEN:
                    log.error(f"Circuit breaker opening after {self.failures} failures")
                self.state = OPEN

    def call(self, fn: Callable[..., Any], *args: Any, **kwargs: Any) -> Any:
        trial = self._admit()
        try:
            result = fn(*args, **kwargs)
        except Exception:
            self.record_failure(trial)
            raise
        self.record_success(trial)
        return result
