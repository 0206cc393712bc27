"""The blocking ``generate`` API and the background serving loop: callers only enqueue and wait on their requests'
events while one thread runs engine steps.  Mixed into :class:`~.engine.LLMEngine`; the reference's counterpart is the
synchronous ``chat_completion`` call (``/root/reference/scheduler.py:425-433``)."""

from __future__ import annotations

import threading
import time
from typing import List, Optional, Sequence, Union
import logging

import torch

from ..parallel.comm import CollectiveError
from .sampling import SamplingParams
from .common import EngineStalled, EngineUnavailable, RequestRejected, Request, Output

log = logging.getLogger(__name__)


class ServingMixin:
    """Background serving loop and the blocking generate API."""

    # ------------------------------------------------------------------ background serving loop
    def start_background(self) -> None:
        """Run engine steps on a dedicated thread.  generate() then only enqueues and waits, so requests
        from any number of caller threads (the scheduler's continuous mode) join the running batch at the
        next step instead of waiting for each other's calls to finish."""
        if self._bg_thread is not None:
            return
        self._bg_stop = False
        self._bg_error = None
        self._bg_thread = threading.Thread(target=self._bg_loop, name="engine-loop", daemon=True)
        self._bg_thread.start()

    def stop_background(self) -> None:
        t = self._bg_thread
        if t is None:
            return
        with self._wake:
            self._bg_stop = True
            self._wake.notify_all()
        t.join()
        self._bg_thread = None

    @property
    def background(self) -> bool:
        return self._bg_thread is not None

    def _bg_loop(self) -> None:
        if self.gpu:
            torch.cuda.set_device(self.s_tokens.device)   # (the tensors carry the index; "cuda" alone does not)
        while True:
            with self._wake:
                while not self._bg_stop and not self._inbox and not self.has_work():
                    self._wake.wait(0.05)
                if self._bg_stop:
                    return
            try:
                if not self.ready:
                    # requests queued while not ready fail fast (the decision service falls back); a recovery
                    # attempt with a short drain bound runs before each wait
                    if not self.recover(drain_timeout=0.05):
                        self._fail_pending(EngineUnavailable(self.health["reason"] or "engine not ready"))
                        with self._wake:
                            self._wake.wait(0.05)
                        continue
                self.step()
                time.sleep(0)   # let threads blocked on the GIL / engine lock in before the next step
            except RequestRejected as e:   # only the offending request fails
                r = e.request
                r.error = e
                self._finish(r, "error")
            except (CollectiveError, EngineStalled, EngineUnavailable) as e:
                # collective state unknown: every in-flight request fails; recovery runs on the next iteration
                self._bg_error = e
                self._fail_pending(e)
            except Exception as e:  # noqa: BLE001 -- host-side bug: fail what was in flight, keep serving
                log.error(f"Engine step failed: {e!r}")
                self._bg_error = e
                self._fail_pending(e)

    def _fail_pending(self, e: BaseException) -> None:
        with self.lock:
            self._drain_inbox()
            for r in list(self.requests.values()):
                if not r.finished:
                    r.error = e
                    if r in self.waiting:
                        self.waiting.remove(r)
                    self._finish(r, "error")

    # ------------------------------------------------------------------ blocking API
    def output(self, r: Request) -> Output:
        end = r.finish_time or time.perf_counter()
        return Output(r.rid, self.tok.decode(r.output_ids), list(r.output_ids), len(r.prompt_ids), r.cached,
                      r.finish_reason, (r.first_token_time or end) - r.arrival, end - r.arrival)

    def generate(self, prompts: Sequence[Union[str, List[int]]],
                 params: Union[SamplingParams, Sequence[SamplingParams], None] = None,
                 deadline: Optional[float] = None) -> List[Output]:
        """Run the given requests to completion (continuous batching with whatever else is
        queued).  ``deadline`` (time.monotonic) aborts unfinished requests and raises
        TimeoutError -- the decision service counts that as an engine failure."""
        if params is None or isinstance(params, SamplingParams):
            params = [params or SamplingParams()] * len(prompts)
        if self._bg_thread is not None:
            return self._generate_bg(prompts, params, deadline)
        self.recovery_trace.append((time.monotonic(), f"generate: ready={self.ready}"))
        if not self.ready and not self.recover(drain_timeout=0.05):
            raise EngineUnavailable(self.health["reason"] or "decision engine not ready")
        with self.lock:
            self._call_deadline = deadline
            try:
                return self._generate_sync(prompts, params, deadline)
            finally:
                self._call_deadline = None

    def _generate_sync(self, prompts, params, deadline: Optional[float]) -> List[Output]:
        reqs = [self.add_request(p, sp) for p, sp in zip(prompts, params)]
        while not all(r.finished for r in reqs):
            if deadline is not None and time.monotonic() > deadline:
                for r in reqs:
                    if not r.finished:
                        r.aborted = True
                if self.control is None:
                    self._reap_aborted()
                for r in reqs:
                    self.requests.pop(r.rid, None) if r.finished else None
                raise TimeoutError("decision engine deadline exceeded")
            try:
                self.step()
            except StopIteration:
                raise
            except RequestRejected as e:
                e.request.error = e
                self._finish(e.request, "error")
                if e.request in reqs:
                    for r in reqs:
                        if not r.finished:
                            if r in self.waiting:
                                self.waiting.remove(r)
                            self._finish(r, "error")
                        self.requests.pop(r.rid, None)
                    raise
            except Exception:
                # an engine / collective failure ends these requests (their slots and KV blocks
                # are released) and propagates to the decision service's retry / breaker path
                for r in reqs:
                    if not r.finished:
                        if r in self.waiting:
                            self.waiting.remove(r)
                        self._finish(r, "error")
                    self.requests.pop(r.rid, None)
                raise
        outs = [self.output(r) for r in reqs]
        for r in reqs:
            self.requests.pop(r.rid, None)
        return outs

    def _generate_bg(self, prompts, params, deadline: Optional[float]) -> List[Output]:
        reqs = [self.add_request(p, sp) for p, sp in zip(prompts, params)]
        for r in reqs:
            left = None if deadline is None else max(0.0, deadline - time.monotonic())
            if not r.done.wait(timeout=left):
                for q in reqs:
                    q.aborted = True   # reaped (and finished) by the loop's next step; no engine lock here
                with self._wake:
                    self._wake.notify()
                raise TimeoutError("decision engine deadline exceeded")
        failed = next((r.error for r in reqs if r.error is not None), None)
        if failed is not None:
            raise RuntimeError(f"decision engine failure: {failed}") from failed
        return [self.output(r) for r in reqs]
