"""Decision backends: what answers the chat request the reference sends to HuggingFace
(``scheduler.py:425-433``).

* :class:`ScriptedBackend`  -- the FakeEngine of SURVEY.md section 4 (T2): scripted texts,
  exceptions, hangs, per-call callables.  Used by tests and by the fault-injection hook.
* :class:`LocalEngineBackend` -- the in-process Llama decision engine on MI355X
  (``engine.LLMEngine``): chat template + tokenize, continuous-batched prefill/decode,
  detokenize.  Enforces ``llm.timeout`` as a per-call deadline.
* ``None`` (no backend) -- "LLM disabled": the decision service falls back immediately
  (BASELINE config 1, CPU-only plumbing).
"""

from __future__ import annotations

import threading
import time
from typing import Callable, List, Optional, Sequence, Union

from .decision import GenerationRequest

Script = Union[str, BaseException, Callable[[GenerationRequest], str], "Hang"]


class Hang:
    """Script entry that blocks for ``seconds`` (then raises TimeoutError) - an engine hang."""

    def __init__(self, seconds: float):
        self.seconds = seconds


class ScriptedBackend:
    name = "scripted"

    def __init__(self, script: Sequence[Script] = (), default: Optional[Script] = None):
        self._script: List[Script] = list(script)
        self.default = default
        self.calls: List[List[GenerationRequest]] = []
        self._lock = threading.Lock()

    def push(self, *entries: Script) -> None:
        with self._lock:
            self._script.extend(entries)

    def _next(self) -> Optional[Script]:
        with self._lock:
            return self._script.pop(0) if self._script else self.default

    def complete(self, requests: Sequence[GenerationRequest]) -> List[str]:
        self.calls.append(list(requests))
        out: List[str] = []
        for r in requests:
            entry = self._next()
            if entry is None:
                raise RuntimeError("scripted backend exhausted")
            if isinstance(entry, BaseException):
                raise entry
            if isinstance(entry, Hang):
                limit = r.deadline_s if r.deadline_s is not None else entry.seconds
                time.sleep(min(entry.seconds, limit))
                raise TimeoutError(f"engine did not answer within {limit}s")
            out.append(entry(r) if callable(entry) else str(entry))
        return out


def first_node_answer(req: GenerationRequest) -> str:
    """A well-formed answer naming the first node listed in the prompt (LLM-success path)."""
    marker = "VALID NODE NAMES: "
    line = req.user[req.user.index(marker) + len(marker):].split("\n", 1)[0]
    node = line.split(", ")[0]
    return ('{"selected_node": "%s", "confidence": 0.85, "reasoning": "Lowest utilisation"}' % node)


class LocalEngineBackend:
    """Adapter from chat requests to the in-process engine (engine.LLMEngine)."""

    name = "local"

    def __init__(self, engine, ignore_eos: Optional[bool] = None,
                 forced_answer: Optional[Callable[[GenerationRequest], str]] = None):
        """``forced_answer`` (tests / benchmarks of the LLM-success path): the engine still runs the
        full prefill and decode, but reports the tokens of ``forced_answer(request)``."""
        self.engine = engine
        self.ignore_eos = ignore_eos
        self.forced_answer = forced_answer

    def complete(self, requests: Sequence[GenerationRequest]) -> List[str]:
        from ..engine.sampling import SamplingParams

        deadline = None
        if requests and requests[0].deadline_s:
            deadline = time.monotonic() + float(requests[0].deadline_s)
        prompts, params = [], []
        for r in requests:
            prompts.append(self.engine.render_chat(r.system, r.user))
            forced = None
            if self.forced_answer is not None:
                forced = self.engine.tok.encode(self.forced_answer(r))
            params.append(SamplingParams(max_tokens=r.max_tokens, temperature=r.temperature, top_p=r.top_p,
                                         ignore_eos=bool(self.ignore_eos) and forced is None,
                                         forced_output_ids=forced))
        outs = self.engine.generate(prompts, params, deadline=deadline)
        return [o.text for o in outs]


class FaultInjectingBackend:
    """Chaos hook around any backend (failure detection): with probability
    ``rate`` an engine call raises, hangs past its deadline, or answers garbage, so the retry /
    circuit-breaker / fallback machinery can be exercised against the real engine.

    Spec string (``engine.fault_injection`` / ``K8S_FAULT_INJECTION``): ``none`` or
    ``<mode>:<rate>`` with mode in raise | hang | garbage, e.g. ``raise:0.1``."""

    MODES = ("raise", "hang", "garbage")

    def __init__(self, inner, mode: str, rate: float, seed: int = 0, hang_s: float = 3600.0):
        if mode not in self.MODES:
            raise ValueError(f"fault mode must be one of {self.MODES}, got {mode!r}")
        import random

        self.inner, self.mode, self.rate, self.hang_s = inner, mode, float(rate), hang_s
        self.name = f"{getattr(inner, 'name', 'backend')}+fault({mode}:{rate})"
        self._rng = random.Random(seed)
        self._lock = threading.Lock()
        self.injected = 0

    @classmethod
    def from_spec(cls, inner, spec: Optional[str], seed: int = 0):
        if not spec or spec.strip().lower() in ("none", "off", ""):
            return inner
        mode, _, rate = spec.partition(":")
        return cls(inner, mode.strip().lower(), float(rate or 1.0), seed=seed)

    def complete(self, requests: Sequence[GenerationRequest]) -> List[str]:
        with self._lock:
            hit = self._rng.random() < self.rate
            if hit:
                self.injected += 1
        if not hit:
            return self.inner.complete(requests)
        if self.mode == "raise":
            raise RuntimeError("injected engine fault")
        if self.mode == "hang":
            limit = min((r.deadline_s for r in requests if r.deadline_s), default=self.hang_s)
            time.sleep(limit)
            raise TimeoutError(f"injected engine hang ({limit}s)")
        return ["\x00garbage{{" for _ in requests]
