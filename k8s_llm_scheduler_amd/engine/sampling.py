"""Per-request generation parameters (the reference sends max_tokens=200, temperature=0.3 and
leaves top_p at the provider default, ``scheduler.py:425-433``)."""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class SamplingParams:
    max_tokens: int = 200
    temperature: float = 0.3
    top_p: float = 1.0
    seed: Optional[int] = None
    ignore_eos: bool = False
    stop_on_json_close: bool = True
    stop_token_ids: List[int] = field(default_factory=list)
    # Forced decode: the engine runs the full prefill + decode but reports these
    # tokens instead of the sampled ones (then stops), so the LLM-success path of the control
    # plane can be driven through the real engine with random-init weights.
    forced_output_ids: Optional[List[int]] = None

    def validate(self) -> "SamplingParams":
        if self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if not (0.0 < self.top_p <= 1.0):
            raise ValueError("top_p must be in (0, 1]")
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        return self
