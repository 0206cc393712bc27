"""Llama-3 architecture presets (public config.json constants, SURVEY.md section 2.5 [ext])."""

from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field, replace
from pathlib import Path
from typing import Optional


@dataclass
class LlamaConfig:
    name: str
    num_layers: int
    hidden: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate: int
    vocab: int
    rms_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    max_position: int = 8192
    bos_id: int = 128000
    eos_ids: tuple = (128001, 128008, 128009)
    init_std: float = 0.02
    extra: dict = field(default_factory=dict)

    @property
    def params(self) -> int:
        L, H, I, V = self.num_layers, self.hidden, self.intermediate, self.vocab
        qkv = H * (self.num_heads + 2 * self.num_kv_heads) * self.head_dim
        o = self.num_heads * self.head_dim * H
        return V * H * 2 + L * (qkv + o + 3 * H * I + 2 * H) + H

    def kv_bytes_per_token(self, tp: int = 1, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * max(1, self.num_kv_heads // tp) * self.head_dim * dtype_bytes

    def validate_tp(self, tp: int) -> None:
        if self.num_heads % tp or self.intermediate % tp or self.vocab % tp:
            raise ValueError(f"{self.name}: heads/intermediate/vocab not divisible by tp={tp}")
        if self.num_kv_heads % tp and tp % self.num_kv_heads:
            raise ValueError(f"{self.name}: kv heads {self.num_kv_heads} incompatible with tp={tp}")

    def to_json(self) -> str:
        return json.dumps(asdict(self))


LLAMA3_ROPE_SCALING = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                       "original_max_position_embeddings": 8192}

PRESETS = {
    "llama-3.3-70b": LlamaConfig("llama-3.3-70b", 80, 8192, 64, 8, 128, 28672, 128256,
                                 rope_scaling=LLAMA3_ROPE_SCALING, max_position=131072),
    "llama-3-8b": LlamaConfig("llama-3-8b", 32, 4096, 32, 8, 128, 14336, 128256, max_position=8192),
    # tiny: same code paths (GQA 2:1, head_dim 128) at a size that runs on CPU in tests
    "tiny": LlamaConfig("tiny", 2, 256, 4, 2, 128, 512, 16384, bos_id=16128, eos_ids=(16129, 16136, 16137),
                        max_position=4096, rope_scaling=LLAMA3_ROPE_SCALING),
    # tiny-tp8: the 70B's head layout scaled down (GQA 2:1, 8 kv heads, head_dim 128), so TP = 1/2/4/8 all
    # shard like the 70B does (one kv head per rank at TP = 8) -- multi-rank tests
    "tiny-tp8": LlamaConfig("tiny-tp8", 2, 2048, 16, 8, 128, 4096, 16384, bos_id=16128,
                            eos_ids=(16129, 16136, 16137), max_position=4096, rope_scaling=LLAMA3_ROPE_SCALING),
}
PRESETS["llama-3-70b"] = PRESETS["llama-3.3-70b"]
PRESETS["llama-3.1-8b"] = LlamaConfig("llama-3.1-8b", 32, 4096, 32, 8, 128, 14336, 128256,
                                      rope_scaling=LLAMA3_ROPE_SCALING, max_position=131072)


def get_config(name_or_path: str) -> LlamaConfig:
    """A preset name, a HuggingFace config.json (or its directory), or ``<preset>@L<n>``: the preset's dimensions with
    ``n`` decoder layers (e.g. ``llama-3.3-70b@L2``: the 70B's exact per-layer and vocabulary shapes -- every kernel,
    shard and collective size of the headline -- at a depth that runs many times per test)."""
    if "@L" in name_or_path:
        base, n = name_or_path.rsplit("@L", 1)
        c = get_config(base)
        if not n.isdigit() or int(n) < 1:
            raise KeyError(f"bad layer count in {name_or_path!r}")
        return replace(c, name=f"{c.name}@L{n}", num_layers=int(n), extra=dict(c.extra))
    if name_or_path in PRESETS:
        return PRESETS[name_or_path]
    p = Path(name_or_path)
    if p.is_dir():
        p = p / "config.json"
    if p.is_file():
        return from_hf_config(json.loads(p.read_text()), p.parent.name)
    key = name_or_path.lower().split("/")[-1]
    for k in ("3.3-70b", "70b"):
        if k in key:
            return PRESETS["llama-3.3-70b"]
    if "8b" in key:
        return PRESETS["llama-3-8b"]
    raise KeyError(f"unknown model preset {name_or_path!r}; known: {sorted(PRESETS)}")


def from_hf_config(c: dict, name: str = "hf") -> LlamaConfig:
    """Map a HuggingFace LlamaForCausalLM config.json to LlamaConfig."""
    H, nh = c["hidden_size"], c["num_attention_heads"]
    eos = c.get("eos_token_id", 128009)
    return LlamaConfig(
        name=name, num_layers=c["num_hidden_layers"], hidden=H, num_heads=nh,
        num_kv_heads=c.get("num_key_value_heads", nh), head_dim=c.get("head_dim", H // nh),
        intermediate=c["intermediate_size"], vocab=c["vocab_size"], rms_eps=c.get("rms_norm_eps", 1e-5),
        rope_theta=c.get("rope_theta", 10000.0), rope_scaling=c.get("rope_scaling"),
        max_position=c.get("max_position_embeddings", 8192), bos_id=c.get("bos_token_id", 128000),
        eos_ids=tuple(eos) if isinstance(eos, list) else (eos,))
