"""Typed configuration with the reference's keys, defaults and precedence.

Reference: ``scheduler.py:44-66`` (loader + module globals) and ``config.yaml:1-43``.
Precedence is the reference's: **environment variable > config.yaml > built-in default**
(``scheduler.py:55-60``).  Differences, all deliberate and documented in docs/CONFIG.md:

* The config is an object injected into components instead of module globals, so tests can
  build variants.
* Keys the reference parses but never uses become live: ``llm.timeout`` is a per-decision
  deadline, ``llm.retry_delay`` is the backoff base (default keeps ``2**attempt`` seconds),
  ``logging.*`` configures logging, ``metrics.*`` starts a Prometheus endpoint,
  ``circuit_breaker.half_open_max_calls`` caps concurrent trial calls, ``scheduler.watch_interval``
  is the watch timeout.  ``ENABLE_CACHE``, ``CACHE_TTL``, ``ENABLE_METRICS`` and ``METRICS_PORT``
  (``.env.example:20-25``) are honoured as well.
* ``HUGGINGFACE_TOKEN`` is **not** required: the LLM runs in-process (``scheduler.py:62-66``
  exits without it; here it is only used if weights are to be downloaded, which never happens
  offline).
* A new ``engine:`` section configures the local decision engine and a ``compat:`` section
  selects reference-quirk preservation.
"""

from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, Mapping, Optional

import yaml


@dataclass
class SchedulerSection:
    name: str = "ai-llama-scheduler"          # config.yaml:3
    watch_interval: int = 60                  # config.yaml:4 (reference hard-codes 60, scheduler.py:666)
    mode: str = "sequential"                  # "sequential" (reference) | "batched" | "continuous"
    max_batch: int = 64                       # pending pods drained per batched round
    batch_window_ms: float = 20.0             # how long to wait for more pending pods
    error_backoff_s: float = 5.0              # scheduler.py:685


@dataclass
class LLMSection:
    model: str = "meta-llama/Llama-3.3-70B-Instruct"   # config.yaml:8
    endpoint: str = "local://mi355x"                    # reference: https://router.huggingface.co
    timeout: float = 60.0                               # config.yaml:10 (live here)
    max_retries: int = 3                                # config.yaml:11
    retry_delay: float = 2.0                            # config.yaml:12 (backoff base)
    temperature: float = 0.3                            # config.yaml:13
    max_tokens: int = 200                               # config.yaml:14
    top_p: float = 1.0                                  # provider default (not sent by reference)
    system_message: str = ("You are an intelligent Kubernetes scheduler. "
                           "Respond only with valid JSON.")  # scheduler.py:427


@dataclass
class CacheSection:
    enabled: bool = True
    ttl: float = 300.0
    max_size: int = 100


@dataclass
class LoggingSection:
    level: str = "INFO"
    format: str = "text"          # reference default via env is text (scheduler.py:28)
    file: Optional[str] = None


@dataclass
class MetricsSection:
    enabled: bool = True
    port: int = 9090


@dataclass
class FallbackSection:
    enabled: bool = True
    strategy: str = "resource_balanced"


@dataclass
class CircuitBreakerSection:
    enabled: bool = True
    failure_threshold: int = 5
    timeout: float = 60.0
    half_open_max_calls: int = 3


@dataclass
class EngineSection:
    """Local decision engine (replaces the HTTPS call at scheduler.py:425-433)."""

    enabled: bool = True               # False == BASELINE config 1 (fallback-only plumbing)
    backend: str = "local"             # local | fallback | scripted
    preset: str = "llama-3.3-70b"      # llama-3.3-70b | llama-3-8b | tiny
    tp: int = 0                        # 0 == WORLD_SIZE (one process per GPU)
    dtype: str = "bf16"
    weights: Optional[str] = None      # safetensors dir; None == deterministic random init
    tokenizer: Optional[str] = None    # tokenizer.json; None == built-in synthetic BPE
    seed: int = 0
    kv_cache_gb: float = 0.0           # 0 == size from free HBM (kv_cache_fraction)
    kv_cache_fraction: float = 0.85
    block_size: int = 16
    max_batch: int = 64
    max_model_len: int = 16384
    max_prefill_tokens: int = 8192     # chunked-prefill token budget per step
    mixed_step_rows: int = 256         # rows (prompt tokens + riding decodes) of a mixed step; 0 = no cap
    cuda_graphs: bool = True
    prefix_caching: bool = True
    speculative_tokens: int = 0        # prompt-lookup speculative decoding: draft tokens per step (0 = off)
    decode_chunk: int = 4              # decode graph replays per engine step (stops are detected on the device)
    watchdog_s: float = 0.0            # bound on any host wait for device results; 0 == llm.timeout
    on_unrecoverable: str = "exit"     # exit (pod restarts, code 70) | stay (not ready) when recovery fails
    ignore_eos: bool = False
    stop_on_json_close: bool = True
    fault_injection: str = "none"      # chaos hook: none | raise:<rate> | hang:<rate> | garbage:<rate>


@dataclass
class CompatSection:
    """Reference quirks: True == preserve the reference behaviour."""

    round_robin_picks_most_pods: bool = True     # scheduler.py:544-545 vs README.md:171
    prompt_status_always_ready: bool = True      # scheduler.py:240
    breaker_cumulative_failures: bool = True     # scheduler.py:325-332
    quantity_parsing: str = "full"               # "reference" reproduces scheduler.py:172-187/747-753
    watch_all_event_types: bool = False          # scheduler.py:664-681 (False: skip DELETED, dedupe)
    snapshot_mode: str = "informer"              # "direct" = N+1 REST calls (scheduler.py:124-147)
    prompt_layout: str = "reference"             # "cluster_first": node block before the pod block (prefix sharing)
    yaml_logging: bool = False                   # False: config.yaml's logging section is ignored, LOG_LEVEL /
                                                 # LOG_FORMAT env only (scheduler.py:27-28); True: section is live


@dataclass
class Config:
    scheduler: SchedulerSection = field(default_factory=SchedulerSection)
    llm: LLMSection = field(default_factory=LLMSection)
    cache: CacheSection = field(default_factory=CacheSection)
    logging: LoggingSection = field(default_factory=LoggingSection)
    metrics: MetricsSection = field(default_factory=MetricsSection)
    fallback: FallbackSection = field(default_factory=FallbackSection)
    circuit_breaker: CircuitBreakerSection = field(default_factory=CircuitBreakerSection)
    engine: EngineSection = field(default_factory=EngineSection)
    compat: CompatSection = field(default_factory=CompatSection)
    source: Optional[str] = None

    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        d.pop("source", None)
        return d


# env var -> (section, key, caster).  The first seven are read by the reference
# (scheduler.py:27-28, 55-60); the rest are advertised by .env.example:20-25 and made live.
def _bool(v: str) -> bool:
    return str(v).strip().lower() in ("1", "true", "yes", "on")


ENV_OVERRIDES = {
    "SCHEDULER_NAME": ("scheduler", "name", str),
    "LLM_MODEL": ("llm", "model", str),
    "LLM_ENDPOINT": ("llm", "endpoint", str),
    "LLM_TIMEOUT": ("llm", "timeout", float),
    "LLM_MAX_RETRIES": ("llm", "max_retries", int),
    "LOG_LEVEL": ("logging", "level", str),
    "LOG_FORMAT": ("logging", "format", str),
    "ENABLE_CACHE": ("cache", "enabled", _bool),
    "CACHE_TTL": ("cache", "ttl", float),
    "ENABLE_METRICS": ("metrics", "enabled", _bool),
    "METRICS_PORT": ("metrics", "port", int),
    "ENGINE_PRESET": ("engine", "preset", str),
    "ENGINE_BACKEND": ("engine", "backend", str),
    "ENGINE_WEIGHTS": ("engine", "weights", str),
    "ENGINE_TOKENIZER": ("engine", "tokenizer", str),
    "K8S_FAULT_INJECTION": ("engine", "fault_injection", str),
    "SCHEDULER_MODE": ("scheduler", "mode", str),
}

# The reference's LOG_LEVEL/LOG_FORMAT come only from env; config.yaml's logging section is
# ignored there (scheduler.py:27-28).  Here the section is honoured only with compat.yaml_logging: true
# (this repo's config.yaml sets it), so the reference's own config.yaml does not switch on JSON logs to
# scheduler.log; env still wins either way.


def load_dotenv(path: str | os.PathLike = ".env", environ: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """Minimal python-dotenv replacement (scheduler.py:23-24): KEY=VALUE lines, ``#`` comments,
    optional quotes; existing environment variables are NOT overridden (dotenv's default)."""
    env = os.environ if environ is None else environ
    p = Path(path)
    loaded: Dict[str, str] = {}
    if not p.is_file():
        return loaded
    for raw in p.read_text().splitlines():
        line = raw.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        if line.startswith("export "):
            line = line[len("export "):]
        key, _, val = line.partition("=")
        key, val = key.strip(), val.strip()
        if len(val) >= 2 and val[0] == val[-1] and val[0] in "\"'":
            val = val[1:-1]
        elif " #" in val:
            val = val.split(" #", 1)[0].rstrip()
        loaded[key] = val
        env.setdefault(key, val)
    return loaded


def _merge_section(obj: Any, values: Mapping[str, Any]) -> None:
    fields = {f.name: f for f in dataclasses.fields(obj)}
    for k, v in (values or {}).items():
        if k not in fields:
            continue  # unknown keys are tolerated, as in the reference (plain dict access)
        cur = getattr(obj, k)
        if v is None:
            setattr(obj, k, v)
        elif isinstance(cur, bool):
            setattr(obj, k, v if isinstance(v, bool) else _bool(v))
        elif isinstance(cur, int) and not isinstance(cur, bool):
            setattr(obj, k, int(v))
        elif isinstance(cur, float):
            setattr(obj, k, float(v))
        else:
            setattr(obj, k, v)


def from_dict(data: Mapping[str, Any]) -> Config:
    cfg = Config()
    for sec in ("compat", "scheduler", "llm", "cache", "logging", "metrics", "fallback",
                "circuit_breaker", "engine"):
        if sec == "logging" and not cfg.compat.yaml_logging:
            continue   # the reference never read it: its config.yaml's json/scheduler.log stay inert
        if isinstance(data.get(sec), Mapping):
            _merge_section(getattr(cfg, sec), data[sec])
    return cfg


def apply_env(cfg: Config, environ: Optional[Mapping[str, str]] = None) -> Config:
    env = os.environ if environ is None else environ
    for var, (sec, key, cast) in ENV_OVERRIDES.items():
        if var in env and env[var] != "":
            setattr(getattr(cfg, sec), key, cast(env[var]))
    return cfg


def default_config_path() -> Optional[Path]:
    """config.yaml lookup: $SCHEDULER_CONFIG, then ./config.yaml, then the repo copy.
    (The reference looks only next to its own script, scheduler.py:48.)"""
    cand = os.environ.get("SCHEDULER_CONFIG")
    if cand and Path(cand).is_file():
        return Path(cand)
    if Path("config.yaml").is_file():
        return Path("config.yaml")
    repo = Path(__file__).resolve().parent.parent / "config.yaml"
    return repo if repo.is_file() else None


def load_config(path: Optional[str | os.PathLike] = None,
                environ: Optional[Mapping[str, str]] = None,
                use_env: bool = True) -> Config:
    """Load YAML (missing file -> defaults, like scheduler.py:49-52) then apply env overrides."""
    p = Path(path) if path is not None else default_config_path()
    data: Dict[str, Any] = {}
    if p is not None and p.is_file():
        with open(p, "r") as f:
            data = yaml.safe_load(f) or {}
    cfg = from_dict(data)
    cfg.source = str(p) if p is not None and p.is_file() else None
    if use_env:
        apply_env(cfg, environ)
    return cfg
