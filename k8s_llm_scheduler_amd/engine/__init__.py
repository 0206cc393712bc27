"""In-process decision engine (replaces the HuggingFace Inference API call of the reference)."""

from __future__ import annotations

import logging
import os
import time
from pathlib import Path
from typing import Optional

from .sampling import SamplingParams  # noqa: F401
from .tokenizer import Tokenizer  # noqa: F401

log = logging.getLogger(__name__)

GEMM_TABLE = Path(__file__).resolve().parent / "assets" / "tunableop_gfx950.csv"
_GEMM_TABLE_LOADED = False


def _load_gemm_table() -> bool:
    """Pin the library GEMMs (hipBLASLt / rocBLAS through F.linear) to the solutions ``tools/tune_gemms.py``
    measured fastest on MI355X (PyTorch TunableOp table, read with tuning OFF, so captured graphs replay fixed
    kernels; shapes missing from the table keep the library default).  The engine only issues library GEMMs
    with K8S_GEMM=library (the A/B oracle of the hand-written kernels) -- the GEMM tuners load it for their
    library columns.  K8S_GEMM_TABLE=0 disables; a table written by another torch / hipBLASLt / arch fails its
    validators and is ignored."""
    global _GEMM_TABLE_LOADED
    if _GEMM_TABLE_LOADED:
        return True
    if os.environ.get("K8S_GEMM_TABLE", "1") == "0" or not GEMM_TABLE.is_file():
        return False
    import torch

    t = torch.cuda.tunable
    try:
        t.enable(True)
        t.tuning_enable(False)
        # anything TunableOp writes back at exit goes to a scratch file, never over the asset
        t.set_filename(os.path.join(os.environ.get("TMPDIR", "/tmp"), f"k8s_tunableop_{os.getpid()}.csv"))
        ok = bool(t.read_file(str(GEMM_TABLE)))
    except Exception as e:  # noqa: BLE001 -- an unusable table only costs the library default
        log.warning(f" GEMM table not loaded: {e}")
        ok = False
    if not ok:
        t.enable(False)
    _GEMM_TABLE_LOADED = ok
    return ok


def resolve_tokenizer(weights: Optional[str], tokenizer: Optional[str]) -> Optional[str]:
    """The tokenizer a checkpoint must be served with: an explicit ``engine.tokenizer``, else the
    checkpoint's own ``tokenizer.json``.  Real weights fed the built-in synthetic vocabulary would
    answer garbage on every request (all decisions silently falling back), so a checkpoint without a
    tokenizer is an error; only random-init engines (no weights) use the synthetic tokenizer."""
    if tokenizer:
        return tokenizer
    if not weights:
        return None
    cand = Path(weights) / "tokenizer.json" if Path(weights).is_dir() else Path(weights).with_name("tokenizer.json")
    if cand.is_file():
        return str(cand)
    raise FileNotFoundError(f"engine.weights={weights} has no tokenizer.json next to it; set engine.tokenizer "
                            "to the checkpoint's tokenizer (the built-in synthetic vocabulary only fits "
                            "random-init weights)")


def warm_gemms(model) -> None:
    """Run every routed GEMM shape the engine can issue below 1k rows (layer 0's projections at each row bucket of
    ops.GEMM_M_BUCKETS) once, so every kernel / tile variant is loaded now instead of inside the first timed
    prefill (a first-use code-object load cost ~0.3 s in a TP=8-shape run)."""
    import torch

    from .. import ops

    w = model.layers[0]
    for W in (w.wqkv, w.wo, w.wgu, w.wdown):
        K = W.q.shape[1] if ops._is_fp8(W) else W.shape[1]
        for M in ops.GEMM_M_BUCKETS:
            x = torch.zeros(M, K, dtype=torch.bfloat16, device=model.device)
            ops.linear(x, W)
    torch.cuda.synchronize()


def build_engine(preset: str = "llama-3.3-70b", *, tp=None, device: Optional[str] = None, weights: Optional[str] = None,
                 tokenizer: Optional[str] = None, seed: int = 0, max_batch: int = 64, block_size: int = 16,
                 num_blocks: Optional[int] = None, kv_cache_gb: float = 0.0, kv_cache_fraction: float = 0.85,
                 max_model_len: int = 16384, max_prefill_tokens: int = 8192, cuda_graphs: bool = True,
                 prefix_caching: bool = True, decode_chunk: int = 4, metrics=None, capture: bool = True, control=None,
                 weight_dtype: str = "bf16", capture_nucleus: bool = False, speculative_tokens: int = 0,
                 watchdog_s: float = 60.0, on_unrecoverable: str = "stay", mixed_step_rows: int = 256):
    """Model + tokenizer + engine on this rank's GPU (or CPU when no GPU is present).
    ``weight_dtype``: "bf16" or "fp8" (row-scaled e4m3 projection weights).  ``capture_nucleus``:
    decode graphs with the top-p sampler passes too (serving with top_p < 1)."""
    import torch

    from ..models.config import get_config
    from ..models.llama import LlamaModel
    from ..parallel import TPGroup
    from .engine import LLMEngine

    tp = tp or TPGroup()
    if device is None:
        device = f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available() else "cpu"
    cfg = get_config(weights or preset) if weights else get_config(preset)
    from .. import ops

    if device.startswith("cuda") and ops.GEMM_BACKEND == "library":
        _load_gemm_table()
    t0 = time.perf_counter()
    model = LlamaModel(cfg, tp, device=device, seed=seed, weights=weights, max_model_len=max_model_len,
                       weight_dtype=weight_dtype)
    if device.startswith("cuda"):
        torch.cuda.synchronize()
    log.info(f" Model {cfg.name} ready on {device} (tp {tp.rank}/{tp.world}, "
             f"{model.weight_bytes() / 1e9:.1f} GB weights, {time.perf_counter() - t0:.1f}s)")
    tok = Tokenizer(resolve_tokenizer(weights, tokenizer), model_vocab=cfg.vocab)
    eng = LLMEngine(model, tok, max_batch=max_batch, block_size=block_size, num_blocks=num_blocks,
                    kv_cache_gb=kv_cache_gb, kv_cache_fraction=kv_cache_fraction, max_model_len=max_model_len,
                    max_prefill_tokens=max_prefill_tokens, cuda_graphs=cuda_graphs, prefix_caching=prefix_caching,
                    decode_chunk=decode_chunk, seed=seed, metrics=metrics, control=control,
                    capture_nucleus=capture_nucleus, speculative_tokens=speculative_tokens, watchdog_s=watchdog_s,
                    on_unrecoverable=on_unrecoverable, mixed_step_rows=mixed_step_rows)
    if device.startswith("cuda"):
        warm_gemms(model)
    if capture and eng.use_graphs:
        t1 = time.perf_counter()
        eng.capture_graphs()
        log.info(f" Captured {len(eng.graphs)} decode graphs in {time.perf_counter() - t1:.1f}s")
    return eng


def engine_from_config(cfg, tp=None, metrics=None, control=None):
    e = cfg.engine
    return build_engine(e.preset, tp=tp, weights=e.weights, tokenizer=e.tokenizer, seed=e.seed,
                        max_batch=e.max_batch, block_size=e.block_size, kv_cache_gb=e.kv_cache_gb,
                        kv_cache_fraction=e.kv_cache_fraction, max_model_len=e.max_model_len,
                        max_prefill_tokens=e.max_prefill_tokens, cuda_graphs=e.cuda_graphs,
                        prefix_caching=e.prefix_caching, metrics=metrics, control=control,
                        weight_dtype="fp8" if e.dtype in ("fp8", "fp8_e4m3") else "bf16",
                        capture_nucleus=cfg.llm.top_p < 1.0 and cfg.llm.temperature > 0,
                        speculative_tokens=e.speculative_tokens, decode_chunk=e.decode_chunk,
                        watchdog_s=e.watchdog_s or float(cfg.llm.timeout), on_unrecoverable=e.on_unrecoverable,
                        mixed_step_rows=e.mixed_step_rows)
