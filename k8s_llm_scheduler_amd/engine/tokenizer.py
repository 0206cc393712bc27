"""Tokenizer + Llama-3 chat template.

``Tokenizer(path)`` loads a real HuggingFace ``tokenizer.json`` (Llama-3's, when available);
without one it uses the built-in synthetic byte-level BPE (``assets/k8s_bpe.json``, trained by
``tools/make_tokenizer.py`` with Llama-3's pre-tokeniser on scheduler prompts: ~3.5 chars/token,
the same granularity as Llama-3 on this text).  Special tokens keep Llama-3's layout at the top
of the model vocabulary: ``<|begin_of_text|>`` = V-256, ``<|end_of_text|>`` = V-255,
``<|start_header_id|>`` = V-250, ``<|end_header_id|>`` = V-249, ``<|eom_id|>`` = V-248,
``<|eot_id|>`` = V-247 (128000.. for V = 128256).
"""

from __future__ import annotations

from pathlib import Path
from typing import List, Optional, Sequence

from tokenizers import Tokenizer as _HFTok

ASSET = Path(__file__).resolve().parent / "assets" / "k8s_bpe.json"
SPECIAL_OFFSETS = {"<|begin_of_text|>": 0, "<|end_of_text|>": 1, "<|start_header_id|>": 6,
                   "<|end_header_id|>": 7, "<|eom_id|>": 8, "<|eot_id|>": 9}


class Tokenizer:
    def __init__(self, path: Optional[str] = None, model_vocab: int = 128256):
        self.model_vocab = model_vocab
        self.synthetic = path is None
        self._tok = _HFTok.from_file(str(path or ASSET))
        if self.synthetic:
            base = model_vocab - 256
            if self._tok.get_vocab_size() > base:
                raise ValueError("synthetic tokenizer does not fit the model vocabulary")
            self.special = {k: base + off for k, off in SPECIAL_OFFSETS.items()}
        else:
            self.special = {}
            for k in SPECIAL_OFFSETS:
                i = self._tok.token_to_id(k)
                if i is None:
                    raise ValueError(f"tokenizer lacks {k}")
                self.special[k] = i
        self._special_ids = set(self.special.values())
        self.bos_id = self.special["<|begin_of_text|>"]
        self.eot_id = self.special["<|eot_id|>"]
        self.eos_ids = {self.special["<|end_of_text|>"], self.special["<|eom_id|>"], self.eot_id}

    def encode(self, text: str) -> List[int]:
        return self._tok.encode(text, add_special_tokens=False).ids

    def decode(self, ids: Sequence[int]) -> str:
        limit = self._tok.get_vocab_size() if self.synthetic else self.model_vocab
        keep = [int(i) for i in ids if int(i) not in self._special_ids and 0 <= int(i) < limit]
        return self._tok.decode(keep, skip_special_tokens=True)

    def chat_ids(self, system: str, user: str, knowledge_dates: bool = True) -> List[int]:
        """Llama-3 chat template, generation prompt for the assistant turn.  Llama-3.3 also puts
        "Cutting Knowledge Date / Today Date" lines at the top of the system turn."""
        sh, eh, eot = self.special["<|start_header_id|>"], self.special["<|end_header_id|>"], self.eot_id
        if knowledge_dates:
            system = "Cutting Knowledge Date: December 2023\nToday Date: 26 Jul 2024\n\n" + system
        ids = [self.bos_id]
        for role, content in (("system", system), ("user", user)):
            ids += [sh] + self.encode(role) + [eh] + self.encode("\n\n" + content.strip()) + [eot]
        ids += [sh] + self.encode("assistant") + [eh] + self.encode("\n\n")
        return ids
