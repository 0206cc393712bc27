#!/usr/bin/env python3
"""Train the built-in synthetic byte-level BPE tokenizer (no network: the Llama-3 tokenizer.json
cannot be downloaded here).

Design goal: token counts close to what Llama-3's 128k-vocab tokenizer produces on scheduler
prompts, so prefill work in benchmarks is realistic.  We therefore use Llama-3's own
pre-tokenisation regex (words, 1-3 digit groups, punctuation runs, newlines) and train a BPE
large enough that domain words become single tokens, exactly like in Llama-3's vocabulary.
The corpus is rendered from the real prompt template with random clusters/pods plus JSON
answers.  Output: k8s_llm_scheduler_amd/engine/assets/k8s_bpe.json (deterministic, seed 0).
"""

import random
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers  # noqa: E402

from k8s_llm_scheduler_amd.engine.synthetic import random_cluster_prompt, random_answer  # noqa: E402

LLAMA3_SPLIT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*"
                r"|\s*[\r\n]+|\s+(?!\S)|\s+")
BASE_VOCAB = 16000


def corpus(n: int = 3000, seed: int = 0):
    rng = random.Random(seed)
    for _ in range(n):
        yield random_cluster_prompt(rng, rng.choice([1, 2, 3, 3, 4, 5, 8, 16, 32]))[0]
        yield random_answer(rng)


def main() -> int:
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_SPLIT), behavior="isolated"),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False),
    ])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=BASE_VOCAB, min_frequency=2, show_progress=False,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(corpus(), trainer=trainer)
    out = ROOT / "k8s_llm_scheduler_amd" / "engine" / "assets" / "k8s_bpe.json"
    out.parent.mkdir(parents=True, exist_ok=True)
    tok.save(str(out))
    rng = random.Random(1)
    p, _ = random_cluster_prompt(rng, 3)
    n = len(tok.encode(p).ids)
    print(f"saved {out} vocab={tok.get_vocab_size()} 3-node prompt: {len(p)} chars -> {n} tokens "
          f"({len(p) / n:.2f} chars/token)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
