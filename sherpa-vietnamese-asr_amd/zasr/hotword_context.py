"""Drop-in `core/hotword_context.py` host side.

The Aho-Corasick automaton itself (reference `core/hotword_context.py:17-184`) is built and
flattened inside libzasr (`build_hotword_dfa`, csrc/engine.cpp) and walked on device by the
search kernel.  What stays on the host is what the reference also does on the host: parse
the hotwords file (:191-222) and tokenize phrases with the model's sentencepiece model
(:225-259).
"""
from __future__ import annotations

import os
import unicodedata
from typing import List, Optional, Sequence, Tuple


def parse_hotwords_file(hotwords_path, default_score=1.5) -> List[Tuple[str, float]]:
    """'phrase' or 'phrase :score' per line; '#' comments; NFC upper-case phrases."""
    if not hotwords_path or not os.path.exists(hotwords_path):
        return []
    out = []
    with open(hotwords_path, "r", encoding="utf-8") as f:
        for raw in f:
            line = raw.strip()
            if not line or line.startswith("#"):
                continue
            score = default_score
            if ":" in line:
                head, tail = line.rsplit(":", 1)
                try:
                    score = float(tail.strip())
                    line = head.strip()
                except ValueError:
                    pass
            phrase = unicodedata.normalize("NFC", line.strip().upper())
            if phrase:
                out.append((phrase, score))
    return out


def build_context_graph(hotwords_path, bpe_model_path, default_score=1.5
                        ) -> Optional[Tuple[List[List[int]], List[float]]]:
    """Phrases -> (token id lists, scores) for zasr_create; None when there are no hotwords.
    (The reference returns a Python ContextGraph; here the graph lives in libzasr.)"""
    phrases = parse_hotwords_file(hotwords_path, default_score)
    if not phrases:
        return None
    import sentencepiece as spm
    sp = spm.SentencePieceProcessor()
    sp.load(bpe_model_path)
    seqs, scores = [], []
    for text, score in phrases:
        ids = sp.encode(text, out_type=int)
        if ids:
            seqs.append(list(ids))
            scores.append(float(score))
    return (seqs, scores) if seqs else None
