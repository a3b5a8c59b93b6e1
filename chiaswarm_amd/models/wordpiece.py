"""BERT WordPiece tokenizer (own implementation) for the BLIP decoder.

Uses ``vocab.txt`` from a local model directory when present; otherwise a
deterministic synthetic vocabulary (ids <-> "w<id>") so the captioning
workflow runs end to end with random weights.
"""
from __future__ import annotations

import os
import re
import zlib


class WordPiece:
    def __init__(self, model_dir: str | None = None, vocab_size: int = 30524, lower: bool = True):
        self.lower = lower
        self.vocab: dict[str, int] = {}
        self.inv: dict[int, str] = {}
        self.vocab_size = vocab_size
        path = os.path.join(model_dir, "vocab.txt") if model_dir else None
        if path and os.path.exists(path):
            with open(path, encoding="utf-8") as f:
                for i, tok in enumerate(f.read().split("\n")):
                    if tok:
                        self.vocab[tok] = i
            self.inv = {i: t for t, i in self.vocab.items()}

    def _synthetic(self, word: str) -> int:
        lo = min(1000, self.vocab_size // 4)
        return lo + zlib.crc32(word.encode()) % max(1, self.vocab_size - lo - 4)

    def encode(self, text: str) -> list[int]:
        words = re.findall(r"\w+|[^\w\s]", text.lower() if self.lower else text)
        if not self.vocab:
            return [self._synthetic(w) for w in words]
        ids = []
        for w in words:
            start = 0
            while start < len(w):
                end, cur = len(w), None
                while start < end:
                    piece = ("##" if start else "") + w[start:end]
                    if piece in self.vocab:
                        cur = self.vocab[piece]
                        break
                    end -= 1
                if cur is None:
                    ids.append(self.vocab.get("[UNK]", 100))
                    break
                ids.append(cur)
                start = end
        return ids

    def decode(self, ids: list[int]) -> str:
        if not self.inv:
            return " ".join(f"w{i}" for i in ids)
        toks = [self.inv.get(i, "") for i in ids]
        toks = [t for t in toks if t and not (t.startswith("[") and t.endswith("]"))]
        s = " ".join(toks).replace(" ##", "")
        return re.sub(r" ([.,!?;:'])", r"\1", s).strip()
