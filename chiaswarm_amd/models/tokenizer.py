"""CLIP byte-level BPE tokenizer (own implementation).

Loads ``vocab.json`` + ``merges.txt`` from a local model directory when one is
present (HF ``tokenizer/`` layout).  With no vocabulary on disk (this image has
no network and no checkpoints) it falls back to a deterministic hashing
tokenizer with the same interface and special tokens, which is what the
synthetic-prompt benchmarks use.
"""
from __future__ import annotations

import functools
import hashlib
import json
import os
import re

import torch

BOS, EOS = 49406, 49407

_PAT = re.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\w]+|[^\s\w]+""",
                  re.IGNORECASE)


@functools.lru_cache()
def _bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


class CLIPTokenizer:
    def __init__(self, model_dir: str | None = None, max_length: int = 77, pad_with_eos: bool = True,
                 vocab_size: int = 49408):
        self.max_length = max_length
        self.pad_with_eos = pad_with_eos
        self.vocab_size = vocab_size
        self.encoder = None
        if model_dir and os.path.exists(os.path.join(model_dir, "vocab.json")):
            with open(os.path.join(model_dir, "vocab.json"), encoding="utf-8") as f:
                self.encoder = json.load(f)
            with open(os.path.join(model_dir, "merges.txt"), encoding="utf-8") as f:
                merges = f.read().split("\n")[1:]
            merges = [tuple(m.split()) for m in merges if m.strip()]
            self.bpe_ranks = dict(zip(merges, range(len(merges))))
            self.byte_encoder = _bytes_to_unicode()
            self.cache: dict[str, str] = {}

    @property
    def bos(self):
        return BOS if self.vocab_size > BOS else self.vocab_size - 2

    @property
    def eos(self):
        return EOS if self.vocab_size > EOS else self.vocab_size - 1

    def _bpe(self, token: str) -> list[str]:
        if token in self.cache:
            return self.cache[token].split(" ")
        word = tuple(token[:-1]) + (token[-1] + "</w>",)
        while len(word) > 1:
            pairs = {(word[i], word[i + 1]) for i in range(len(word) - 1)}
            best = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if best not in self.bpe_ranks:
                break
            first, second = best
            new, i = [], 0
            while i < len(word):
                if i < len(word) - 1 and word[i] == first and word[i + 1] == second:
                    new.append(first + second)
                    i += 2
                else:
                    new.append(word[i])
                    i += 1
            word = tuple(new)
        self.cache[token] = " ".join(word)
        return list(word)

    def encode(self, text: str) -> list[int]:
        added = getattr(self, "added_tokens", None)
        if added:  # textual-inversion placeholders map to their appended embedding rows
            for tok, tids in added.items():
                if tok in text:
                    parts = text.split(tok)
                    out: list[int] = []
                    for i, part in enumerate(parts):
                        out.extend(self.encode_plain(part))
                        if i < len(parts) - 1:
                            out.extend(tids)
                    return out
        return self.encode_plain(text)

    def encode_plain(self, text: str) -> list[int]:
        text = " ".join(text.strip().lower().split())
        ids: list[int] = []
        for tok in _PAT.findall(text):
            if self.encoder is not None:
                t = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
                ids.extend(self.encoder[p] for p in self._bpe(t) if p in self.encoder)
            else:
                h = int.from_bytes(hashlib.blake2b(tok.encode(), digest_size=8).digest(), "little")
                ids.append(h % (min(self.vocab_size, BOS) - 1) + 1)
        return ids

    def __call__(self, texts: list[str] | str) -> torch.Tensor:
        if isinstance(texts, str):
            texts = [texts]
        out = []
        for t in texts:
            ids = [self.bos] + self.encode(t)[: self.max_length - 2] + [self.eos]
            pad = self.eos if self.pad_with_eos else 0
            ids = ids + [pad] * (self.max_length - len(ids))
            out.append(ids)
        return torch.tensor(out, dtype=torch.long)


class ByteBPETokenizer(CLIPTokenizer):
    """GPT-2 / RoBERTa byte-level BPE (``vocab.json`` + ``merges.txt``): the
    CLAP text tower of AudioLDM (RobertaTokenizer).  No lower-casing, no
    ``</w>`` suffix, spaces folded into the following token ("Ġ").  Hash
    fallback without vocabulary files, like ``CLIPTokenizer``."""

    def __init__(self, model_dir: str | None = None, max_length: int = 77, vocab_size: int = 50265,
                 bos: int = 0, eos: int = 2, pad: int = 1):
        super().__init__(model_dir, max_length, pad_with_eos=False, vocab_size=vocab_size)
        self._bos, self._eos, self.pad = bos, eos, pad
        import regex

        self._pat = regex.compile(r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")

    @property
    def bos(self):
        return self._bos

    @property
    def eos(self):
        return self._eos

    def _bpe(self, token: str) -> list[str]:
        if token in self.cache:
            return self.cache[token].split(" ")
        word = tuple(token)
        while len(word) > 1:
            pairs = {(word[i], word[i + 1]) for i in range(len(word) - 1)}
            best = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if best not in self.bpe_ranks:
                break
            first, second = best
            new, i = [], 0
            while i < len(word):
                if i < len(word) - 1 and word[i] == first and word[i + 1] == second:
                    new.append(first + second)
                    i += 2
                else:
                    new.append(word[i])
                    i += 1
            word = tuple(new)
        self.cache[token] = " ".join(word)
        return list(word)

    def encode_plain(self, text: str) -> list[int]:
        ids: list[int] = []
        for tok in self._pat.findall(text):
            if self.encoder is not None:
                t = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
                ids.extend(self.encoder[p] for p in self._bpe(t) if p in self.encoder)
            else:
                h = int.from_bytes(hashlib.blake2b(tok.encode(), digest_size=8).digest(), "little")
                ids.append(h % (self.vocab_size - 4) + 4)
        return ids

    def __call__(self, texts: list[str] | str, pad: bool = False) -> list[list[int]]:  # type: ignore[override]
        """Unpadded id lists ([bos] ids [eos]); attention needs no padding mask."""
        if isinstance(texts, str):
            texts = [texts]
        out = []
        for t in texts:
            ids = [self.bos] + self.encode(t)[: self.max_length - 2] + [self.eos]
            if pad:
                ids = ids + [self.pad] * (self.max_length - len(ids))
            out.append(ids)
        return out
