r"""CLIP byte-level BPE tokenizer (own implementation).

Loads a HF ``tokenizer/`` directory (``vocab.json`` + ``merges.txt`` and, when
present, ``tokenizer_config.json`` / ``special_tokens_map.json`` for the
bos/eos/pad/unk tokens and ``model_max_length``) — the files the reference's
``DiffusionPipeline.from_pretrained`` reads (swarm/diffusion/diffusion_func.py:41-46).
Behaviour follows OpenAI CLIP / ``transformers.CLIPTokenizer``: NFC + whitespace
collapse + lower-case, the split pattern
``<|startoftext|>|<|endoftext|>|'s|'t|'re|'ve|'m|'ll|'d|\p{L}+|\p{N}|[^\s\p{L}\p{N}]+``
(digits are single tokens), byte-level BPE with a ``</w>`` word suffix, unknown
pieces -> unk, ``[bos] ids[:max-2] [eos]`` then pad.  The pad token is read
from the directory: SD1.x (CLIP-L) pads with ``<|endoftext|>``, SD2.x and
SDXL's second tokenizer (OpenCLIP) pad with ``!`` (id 0).

With no vocabulary on disk (this image has no network and no checkpoints) it
falls back to a deterministic hashing tokenizer with the same interface and
special tokens, which is what the synthetic-prompt benchmarks use.
"""
from __future__ import annotations

import functools
import hashlib
import json
import os
import unicodedata

import regex
import torch

BOS, EOS = 49406, 49407

_PAT = regex.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""",
                     regex.IGNORECASE)
_WS = regex.compile(r"\s+")


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


def _special(v):
    if isinstance(v, dict):
        return v.get("content")
    return v


def _read_specials(model_dir: str) -> dict:
    """bos/eos/pad/unk strings + model_max_length from the tokenizer directory."""
    out: dict = {}
    for name in ("special_tokens_map.json", "tokenizer_config.json"):
        f = os.path.join(model_dir, name)
        if not os.path.exists(f):
            continue
        with open(f, encoding="utf-8") as fh:
            cfg = json.load(fh)
        for k in ("bos_token", "eos_token", "pad_token", "unk_token"):
            if k in cfg and cfg[k] is not None and k not in out:
                out[k] = _special(cfg[k])
        if "model_max_length" in cfg and "model_max_length" not in out:
            try:
                m = int(cfg["model_max_length"])
                if 0 < m < 100000:
                    out["model_max_length"] = m
            except (TypeError, ValueError):
                pass
    return out


class CLIPTokenizer:
    def __init__(self, model_dir: str | None = None, max_length: int = 77, pad_with_eos: bool = True,
                 vocab_size: int = 49408):
        self.max_length = max_length
        self.pad_with_eos = pad_with_eos
        self.vocab_size = vocab_size
        self.encoder = None
        self.added_tokens: dict = {}
        self._pad_id = None
        self.source = "hash-fallback"
        if model_dir and os.path.exists(os.path.join(model_dir, "vocab.json")):
            self._load_bpe(model_dir, "</w>")
            sp = _read_specials(model_dir)
            self.max_length = sp.get("model_max_length", max_length)
            self._bos_id = self.encoder[sp.get("bos_token") or "<|startoftext|>"]
            self._eos_id = self.encoder[sp.get("eos_token") or "<|endoftext|>"]
            self._unk_id = self.encoder.get(sp.get("unk_token") or "<|endoftext|>", self._eos_id)
            pad = sp.get("pad_token")
            if pad is not None and pad in self.encoder:
                self._pad_id = self.encoder[pad]
            # special tokens are cut out of the raw text before BPE, exactly like
            # transformers' added-token matching (OpenCLIP's pad "!" included:
            # "wow!!" -> ..., pad, pad)
            specials = {t for t in (sp.get("bos_token") or "<|startoftext|>", sp.get("eos_token") or "<|endoftext|>",
                                    sp.get("unk_token") or "<|endoftext|>", pad) if t and t in self.encoder}
            self._special_re = regex.compile("(" + "|".join(regex.escape(t) for t in
                                                            sorted(specials, key=len, reverse=True)) + ")")
            self._specials = specials
            self.source = model_dir

    def _load_bpe(self, model_dir, suffix):
        with open(os.path.join(model_dir, "vocab.json"), encoding="utf-8") as f:
            self.encoder = json.load(f)
        with open(os.path.join(model_dir, "merges.txt"), encoding="utf-8") as f:
            lines = f.read().split("\n")
        if lines and lines[0].startswith("#version"):
            lines = lines[1:]
        merges = [tuple(m.split()) for m in lines if m.strip()]
        self.bpe_ranks = dict(zip(merges, range(len(merges))))
        self.byte_encoder = _bytes_to_unicode()
        self.cache: dict[str, str] = {}
        self.vocab_size = max(self.vocab_size, len(self.encoder))

    @property
    def loaded(self) -> bool:
        return self.encoder is not None

    @property
    def bos(self):
        if self.encoder is not None:
            return self._bos_id
        return BOS if self.vocab_size > BOS else self.vocab_size - 2

    @property
    def eos(self):
        if self.encoder is not None:
            return self._eos_id
        return EOS if self.vocab_size > EOS else self.vocab_size - 1

    @property
    def pad(self):
        if self._pad_id is not None:
            return self._pad_id
        return self.eos if self.pad_with_eos else 0

    def _merge(self, word: tuple) -> tuple:
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
        return word

    def _bpe(self, token: str) -> list[str]:
        if token in self.cache:
            return self.cache[token].split(" ")
        word = self._merge(tuple(token[:-1]) + (token[-1] + "</w>",))
        self.cache[token] = " ".join(word)
        return list(word)

    def encode(self, text: str) -> list[int]:
        added = self.added_tokens
        if added:  # textual-inversion placeholders map to their appended embedding rows
            for tok, tids in added.items():
                if tok in text:
                    parts = text.split(tok)
                    out: list[int] = []
                    for i, part in enumerate(parts):
                        out.extend(self.encode(part))
                        if i < len(parts) - 1:
                            out.extend(tids)
                    return out
        return self.encode_plain(text)

    def encode_plain(self, text: str) -> list[int]:
        if self.encoder is not None and getattr(self, "_special_re", None) is not None:
            ids: list[int] = []
            for part in self._special_re.split(text):
                if part in self._specials:
                    ids.append(self.encoder[part])
                elif part:
                    ids.extend(self._encode_segment(part))
            return ids
        return self._encode_segment(text)

    def _encode_segment(self, text: str) -> list[int]:
        text = _WS.sub(" ", unicodedata.normalize("NFC", text)).lower()
        ids: list[int] = []
        for tok in _PAT.findall(text):
            if self.encoder is not None:
                if tok in ("<|startoftext|>", "<|endoftext|>"):
                    ids.append(self.encoder[tok])
                    continue
                t = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
                ids.extend(self.encoder.get(p, self._unk_id) for p in self._bpe(t))
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
            ids = ids + [self.pad] * (self.max_length - len(ids))
            out.append(ids)
        return torch.tensor(out, dtype=torch.long)


class ByteBPETokenizer(CLIPTokenizer):
    """GPT-2 / RoBERTa byte-level BPE (``vocab.json`` + ``merges.txt``): the
    CLAP text tower of AudioLDM (RobertaTokenizer).  No lower-casing, no
    ``</w>`` suffix, spaces folded into the following token ("Ġ").  Hash
    fallback without vocabulary files, like ``CLIPTokenizer``."""

    def __init__(self, model_dir: str | None = None, max_length: int = 77, vocab_size: int = 50265,
                 bos: int = 0, eos: int = 2, pad: int = 1):
        super().__init__(None, max_length, pad_with_eos=False, vocab_size=vocab_size)
        if model_dir and os.path.exists(os.path.join(model_dir, "vocab.json")):
            self._load_bpe(model_dir, "")
            self._unk_id = self.encoder.get("<unk>", 3)
            self.source = model_dir
        self._bos, self._eos, self._pad_id = bos, eos, pad
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
        word = self._merge(tuple(token))
        self.cache[token] = " ".join(word)
        return list(word)

    def encode_plain(self, text: str) -> list[int]:
        ids: list[int] = []
        for tok in self._pat.findall(text):
            if self.encoder is not None:
                t = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
                ids.extend(self.encoder.get(p, self._unk_id) for p in self._bpe(t))
            else:
                h = int.from_bytes(hashlib.blake2b(tok.encode(), digest_size=8).digest(), "little")
                ids.append(h % (self.vocab_size - 4) + 4)
        return ids

    def decode(self, ids: list[int]) -> str:
        """Text of ``ids`` with bos / eos / pad dropped (``skip_special_tokens``)."""
        skip = {self._bos, self._eos, self._pad_id}
        ids = [i for i in ids if i not in skip]
        if self.encoder is None:
            return " ".join(f"w{i}" for i in ids)
        if not hasattr(self, "_decoder"):
            self._decoder = {v: k for k, v in self.encoder.items()}
            self._byte_decoder = {c: b for b, c in self.byte_encoder.items()}
        text = "".join(self._decoder.get(i, "") for i in ids)
        return bytes(self._byte_decoder[c] for c in text if c in self._byte_decoder).decode("utf-8", "replace")

    def __call__(self, texts: list[str] | str, pad: bool = False) -> list[list[int]]:  # type: ignore[override]
        """Unpadded id lists ([bos] ids [eos]); attention needs no padding mask."""
        if isinstance(texts, str):
            texts = [texts]
        out = []
        for t in texts:
            ids = [self.bos] + self.encode(t)[: self.max_length - 2] + [self.eos]
            if pad:
                ids = ids + [self._pad_id] * (self.max_length - len(ids))
            out.append(ids)
        return out
