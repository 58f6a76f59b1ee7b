"""Offline tokenizers for the random-init diagnostic models.

No tokenizer files can be fetched (no network), so the framework ships its own byte-level BPE:

* ids ``0..255`` are raw bytes, ``256..256+len(merges)-1`` are learned merges;
* the model's special ids (``bos``/``eos`` from the preset) are honoured as-is;
* ``decode`` maps any id the vocabulary does not cover (a random-init model samples from the whole
  128k vocab) onto the covered range, so answers always decode to text.

Merges are learned from synthetic cluster-state text (``train_bpe``); the hot encode path runs
in the C++ runtime (``_k8sllm_runtime.BPE``) when it is built, else in Python with a word cache.
"""
from __future__ import annotations

import json
import re
from collections import Counter
from pathlib import Path
from typing import Iterable, Optional

_PRE = re.compile(r"""'s|'t|'re|'ve|'m|'ll|'d| ?[A-Za-z]+| ?[0-9]{1,3}| ?[^\sA-Za-z0-9]+|\s+(?!\S)|\s+""")

DEFAULT_MERGES = Path(__file__).resolve().parent / "data" / "bpe_merges.json"


class ByteBPETokenizer:
    def __init__(self, merges: Optional[list[tuple[int, int]]] = None, bos_id: int = 1, eos_id: int = 2,
                 vocab_size: int = 0):
        self.merges = list(merges or [])
        self.ranks = {tuple(p): i for i, p in enumerate(self.merges)}
        self.bos_id = bos_id
        self.eos_id = eos_id
        self.n_base = 256 + len(self.merges)
        self.vocab_size = max(vocab_size, self.n_base)
        self._bytes: list[bytes] = [bytes([i]) for i in range(256)]
        for a, b in self.merges:
            self._bytes.append(self._bytes[a] + self._bytes[b])
        self._cache: dict[str, list[int]] = {}
        self._dec_tables: dict[bool, list[bytes]] = {}
        self._native = None
        try:
            from ..runtime import native_runtime

            rt = native_runtime()
            if rt is not None and self.merges:
                self._native = rt.BPE([a for a, _ in self.merges], [b for _, b in self.merges])
        except Exception:  # noqa: BLE001
            self._native = None

    # --------------------------------------------------------------- encode / decode
    def _bpe_word(self, w: bytes) -> list[int]:
        ids = list(w)
        ranks = self.ranks
        while len(ids) > 1:
            best, bi = None, -1
            for i in range(len(ids) - 1):
                r = ranks.get((ids[i], ids[i + 1]))
                if r is not None and (best is None or r < best):
                    best, bi = r, i
            if best is None:
                break
            ids[bi:bi + 2] = [256 + best]
        return ids

    def encode(self, text: str, bos: bool = True) -> list[int]:
        if self._native is not None:
            out = self._native.encode(text.encode("utf-8"))
            return ([self.bos_id] if bos else []) + list(out)
        out = [self.bos_id] if bos else []
        cache = self._cache
        for m in _PRE.finditer(text):
            w = m.group(0)
            ids = cache.get(w)
            if ids is None:
                ids = self._bpe_word(w.encode("utf-8"))
                if len(cache) < 200_000:
                    cache[w] = ids
            out.extend(ids)
        return out

    def _token_bytes(self, t: int, skip_special: bool) -> bytes:
        if t < 0 or (skip_special and t in (self.bos_id, self.eos_id)):
            return b""
        nb = self.n_base
        if t < nb:
            return self._bytes[t]
        if nb > 256:  # uncovered id from a random-init model: fold onto the merge range
            return self._bytes[256 + (t - nb) % (nb - 256)]
        return self._bytes[t % 256]

    def decode(self, ids: Iterable[int], skip_special: bool = True) -> str:
        # one bytes object per vocabulary id, built on first use: a whole answer is then one
        # list lookup per token and one join (an engine step's finished answers are decoded on the
        # engine thread)
        tbl = self._dec_tables.get(skip_special)
        if tbl is None:
            tbl = [self._token_bytes(t, skip_special) for t in range(self.vocab_size)]
            self._dec_tables[skip_special] = tbl
        n = len(tbl)
        buf = b"".join([tbl[t] if 0 <= t < n else self._token_bytes(t, skip_special) for t in ids])
        return buf.decode("utf-8", errors="replace")

    # --------------------------------------------------------------- persistence
    def save(self, path: Path) -> None:
        path.parent.mkdir(parents=True, exist_ok=True)
        path.write_text(json.dumps({"merges": self.merges}))

    @classmethod
    def load(cls, path: Path = DEFAULT_MERGES, **kw) -> "ByteBPETokenizer":
        merges = []
        if Path(path).exists():
            merges = [tuple(p) for p in json.loads(Path(path).read_text())["merges"]]
        return cls(merges, **kw)


def train_bpe(texts: Iterable[str], num_merges: int = 4000, min_freq: int = 2) -> list[tuple[int, int]]:
    """Classic word-level BPE training with incremental pair counts."""
    words = Counter()
    for t in texts:
        for m in _PRE.finditer(t):
            words[m.group(0).encode("utf-8")] += 1
    seqs = [list(w) for w in words]
    freqs = [words[w] for w in words]
    pairs: Counter = Counter()
    where: dict[tuple[int, int], set[int]] = {}
    for wi, s in enumerate(seqs):
        f = freqs[wi]
        for i in range(len(s) - 1):
            p = (s[i], s[i + 1])
            pairs[p] += f
            where.setdefault(p, set()).add(wi)
    merges: list[tuple[int, int]] = []
    for _ in range(num_merges):
        if not pairs:
            break
        best, cnt = max(pairs.items(), key=lambda kv: (kv[1], -kv[0][0], -kv[0][1]))
        if cnt < min_freq:
            break
        new_id = 256 + len(merges)
        merges.append(best)
        for wi in list(where.get(best, ())):
            s, f = seqs[wi], freqs[wi]
            for i in range(len(s) - 1):  # remove old pair counts of this word
                p = (s[i], s[i + 1])
                pairs[p] -= f
                if pairs[p] <= 0:
                    del pairs[p]
            i, out = 0, []
            while i < len(s):
                if i < len(s) - 1 and s[i] == best[0] and s[i + 1] == best[1]:
                    out.append(new_id)
                    i += 2
                else:
                    out.append(s[i])
                    i += 1
            seqs[wi] = out
            for i in range(len(out) - 1):
                p = (out[i], out[i + 1])
                pairs[p] += f
                where.setdefault(p, set()).add(wi)
        where.pop(best, None)
    return merges


def tokenizer_for(model_cfg, merges_path: Path = DEFAULT_MERGES) -> ByteBPETokenizer:
    """Tokenizer whose ids all fit the model's vocabulary (merges truncated for tiny vocabs)."""
    merges = []
    if Path(merges_path).exists():
        merges = [tuple(p) for p in json.loads(Path(merges_path).read_text())["merges"]]
    specials_hi = max(model_cfg.bos_id, *model_cfg.eos_ids)
    room = model_cfg.vocab_size - 256
    if specials_hi >= 256 and specials_hi < model_cfg.vocab_size:
        room = min(room, specials_hi - 256)  # keep merges below the special ids (Llama-3: 128000)
    merges = merges[:max(0, room)]
    return ByteBPETokenizer(merges, bos_id=model_cfg.bos_id, eos_id=model_cfg.eos_ids[0],
                            vocab_size=model_cfg.vocab_size)


class HFTokenizer:
    """A Hugging Face ``tokenizer.json`` (the ``tokenizers`` library, Rust BPE) behind the same
    encode / decode interface, for engines loading real checkpoints (EngineConfig.weights)."""

    def __init__(self, path: Path, bos_id: Optional[int], eos_id: Optional[int]):
        from tokenizers import Tokenizer

        self.tok = Tokenizer.from_file(str(path))
        self.bos_id, self.eos_id = bos_id, eos_id
        self.vocab_size = self.tok.get_vocab_size()

    def encode(self, text: str, bos: bool = True) -> list[int]:
        ids = self.tok.encode(text, add_special_tokens=False).ids
        return ([self.bos_id] if bos and self.bos_id is not None else []) + ids

    def decode(self, ids: Iterable[int], skip_special: bool = True) -> str:
        return self.tok.decode([int(t) for t in ids if t >= 0], skip_special_tokens=skip_special)


def tokenizer_from_dir(path, model_cfg):
    """``path/tokenizer.json`` as an :class:`HFTokenizer` when present, else the built-in BPE."""
    f = Path(path) / "tokenizer.json"
    if f.exists():
        return HFTokenizer(f, model_cfg.bos_id, model_cfg.eos_ids[0])
    return tokenizer_for(model_cfg)
