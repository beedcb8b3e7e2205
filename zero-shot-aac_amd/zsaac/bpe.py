"""GPT-2 byte-level BPE (the tokenizer the reference loads with ``GPT2Tokenizer.from_pretrained``,
dataset/dataset.py:460, predict_prompt.py:185), from a local ``vocab.json`` + ``merges.txt``.

The reference only calls ``encode`` (the hard prompt, utils.py:174, and ``encode('.')``,
gpt2_prefix_eval.py:103,176) and ``decode`` (the generated ids, gpt2_prefix_eval.py:155,219,
and get_prefix_tokens, :275).  This restates the published GPT-2 algorithm (OpenAI
``encoder.py``, as wrapped by transformers' ``GPT2Tokenizer``):

* pre-tokenise with the GPT-2 pattern (contractions, `` ?\\p{L}+``, `` ?\\p{N}+``, `` ?[^\\s\\p{L}\\p{N}]+``,
  trailing / other whitespace);
* map each piece's UTF-8 bytes to printable unicode (``bytes_to_unicode``) and merge pairs in
  ``merges.txt`` rank order until no ranked pair remains;
* ids from ``vocab.json``; ``decode`` inverts the byte map.

``decode`` applies transformers' ``clean_up_tokenization_spaces`` by default, as the pinned
transformers 4.24 (retrieval/work.yaml) did for GPT-2 (" ." -> ".", " ," -> ",", " 's" -> "'s",
...): the reference's captions end with the stop id 764 (" .") and come out as "...word.".

No vocab files exist offline: the parity test builds a synthetic vocab/merges pair and compares
against transformers' own ``GPT2Tokenizer`` loaded from the same files.
"""
from __future__ import annotations

import json
import os
from functools import lru_cache
from typing import Dict, List, Sequence, Tuple

import regex

_PAT = regex.compile(r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""")


@lru_cache()
def bytes_to_unicode() -> Dict[int, str]:
    """GPT-2's reversible byte -> printable-unicode map (printable Latin-1 bytes map to
    themselves, the other 68 bytes to U+0100 onwards)."""
    bs = (list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1))
          + list(range(ord("®"), ord("ÿ") + 1)))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def clean_up_tokenization(text: str) -> str:
    """transformers' ``PreTrainedTokenizerBase.clean_up_tokenization``."""
    return (text.replace(" .", ".").replace(" ?", "?").replace(" !", "!").replace(" ,", ",")
            .replace(" ' ", "'").replace(" n't", "n't").replace(" 'm", "'m").replace(" 's", "'s")
            .replace(" 've", "'ve").replace(" 're", "'re"))


class GPT2BPE:
    """``encode(text) -> ids`` / ``decode(ids) -> str`` with GPT-2 byte-level BPE."""

    def __init__(self, vocab_file: str, merges_file: str, clean_up_tokenization_spaces: bool = True):
        with open(vocab_file, encoding="utf-8") as f:
            self.encoder: Dict[str, int] = json.load(f)
        self.decoder: Dict[int, str] = {v: k for k, v in self.encoder.items()}
        with open(merges_file, encoding="utf-8") as f:
            lines = f.read().split("\n")
        merges: List[Tuple[str, str]] = []
        for ln in lines:
            if not ln.strip() or ln.startswith("#version"):
                continue
            a, b = ln.split()
            merges.append((a, b))
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.byte_encoder = bytes_to_unicode()
        self.byte_decoder = {v: k for k, v in self.byte_encoder.items()}
        self.clean_up = clean_up_tokenization_spaces
        self._cache: Dict[str, List[str]] = {}

    @classmethod
    def from_dir(cls, path: str, **kw) -> "GPT2BPE":
        return cls(os.path.join(path, "vocab.json"), os.path.join(path, "merges.txt"), **kw)

    def _bpe(self, token: str) -> List[str]:
        hit = self._cache.get(token)
        if hit is not None:
            return hit
        word = list(token)
        while len(word) > 1:
            best, best_rank = None, None
            for i in range(len(word) - 1):
                r = self.bpe_ranks.get((word[i], word[i + 1]))
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = i, r
            if best is None:
                break
            a, b = word[best], word[best + 1]
            merged: List[str] = []
            i = 0
            while i < len(word):     # merge every occurrence of the best pair, left to right
                if i < len(word) - 1 and word[i] == a and word[i + 1] == b:
                    merged.append(a + b)
                    i += 2
                else:
                    merged.append(word[i])
                    i += 1
            word = merged
        self._cache[token] = word
        return word

    def tokenize(self, text: str) -> List[str]:
        out: List[str] = []
        for piece in _PAT.findall(text):
            out.extend(self._bpe("".join(self.byte_encoder[b] for b in piece.encode("utf-8"))))
        return out

    def encode(self, text: str) -> List[int]:
        return [self.encoder[t] for t in self.tokenize(text)]

    def decode(self, ids, clean_up_tokenization_spaces=None) -> str:
        if hasattr(ids, "tolist"):
            ids = ids.tolist()
        if isinstance(ids, int):
            ids = [ids]
        text = "".join(self.decoder.get(int(i), "") for i in ids)
        text = bytearray(self.byte_decoder[c] for c in text).decode("utf-8", errors="replace")
        clean = self.clean_up if clean_up_tokenization_spaces is None else clean_up_tokenization_spaces
        return clean_up_tokenization(text) if clean else text


def write_vocab(path: str, vocab: Dict[str, int], merges: Sequence[Tuple[str, str]]) -> None:
    """Writes a vocab.json / merges.txt pair (test fixtures, synthetic vocabularies)."""
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "vocab.json"), "w", encoding="utf-8") as f:
        json.dump(vocab, f, ensure_ascii=False)
    with open(os.path.join(path, "merges.txt"), "w", encoding="utf-8") as f:
        f.write("#version: 0.2\n" + "".join(f"{a} {b}\n" for a, b in merges))
