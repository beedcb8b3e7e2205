"""Host-side tokenisation for the hard prompt (no GPT-2 vocab files exist offline).

The reference builds the hard prompt string ``"There are l1, l2, l3 in this audio."``
(utils.py:158-176) and BPE-encodes it with ``GPT2Tokenizer`` (utils.py:174).  GPT-2's
pre-tokenizer splits on the regex below before BPE, and every piece boundary of the prompt is a
space or punctuation, so the prompt's ids are the concatenation of the ids of its pieces:
``enc("There") + enc(" are") + enc(" l1") + enc(",") + ... + enc(" in") + enc(" this") +
enc(" audio") + enc(".")``.  :class:`TableTokenizer` holds exactly that piece->ids table, so a
deployment fills it once from the real tokenizer (``{p: tok.encode(p)}`` for the template pieces
and ``' ' + label.lower()`` for the 527 AudioSet labels) and the device can assemble prompts from
a [labels, max_ids] table (zs_prompt_assemble).

Only ``encode`` and ``decode`` are used by the decoding API (gpt2_prefix_eval.py:103,155,176,219),
so this duck-types the part of ``GPT2Tokenizer`` the hot path touches.
"""
from __future__ import annotations

import re
from typing import Dict, Iterable, List, Sequence

# GPT-2's pre-tokenisation pattern (the \p{L}/\p{N} classes approximated with str classes)
_PAT = re.compile(r"""'s|'t|'re|'ve|'m|'ll|'d| ?[A-Za-z]+| ?[0-9]+| ?[^\sA-Za-z0-9]+|\s+(?!\S)|\s+""")

# GPT-2 BPE ids of the template pieces (each is a single BPE token in the GPT-2 vocab)
TEMPLATE_IDS: Dict[str, List[int]] = {
    "There": [1858],
    " are": [389],
    " something": [1223],
    " in": [287],
    " this": [428],
    " audio": [6597],
    ".": [13],
    ",": [11],
}
PROMPT_HEAD = ["There", " are"]
PROMPT_TAIL = [" in", " this", " audio", "."]
STOP_DOT = 13        # '.'
STOP_SPACE_DOT = 764  # ' .'  (generate2's second stop id, gpt2_prefix_eval.py:214)


def synthetic_label_names(n: int = 527) -> List[str]:
    """Single-word (alphabetic, so one pre-tokenizer piece) stand-ins for the 527 AudioSet label
    strings of audioset_label.pkl: 'sndaa', 'sndab', ..."""
    def letters(i):
        return chr(97 + i // 26 // 26 % 26) + chr(97 + i // 26 % 26) + chr(97 + i % 26)
    return ["snd" + letters(i) for i in range(n)]


class TableTokenizer:
    """Piece-table tokenizer: ``encode`` = regex split + per-piece id lookup; ``decode`` = ids
    rendered through the reverse table (unknown ids as ``<id>``)."""

    def __init__(self, pieces: Dict[str, Sequence[int]]):
        self.pieces = {k: list(v) for k, v in pieces.items()}
        self.rev: Dict[int, str] = {}
        for p, ids in self.pieces.items():
            if len(ids) == 1:
                self.rev.setdefault(int(ids[0]), p)

    @classmethod
    def for_labels(cls, label_names: Sequence[str], label_ids: Sequence[Sequence[int]]):
        pieces = dict(TEMPLATE_IDS)
        for name, ids in zip(label_names, label_ids):
            pieces[" " + name.lower()] = list(ids)
        return cls(pieces)

    def encode(self, text: str) -> List[int]:
        out: List[int] = []
        for piece in _PAT.findall(text):
            if piece not in self.pieces:
                raise KeyError(f"piece {piece!r} not in the tokenizer table")
            out.extend(self.pieces[piece])
        return out

    def decode(self, ids) -> str:
        if hasattr(ids, "tolist"):
            ids = ids.tolist()
        if isinstance(ids, int):
            ids = [ids]
        return "".join(self.rev.get(int(i), f"<{int(i)}>") for i in ids)


class IdTokenizer:
    """Tokenizer used when only ids matter: ``decode`` renders ids as a space-separated string
    (round-trippable by :func:`parse_ids`), ``encode('.')`` is [13] as in GPT-2."""

    def encode(self, text: str) -> List[int]:
        if text in TEMPLATE_IDS:
            return list(TEMPLATE_IDS[text])
        raise KeyError(text)

    def decode(self, ids) -> str:
        if hasattr(ids, "tolist"):
            ids = ids.tolist()
        if isinstance(ids, int):
            ids = [ids]
        return " ".join(str(int(i)) for i in ids)


def parse_ids(text: str) -> List[int]:
    return [int(t) for t in text.split()] if text.strip() else []


def compose_prompt_text(labels: Iterable[str]) -> str:
    """utils.py:158-176 ``compose_discrete_prompts`` string construction (mask_probability 0)."""
    labels = list(labels)
    if not labels:
        return "There are something in this audio."
    s = ""
    for e in labels:
        s += " " + e + ","
    return "There are" + s[:-1] + " in this audio."


class WordTokenizer:
    """A GPT-2-like decode for the CLAP-guided ("magic") decoding tests, where generated ids are
    turned into TEXT and re-tokenised by the BERT text encoder (gpt2_prefix_eval.py:440-445,
    582-586): ``decode`` concatenates one piece per id -- ' w<id>' starts a new word, 'q<id>'
    (ids divisible by 5) continues the previous one, and the stop ids render as GPT-2 renders
    them ('.' = 13, ' .' = 764, ',' = 11).  Every id has its own piece, so :meth:`parse` inverts
    ``decode``.  ``encode('.')`` is [13] as in GPT-2."""

    _RE = re.compile(r" w\d+|q\d+| \.|\.|,")
    concat_decode = True    # decode(ids) == "".join(decode([i]) for i in ids)

    @staticmethod
    def piece(i: int) -> str:
        i = int(i)
        if i == 13:
            return "."
        if i == 764:
            return " ."
        if i == 11:
            return ","
        return f"q{i}" if i % 5 == 0 else f" w{i}"

    def encode(self, text: str) -> List[int]:
        if text in TEMPLATE_IDS:
            return list(TEMPLATE_IDS[text])
        raise KeyError(text)

    def decode(self, ids) -> str:
        if hasattr(ids, "tolist"):
            ids = ids.tolist()
        if isinstance(ids, int):
            ids = [ids]
        return "".join(self.piece(i) for i in ids)

    @classmethod
    def parse(cls, text: str) -> List[int]:
        out = []
        for m in cls._RE.findall(text):
            out.append({".": 13, " .": 764, ",": 11}.get(m) or int(m.lstrip(" wq")))
        return out
