"""Deterministic toy tokenizer for the decode-repair fixtures (test infrastructure).

Vocabulary of V strings: the 26 letters, a space, "\\n" at id 198, "\\n\\n" at id 628, "<eos>" at id 650,
and seeded random 2-4 letter pieces elsewhere.  ``encode`` is greedy longest match (ties: lowest id), so
decode -> encode can re-split a cover text differently from the tokens the coder emitted -- exactly the
BPE ambiguity the reference's decode repair (code_base/arithmetic.py:300-342) handles.
"""

from __future__ import annotations

import numpy as np


class ToyTokenizer:
    def __init__(self, vocab: int = 700, seed: int = 3):
        rng = np.random.default_rng(seed)
        letters = "abcdefghijklmnopqrstuvwxyz"
        pieces = {}
        for i, ch in enumerate(letters):
            pieces[i] = ch
        pieces[26] = " "
        fixed = {198: "\n", 628: "\n\n", 650: "<eos>"}
        pieces.update(fixed)
        seen = set(pieces.values())
        for i in range(vocab):
            if i in pieces:
                continue
            while True:
                n = int(rng.integers(2, 5))
                s = "".join(letters[int(k)] for k in rng.integers(0, 8, n))  # small alphabet: many overlaps
                if s not in seen:
                    break
            pieces[i] = s
            seen.add(s)
        self.pieces = [pieces[i] for i in range(vocab)]
        self.lookup = {}
        for i, s in enumerate(self.pieces):
            self.lookup.setdefault(s, i)
        self.maxlen = max(len(s) for s in self.pieces)

    def encode(self, text: str, add_special_tokens: bool = False):
        _ = add_special_tokens
        out, i = [], 0
        while i < len(text):
            for L in range(min(self.maxlen, len(text) - i), 0, -1):
                t = self.lookup.get(text[i:i + L])
                if t is not None:
                    out.append(t)
                    i += L
                    break
            else:
                i += 1  # unknown character: dropped
        return out

    def decode(self, ids):
        return "".join(self.pieces[int(i)] for i in ids)
