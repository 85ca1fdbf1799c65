"""C1 provider: the identity coder behind ``load_lm("mock")`` (behaviour of ``src/neuralstego/lm/mock.py``).

Cover tokens ARE the packet bytes: ``encode_arithmetic`` packs the LSB-first bit list into bytes and returns
their values; ``decode_arithmetic`` unpacks token values (mod 256) back into bits.  Pure host code (no model,
no GPU); it exists so framing and api tests run anywhere, as in the reference.
"""

from __future__ import annotations

from typing import Dict, Iterable, List

import numpy as np


class MockTokenizer:
    """UTF-8 bytes as token ids."""

    def encode(self, text: str) -> List[int]:
        return [int(v) for v in text.encode("utf-8")]

    def decode(self, tokens: Iterable[int]) -> str:
        raw = np.asarray(list(tokens), dtype=np.int64) % 256
        return raw.astype(np.uint8).tobytes().decode("utf-8", errors="ignore")


class MockLM:
    """Identity packet-bytes <-> tokens provider (api ``LMProvider`` protocol)."""

    def __init__(self) -> None:
        self.tokenizer = MockTokenizer()

    def encode_seed(self, text: str) -> List[int]:
        return self.tokenizer.encode(text)

    def encode_arithmetic(self, bits: List[int], context: List[int], *, quality: Dict[str, float]) -> List[int]:
        del context, quality
        if len(bits) % 8:
            raise ValueError("bit stream length must be a multiple of 8")
        if not bits:
            return []
        packed = np.packbits(np.asarray(bits, dtype=np.uint8) & 1, bitorder="little")
        return packed.astype(np.int64).tolist()

    def decode_arithmetic(self, tokens: List[int], context: List[int], *, quality: Dict[str, float]) -> List[int]:
        del context, quality
        raw = (np.asarray(list(tokens), dtype=np.int64) % 256).astype(np.uint8)
        return np.unpackbits(raw, bitorder="little").astype(np.int64).tolist()


__all__ = ["MockLM", "MockTokenizer"]
