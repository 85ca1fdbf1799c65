"""Deterministic mock provider (config C1), mirroring ``src/neuralstego/lm/mock.py:36-59``.

Identity coder: packet bytes are the token ids.  It runs no GPU code and exists so that the drop-in
registry answers ``load_lm("mock")`` exactly like the reference.
"""

from __future__ import annotations

from typing import Dict, Iterable, List


class MockTokenizer:
    def encode(self, text: str) -> List[int]:
        return list(text.encode("utf-8"))

    def decode(self, tokens: Iterable[int]) -> str:
        return bytes(int(t) % 256 for t in tokens).decode("utf-8", errors="ignore")


def _bits_to_bytes(bits: Iterable[int]) -> bytes:
    data = list(bits)
    if len(data) % 8:
        raise ValueError("bit stream length must be a multiple of 8")
    out = bytearray()
    for i in range(0, len(data), 8):
        v = 0
        for off, bit in enumerate(data[i : i + 8]):
            v |= (int(bit) & 1) << off
        out.append(v)
    return bytes(out)


def _bytes_to_bits(data: bytes) -> List[int]:
    return [(byte >> i) & 1 for byte in data for i in range(8)]


class MockLM:
    def __init__(self) -> None:
        self.tokenizer = MockTokenizer()

    def encode_seed(self, text: str) -> List[int]:
        return self.tokenizer.encode(text)

    def encode_arithmetic(self, bits: List[int], context: List[int], *, quality: Dict[str, float]) -> List[int]:
        _ = context, quality
        return [int(b) for b in _bits_to_bytes(bits)] if bits else []

    def decode_arithmetic(self, tokens: List[int], context: List[int], *, quality: Dict[str, float]) -> List[int]:
        _ = context, quality
        return _bytes_to_bits(bytes(int(t) % 256 for t in tokens))


__all__ = ["MockLM", "MockTokenizer"]
