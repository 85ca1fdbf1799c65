"""The codec slot ``encode_arithmetic`` / ``decode_arithmetic`` of ``src/neuralstego/codec/api.py:10-31``.

The reference leaves both unimplemented ("will be implemented in a later phase"); here they run the true
arithmetic coder through any provider that speaks the api ``LMProvider`` protocol (``api.py:42-56``),
normally :class:`~neuralsteganography_amd.lm.arithmetic.HipArithmeticLM`.  Payload bytes become bits
LSB-first per byte, the api convention (``api.py:153-157``).
"""

from __future__ import annotations

from typing import Sequence

from ..exceptions import ConfigurationError


def _bytes_to_bits(data: bytes):
    return [(byte >> i) & 1 for byte in data for i in range(8)]


def _bits_to_bytes(bits) -> bytes:
    bits = list(bits)
    if len(bits) % 8:
        raise ConfigurationError("decoded bit stream is not byte aligned")
    out = bytearray()
    for i in range(0, len(bits), 8):
        v = 0
        for off, bit in enumerate(bits[i : i + 8]):
            v |= (int(bit) & 1) << off
        out.append(v)
    return bytes(out)


def encode_arithmetic(bits: bytes, lm, *, quality: dict, seed_text: str = "") -> list[int]:
    """Encode a payload into token ids (codec/api.py:10-19)."""
    payload = bytes(bits)
    if not payload:
        return []
    context = lm.encode_seed(seed_text)
    return [int(t) for t in lm.encode_arithmetic(_bytes_to_bits(payload), context, quality=dict(quality or {}))]


def decode_arithmetic(token_ids: Sequence[int], lm, *, quality: dict, seed_text: str = "") -> bytes:
    """Decode token ids back into the payload (codec/api.py:22-31)."""
    tokens = [int(t) for t in token_ids]
    if not tokens:
        return b""
    context = lm.encode_seed(seed_text)
    bits = lm.decode_arithmetic(tokens, context, quality=dict(quality or {}))
    return _bits_to_bytes(bits)


__all__ = ["encode_arithmetic", "decode_arithmetic"]
