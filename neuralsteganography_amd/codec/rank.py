"""``encode_with_lm`` / ``decode_with_lm`` (``src/neuralstego/codec/arithmetic.py:122-231``) on the HIP rank kernel.

Same signatures, state dict (``history`` = bits consumed per token, ``residual_bits`` = 8-byte big-endian
payload bit count) and errors as the reference; ``lm`` is a :class:`~neuralsteganography_amd.lm.rank.HipRankLM`
(the reference passes a ``next_token_probs`` provider; here the provider owns the batched GPT-2 and the
probabilities are computed on the GPU inside the kernel).  ``max_context`` is accepted for signature
compatibility (see ``HipRankLM`` for the KV-cache note).
"""

from __future__ import annotations

from typing import Mapping, MutableMapping, Sequence

from .errors import DecodeDivergenceError


def encode_with_lm(bits: bytes, lm, *, context: Sequence[int] | None = None, quality: Mapping[str, object] | None = None,
                   state: MutableMapping[str, object] | None = None, max_context: int | None = None) -> list:
    _ = max_context
    bit_list = [(b >> k) & 1 for b in bytes(bits) for k in range(8)]
    if not bit_list:
        if state is not None:
            state["history"] = tuple()
            state["residual_bits"] = (0).to_bytes(8, byteorder="big", signed=False)
        return []
    tokens = lm.encode_batch([bit_list], list(context or []), quality=dict(quality or {}))[0]
    st = lm.drain_states()[-1]
    lm._decode_states.pop()  # the queued copy belongs to this call, not to a later decode_arithmetic
    if state is not None:
        state["history"] = tuple(st["history"])
        state["residual_bits"] = st["residual_bits"]
    return tokens


def decode_with_lm(tokens: Sequence[int], lm, *, context: Sequence[int] | None = None,
                   quality: Mapping[str, object] | None = None, state: MutableMapping[str, object] | None = None,
                   max_context: int | None = None) -> bytes:
    _ = max_context
    if not tokens:
        return b""
    history = state.get("history") if state is not None else None
    if history is None or len(history) < len(tokens):
        raise DecodeDivergenceError("Bit consumption history is required for decoding")
    st = {"history": tuple(history[: len(tokens)])}
    if state is not None and state.get("residual_bits"):
        st["residual_bits"] = state["residual_bits"]
    bits = lm.decode_batch([list(tokens)], list(context or []), quality=dict(quality or {}), states=[st])[0]
    if state is not None:
        rest = list(history[len(tokens):])
        if rest:
            state["history"] = tuple(rest)
        else:
            state.pop("history", None)
    out = bytearray(len(bits) // 8)
    for i in range(len(out)):
        out[i] = sum(bits[8 * i + k] << k for k in range(8))
    return bytes(out)


__all__ = ["encode_with_lm", "decode_with_lm"]
