"""``encode_with_lm`` / ``decode_with_lm`` (``src/neuralstego/codec/arithmetic.py:122-231``) on the HIP rank kernel.

Same signatures, state dict (``history`` = bits consumed per token, ``residual_bits`` = 8-byte big-endian
payload bit count) and errors as the reference.  ``lm`` is either

* a :class:`~neuralsteganography_amd.lm.rank.HipRankLM` (the provider owns the batched GPT-2; the
  ``_ModelAdapter`` softmax of ``lm/arithmetic.py:45-74`` is computed inside the kernel, temperature from the
  quality), or
* ANY ``next_token_probs`` provider (the L2 protocol of ``codec/types.py:41-45``: the Zipf ``MockLM`` of
  ``codec/distribution.py:17-37``, ``CachedLM``, a user model): its ProbDists (float64 arrays or ``{id: p}``
  dicts) are queried on the host per step, staged to the device AS float64 values
  (:class:`~neuralsteganography_amd.codec.distribution.ProbRows`, ``NS_DTYPE_F64``) and ranked, filtered and
  renormalised by the rank kernel's provider-row form exactly as the reference's numpy does.  As in the reference,
  only the ``top_k`` / ``top_p`` / ``min_prob`` / ``cap_per_token_bits`` keys of ``quality`` act (``_apply_quality``,
  ``:350-363``) and the context is trimmed to ``max_context`` or the provider's ``context_window``
  (``_resolve_context_window``, ``:328-334``).

For a ``HipRankLM``, ``max_context`` (or the quality key of the same name) re-runs every stream's trimmed window
per token, as the reference's ``_ModelAdapter`` does (``lm/arithmetic.py:45-74``; :class:`~neuralsteganography_amd.lm.
rank.WindowedLM`).
"""

from __future__ import annotations

from typing import Mapping, MutableMapping, Optional, Sequence

from .errors import DecodeDivergenceError

# what reaches the coder for a generic provider (_apply_quality, codec/arithmetic.py:351-367), plus this build's
# crypto policy key (crypto/arithmetic.py's _QualityControlledLM, applied by the rank kernel)
_CODEC_QUALITY_KEYS = ("top_k", "top_p", "min_prob", "cap_per_token_bits", "prob_temp")


def _resolve_context_window(lm, override: Optional[int]) -> Optional[int]:
    """``codec/arithmetic.py:328-334``."""
    if override is not None and override > 0:
        return override
    window = getattr(lm, "context_window", None)
    if isinstance(window, int) and window > 0:
        return window
    return None


def _rank_provider(lm, context, max_context):
    """(rank-coder provider, quality filter) for ``lm``: a HipRankLM as is, else a HipRankLM over the
    provider's staged distributions."""
    if hasattr(lm, "encode_batch_states") and hasattr(lm, "decode_batch"):
        return lm, None
    if not hasattr(lm, "next_token_probs"):
        raise TypeError("lm must be a HipRankLM or provide next_token_probs(context_ids)")
    from ..lm.rank import HipRankLM
    from .distribution import ProviderBatchedLM

    batched = ProviderBatchedLM(lm, list(context or []), context_window=_resolve_context_window(lm, max_context))
    return HipRankLM(batched_lm=batched, max_batch=1), _CODEC_QUALITY_KEYS


def _codec_quality(quality, keys, max_context=None):
    q = dict(quality or {})
    if keys is None:  # HipRankLM: the provider reads every key; an explicit max_context trims its window
        if max_context is not None and max_context > 0:
            q["max_context"] = int(max_context)
        return q
    return {k: q[k] for k in keys if q.get(k) is not None}  # temperature etc. belong to the provider


def encode_with_lm(bits: bytes, lm, *, context: Sequence[int] | None = None, quality: Mapping[str, object] | None = None,
                   state: MutableMapping[str, object] | None = None, max_context: int | None = None) -> list:
    bit_list = [(b >> k) & 1 for b in bytes(bits) for k in range(8)]
    if not bit_list:
        if state is not None:
            state["history"] = tuple()
            state["residual_bits"] = (0).to_bytes(8, byteorder="big", signed=False)
        return []
    prov, keys = _rank_provider(lm, context, max_context)
    toks, states = prov.encode_batch_states([bit_list], list(context or []),
                                            quality=_codec_quality(quality, keys, max_context))
    if state is not None:
        state["history"] = tuple(states[0]["history"])
        state["residual_bits"] = states[0]["residual_bits"]
    return toks[0]


def decode_with_lm(tokens: Sequence[int], lm, *, context: Sequence[int] | None = None,
                   quality: Mapping[str, object] | None = None, state: MutableMapping[str, object] | None = None,
                   max_context: int | None = None) -> bytes:
    if not tokens:
        return b""
    history = state.get("history") if state is not None else None
    if history is None or len(history) < len(tokens):
        raise DecodeDivergenceError("Bit consumption history is required for decoding")
    st = {"history": tuple(history[: len(tokens)])}
    total_bits = None
    if state is not None and state.get("residual_bits"):
        st["residual_bits"] = state["residual_bits"]
        total_bits = int.from_bytes(bytes(state["residual_bits"]), byteorder="big", signed=False)
    prov, keys = _rank_provider(lm, context, max_context)
    bits = prov.decode_batch([list(tokens)], list(context or []), quality=_codec_quality(quality, keys, max_context),
                             states=[st])[0]
    if total_bits is not None and total_bits > sum(st["history"]):
        raise DecodeDivergenceError("Decoded bitstream shorter than expected")  # codec/arithmetic.py:222-223
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
