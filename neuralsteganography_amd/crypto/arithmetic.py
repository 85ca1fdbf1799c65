"""The crypto package's quality-controlled rank coder (``src/neuralstego/crypto/arithmetic.py:20-123`` with
``crypto/quality.py:15-89``) on the HIP rank kernel.

Reference behaviour restated:

* ``_QualityControlledLM`` (``crypto/arithmetic.py:20-40``) wraps a ``next_token_probs`` provider and applies
  ``crypto.quality.apply_quality``: the temperature acts on the PROBABILITIES
  (``log(p + 1e-12) / T``, shifted by the max, exponentiated and renormalised, ``quality.py:57-64``; skipped
  when ``math.isclose(T, 1.0)``), then ``top_k`` and ``top_p`` (cumsum + searchsorted ``'left'``) filter that
  tempered distribution.  With ``T != 1`` every id keeps nonzero mass (the ``1e-12`` floor), so the rank
  coder's capacity becomes ``floor(log2 V)`` unless a filter is set.
* ``encode_arithmetic(payload, lm, *, quality, seed_text, state) -> (tokens, state)`` runs ``encode_with_lm``
  through that wrapper with no codec quality of its own (``:43-63``); ``decode_arithmetic`` needs the state
  (``ValueError`` otherwise, ``:76-77``) and starts from ``{"history": (), "residual_bits": b""}`` updated
  by it (``:82-83``).
* ``_extract_quality`` (``:94-117``) reads ``top_k``, ``top_p``, ``temperature`` (defaults None, None, 1.0).

Here the whole policy runs inside the rank kernel (``ns_rank_quality.prob_temp``, canonical step R1c of
``oracle/nsg_oracle.c``): ``lm`` is a :class:`~neuralsteganography_amd.lm.rank.HipRankLM` (batched GPT-2 +
HIP rank coder).  The rank order is the canonical (probability desc, id asc) order of the untempered logits
-- the tempering is monotone -- and the support/top_p decisions use libm-equivalent ``log``/``exp`` on the
device (tolerance-level, like the reference's numpy).
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Mapping, MutableMapping, Optional, Sequence, Tuple

from ..codec.errors import QualityConfigError


def _extract_quality(quality: Optional[Mapping[str, object]]) -> dict:
    """``crypto/arithmetic.py:94-117``."""
    if not quality:
        return {"top_k": None, "top_p": None, "temperature": 1.0}
    top_k = quality.get("top_k") if "top_k" in quality else None
    top_p = quality.get("top_p") if "top_p" in quality else None
    return {"top_k": int(top_k) if top_k is not None else None,
            "top_p": float(top_p) if top_p is not None else None,
            "temperature": float(quality["temperature"]) if "temperature" in quality else 1.0}


def _validate(top_k, top_p, temperature) -> None:
    """The domain checks of ``crypto/quality.py:52-53,67-69,75-76`` (``QualityConfigError``)."""
    if temperature <= 0.0:
        raise QualityConfigError("temperature must be positive")
    if top_k is not None and top_k <= 0:
        raise QualityConfigError("top_k must be positive")
    if top_p is not None and not 0.0 < top_p <= 1.0:
        raise QualityConfigError("top_p must lie within (0, 1]")


def _rank_quality(top_k, top_p, temperature) -> dict:
    """The policy as the rank kernel's quality keys.  ``prob_temp`` = 1.0 is the isclose no-op of the tempering
    (the row is still normalised and filtered, quality.py:54-89); no keys at all when ``_QualityControlledLM``
    returns the base distribution unchanged (top_k and top_p None and temperature exactly 1.0, :31-32)."""
    _validate(top_k, top_p, temperature)
    if top_k is None and top_p is None and temperature == 1.0:
        return {}
    q = {"prob_temp": 1.0 if math.isclose(temperature, 1.0) else float(temperature)}
    if top_k is not None:
        q["top_k"] = int(top_k)
    if top_p is not None:
        q["top_p"] = float(top_p)
    return q


@dataclass
class QualityControlledLM:
    """``_QualityControlledLM`` (``crypto/arithmetic.py:20-40``) over a GPU ``next_token_probs`` provider
    (:class:`~neuralsteganography_amd.codec.distribution.HipTransformersLM` without filters of its own): the
    tempered, filtered, renormalised distribution is computed by the HIP kernel (``ns_token_probs``)."""

    base: object
    top_k: Optional[int] = None
    top_p: Optional[float] = None
    temperature: float = 1.0

    def next_token_probs(self, context_ids: Sequence[int]):
        if self.top_k is None and self.top_p is None and self.temperature == 1.0:
            return self.base.next_token_probs(context_ids)
        from ..coder import rank_quality

        if not hasattr(self.base, "_probs_with"):
            raise TypeError("QualityControlledLM needs a HIP next_token_probs provider (HipTransformersLM)")
        if any(f is not None for f in getattr(self.base, "_filters", ())):
            raise QualityConfigError("the base provider's own top_k/top_p/min_prob cannot be chained with the "
                                     "crypto quality policy on the GPU path")
        q = rank_quality(_rank_quality(self.top_k, self.top_p, self.temperature))
        return self.base._probs_with(context_ids, q)


def encode_arithmetic(payload: bytes, lm, *, quality: Optional[Mapping[str, object]] = None,
                      seed_text: Optional[Sequence[int]] = None,
                      state: Optional[MutableMapping[str, object]] = None) -> Tuple[List[int], dict]:
    """Encode ``payload`` (bytes) with the rank coder under the crypto quality policy."""
    from ..codec.rank import encode_with_lm

    pol = _extract_quality(quality)
    encode_state: dict = {}
    tokens = encode_with_lm(bytes(payload), lm, context=tuple(seed_text or ()),
                            quality=_rank_quality(pol["top_k"], pol["top_p"], pol["temperature"]),
                            state=encode_state)
    if state is not None:
        state.update(encode_state)
    return tokens, encode_state


def decode_arithmetic(token_ids: Sequence[int], lm, *, quality: Optional[Mapping[str, object]] = None,
                      seed_text: Optional[Sequence[int]] = None,
                      state: Optional[MutableMapping[str, object]] = None) -> bytes:
    """Decode ``token_ids`` back into the payload bytes (needs the encode state's consumption history)."""
    from ..codec.rank import decode_with_lm

    if state is None:
        raise ValueError("state with bit consumption history is required for decoding")
    pol = _extract_quality(quality)
    decode_state: dict = {"history": tuple(), "residual_bits": b""}
    decode_state.update(state)
    return decode_with_lm(list(token_ids), lm, context=tuple(seed_text or ()),
                          quality=_rank_quality(pol["top_k"], pol["top_p"], pol["temperature"]),
                          state=decode_state)


__all__ = ["QualityControlledLM", "encode_arithmetic", "decode_arithmetic"]
