"""Token spans <-> cover text (``src/neuralstego/codec/textio.py``).

``seed_to_ids`` and ``spans_to_text`` behave as the reference's (tokenizer ``encode`` without special tokens,
falling back as it does; ``decode`` of seed + spans with ``skip_special_tokens``, stripped).  ``text_to_spans``
is a placeholder in the reference (``:58-63``, ``NotImplementedError``, so ``cover_reveal`` falls back to a
JSON spans payload); here it raises the same way unless a span splitter is supplied (see
:func:`neuralsteganography_amd.cover.cover_reveal`).
"""

from __future__ import annotations

from typing import List, Optional, Sequence


def _need(tok):
    if tok is None:
        raise ValueError("tokenizer instance is required")
    return tok


def seed_to_ids(seed: str, tok) -> List[int]:
    """``textio.py:13-34``."""
    t = _need(tok)
    if hasattr(t, "encode"):
        try:
            ids = t.encode(seed, add_special_tokens=False)
        except TypeError:
            ids = t.encode(seed)
        else:
            if not ids:
                ids = t.encode(seed)
        return [int(i) for i in ids]
    if hasattr(t, "tokenize") and hasattr(t, "convert_tokens_to_ids"):
        return [int(i) for i in t.convert_tokens_to_ids(t.tokenize(seed))]
    raise TypeError("tokenizer does not provide an encode method")


def spans_to_text(spans: Sequence[Sequence[int]], seed_ids: Sequence[int], tok) -> str:
    """``textio.py:37-55``: seed ids followed by every span, decoded and stripped."""
    t = _need(tok)
    ids: List[int] = [int(i) for i in seed_ids]
    for span in spans:
        ids.extend(int(i) for i in span)
    if hasattr(t, "decode"):
        try:
            return t.decode(ids, skip_special_tokens=True).strip()
        except TypeError:
            return t.decode(ids).strip()
    if hasattr(t, "convert_ids_to_tokens") and hasattr(t, "convert_tokens_to_string"):
        return t.convert_tokens_to_string(t.convert_ids_to_tokens(ids)).strip()
    raise TypeError("tokenizer does not provide a decode method")


def text_to_spans(text: str, seed_ids: Sequence[int], tok, *, lm=None, quality=None,
                  seed_text: Optional[str] = None) -> List[List[int]]:
    """``textio.py:58-63`` -- a ``NotImplementedError`` placeholder in the reference (span boundaries are not
    in the text).  Given the provider (``lm``), the quality the cover was made with and its ``seed_text``, the
    spans are recovered by decoding (:func:`neuralsteganography_amd.cover.texts_to_spans`).  Without ``lm``
    the reference's behaviour is kept (``cover_reveal`` then reads a JSON spans payload)."""
    if lm is None:
        raise NotImplementedError("text_to_spans is not yet implemented; provide spans JSON payloads for decoding")
    from ..cover import texts_to_spans

    if seed_text is None:
        seed_text = _need(tok).decode([int(i) for i in seed_ids])
    return texts_to_spans([text], seed_text=seed_text, lm=lm, quality=quality)[0]


__all__ = ["seed_to_ids", "spans_to_text", "text_to_spans"]
