"""Codec surface of the drop-in (errors + the encode/decode slot)."""

from .errors import ArithmeticRangeError, CodecError, DecodeDivergenceError, QualityConfigError

__all__ = ["ArithmeticRangeError", "CodecError", "DecodeDivergenceError", "QualityConfigError"]
