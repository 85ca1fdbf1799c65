"""Codec exceptions, mirroring ``src/neuralstego/codec/errors.py:6-19``."""

from __future__ import annotations


class CodecError(Exception):
    """Base class for codec-specific exceptions."""


class ArithmeticRangeError(CodecError):
    """The arithmetic coder found no bucket for the payload index (``codec/arithmetic.py:150``)."""


class DecodeDivergenceError(CodecError):
    """Decoding left the arithmetic interval: a received token is outside the kept top-k."""


class QualityConfigError(CodecError):
    """Quality or capacity policies are misconfigured."""


__all__ = ["CodecError", "ArithmeticRangeError", "DecodeDivergenceError", "QualityConfigError"]
