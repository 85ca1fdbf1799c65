"""Crypto-side arithmetic helpers (``src/neuralstego/crypto/arithmetic.py``), row a14 of SURVEY §8."""

from .arithmetic import QualityControlledLM, decode_arithmetic, encode_arithmetic

__all__ = ["QualityControlledLM", "encode_arithmetic", "decode_arithmetic"]
