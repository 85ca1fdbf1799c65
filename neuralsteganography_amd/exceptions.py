"""Error surface of the drop-in boundary, mirroring ``src/neuralstego/exceptions.py:8-52``."""

from __future__ import annotations


class NeuralStegoError(Exception):
    """Base class for all neural-steganography errors (``exceptions.py:8``)."""


class ConfigurationError(NeuralStegoError):
    """Invalid user configuration (``exceptions.py:12``)."""


__all__ = ["NeuralStegoError", "ConfigurationError"]
