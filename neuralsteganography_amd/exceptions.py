"""Error surface of the drop-in boundary, mirroring ``src/neuralstego/exceptions.py:8-52``."""

from __future__ import annotations


class NeuralStegoError(Exception):
    """Base class for all neural-steganography errors (``exceptions.py:8``)."""


class ConfigurationError(NeuralStegoError):
    """Invalid user configuration (``exceptions.py:12``)."""


class FramingError(NeuralStegoError):
    """Packet framing or chunk assembly failed (``exceptions.py:16``)."""


class PacketECCError(FramingError):
    """Reed-Solomon decoding (or the packet envelope) failed irrecoverably (``exceptions.py:20``)."""


class PacketCRCError(FramingError):
    """CRC32 verification failed (``exceptions.py:24``)."""


class MissingChunksError(FramingError):
    """Some packets of a message never arrived (``exceptions.py:28-35``); ``partial_payload`` holds the
    payloads that did, in sequence order."""

    def __init__(self, missing_indices, partial_payload: bytes = b""):
        self.missing_indices = list(missing_indices)
        self.partial_payload = bytes(partial_payload)
        super().__init__(self.missing_indices, self.partial_payload)

    def __str__(self) -> str:
        return "Missing chunks at indices: " + ", ".join(str(i) for i in self.missing_indices)


class QualityGateError(NeuralStegoError):
    """Every cover-generation attempt was rejected by the quality gate (``exceptions.py:38-50``): the last
    attempt's ``cover_text``, its rejection ``reasons`` and ``metrics``."""

    def __init__(self, cover_text: str, reasons, metrics):
        self.cover_text = str(cover_text)
        self.reasons = list(reasons)
        self.metrics = dict(metrics)
        super().__init__(self.cover_text, self.reasons, self.metrics)

    def __str__(self) -> str:
        if not self.reasons:
            return "quality gate rejected the generated cover"
        return "quality gate rejected the generated cover: " + "; ".join(self.reasons)


class KVCapacityError(NeuralStegoError, RuntimeError):
    """The paged KV cache cannot give a stream its next page: the device has no memory left for it (a library
    error, never PyTorch's out-of-memory).  The reference keeps one unbounded cache per message
    (``code_base/arithmetic.py:96-122``) and has no such limit short of the machine's memory."""


__all__ = ["NeuralStegoError", "ConfigurationError", "FramingError", "PacketECCError", "PacketCRCError",
           "MissingChunksError", "QualityGateError", "KVCapacityError"]
