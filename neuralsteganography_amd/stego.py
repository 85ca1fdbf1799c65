"""Batched message front end: the api's chunk -> packet -> bits -> cover-token path for many messages at once.

Restates ``stego_encode`` / ``stego_decode`` (``src/neuralstego/api.py:707-807``) with the same arguments,
defaults, packet bytes and errors, but feeds the LM provider one batch: every chunk of every message is an
independent stream of ONE lockstep GPT-2 + HIP-coder loop (``HipArithmeticLM.encode_batch``), instead of one
full LM loop per chunk.  Providers without batched entry points (e.g. ``MockLM``) are driven per packet,
exactly as the reference drives them.

Reed-Solomon (the api default ``ecc="rs"``) uses :mod:`~neuralsteganography_amd.framing.rs`, a restatement
of reedsolo's byte format (reedsolo itself is absent from this image, where the reference's ``ecc="rs"``
raises ``ConfigurationError``).

Decode needs no bit-count side channel: all emitted bits are decoded and the JSON packet is read up to its
closing brace (trailing bits of the last token's interval are ignored); a provider state queue, when
present, is still consumed in order so mixed use with ``encode_text``/``decode_text`` stays aligned.
"""

from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Any, Dict, Iterable, List, Mapping, Optional, Sequence

from .exceptions import ConfigurationError, MissingChunksError, PacketECCError
from .framing.packets import Packet, assemble_bytes, build_packets, chunk_bytes, make_msg_id, parse_packet

DEFAULT_QUALITY: Dict[str, Any] = {"temp": 1.0, "precision": 16, "topk": 50000, "finish_sent": True}  # api.py:81-86

QUALITY_KEY_ALIASES = {  # api.py:130-141
    "temperature": "temp", "top-k": "top_k", "topk": "top_k", "top_p": "top_p", "top-p": "top_p",
    "cap-per-token-bits": "cap_per_token_bits", "cap_bits_per_token": "cap_per_token_bits",
    "cap-bits-per-token": "cap_per_token_bits", "max-context": "max_context", "maxContext": "max_context",
}


@dataclass
class EncodeMetadata:
    msg_id: str
    total: int
    cfg: Dict[str, object]


class EncodeResult(list):
    """Spans (one token list per packet) with the message's framing metadata (``api.py:65-70``)."""

    def __init__(self, spans: Iterable[List[int]], metadata: EncodeMetadata) -> None:
        super().__init__(spans)
        self.metadata = metadata


def normalise_ecc(ecc: Optional[str]) -> str:
    if not ecc:
        return "none"
    e = ecc.lower()
    if e not in ("none", "rs"):
        raise ConfigurationError(f"unsupported ecc mode: {ecc}")
    return e


def normalise_quality(quality: Optional[Mapping[str, object]]) -> Dict[str, Any]:
    return {QUALITY_KEY_ALIASES.get(k, k): v for k, v in (quality or {}).items()}


def _quality_args(quality) -> Dict[str, Any]:
    return {**DEFAULT_QUALITY, **normalise_quality(quality)}


def bytes_to_bits_lsb(data: bytes) -> List[int]:
    """``api.py:153-157``: LSB-first bits of every byte."""
    return [(b >> i) & 1 for b in bytes(data) for i in range(8)]


def bits_to_bytes_lsb(bits: Sequence[int]) -> bytes:
    """Whole bytes of an LSB-first bit list (a trailing partial byte is dropped)."""
    n = len(bits) // 8
    out = bytearray(n)
    for i in range(n):
        v = 0
        for k in range(8):
            v |= (int(bits[8 * i + k]) & 1) << k
        out[i] = v
    return bytes(out)


def packet_prefix(data: bytes) -> bytes:
    """The leading JSON packet of ``data`` (decoded bits may run past it): raw_decode stops at its end."""
    text = bytes(data).decode("utf-8", errors="replace")
    try:
        obj, end = json.JSONDecoder().raw_decode(text)
    except ValueError as exc:
        raise PacketECCError("decoded bits do not start with a packet") from exc
    if not isinstance(obj, dict):
        raise PacketECCError("decoded packet is not a JSON object")
    return text[:end].encode("utf-8")


def _encode_streams(lm, bit_lists: List[List[int]], context: List[int], quality: Dict[str, Any]) -> List[List[int]]:
    if hasattr(lm, "encode_batch"):
        return lm.encode_batch(bit_lists, context, quality=quality)
    return [lm.encode_arithmetic(bits, context, quality=quality) for bits in bit_lists]


def _decode_streams(lm, spans: List[List[int]], context: List[int], quality: Dict[str, Any]) -> List[List[int]]:
    if hasattr(lm, "decode_batch"):
        if getattr(lm, "decodes_without_state", False):
            # the arithmetic coder decodes from the tokens alone: drop the queued states to stay aligned
            queue = getattr(lm, "_decode_states", None)
            if queue:
                for _ in range(min(len(spans), len(queue))):
                    queue.popleft()
        # (a provider that needs its history, like the rank coder, pops its own states in decode_batch)
        return lm.decode_batch(spans, context, quality=quality)
    return [lm.decode_arithmetic(list(span), context, quality=quality) for span in spans]


def stego_encode_batch(messages: Sequence[bytes], *, chunk_bytes: int = 256, use_crc: bool = True,
                       ecc: Optional[str] = "rs", nsym: int = 10, quality: Optional[Dict[str, float]] = None,
                       seed_text: str = "", lm) -> List[EncodeResult]:
    """Every message -> its :class:`EncodeResult`; all packets of all messages are encoded as one batch."""
    mode = normalise_ecc(ecc)
    cfg = {"chunk_bytes": int(chunk_bytes), "crc": bool(use_crc), "ecc": mode, "nsym": int(nsym if mode == "rs" else 0)}
    q = _quality_args(quality)
    metas: List[EncodeMetadata] = []
    bit_lists: List[List[int]] = []
    owner: List[int] = []
    for mi, message in enumerate(messages):
        chunks = chunk_bytes_of(message, cfg["chunk_bytes"])
        msg_id = make_msg_id()
        metas.append(EncodeMetadata(msg_id=msg_id, total=len(chunks), cfg=dict(cfg)))
        for pkt in build_packets(chunks, msg_id=msg_id, cfg=cfg):
            bit_lists.append(bytes_to_bits_lsb(pkt))
            owner.append(mi)
    context = list(lm.encode_seed(seed_text))
    spans = _encode_streams(lm, bit_lists, context, q) if bit_lists else []
    per: List[List[List[int]]] = [[] for _ in messages]
    for mi, span in zip(owner, spans):
        per[mi].append([int(t) for t in span])
    return [EncodeResult(per[mi], metas[mi]) for mi in range(len(messages))]


def chunk_bytes_of(message: bytes, size: int) -> List[bytes]:
    return chunk_bytes(bytes(message), chunk_size=size)


def stego_encode(message: bytes, *, chunk_bytes: int = 256, use_crc: bool = True, ecc: Optional[str] = "rs",
                 nsym: int = 10, quality: Optional[Dict[str, float]] = None, seed_text: str = "", lm) -> EncodeResult:
    """``api.py:707`` -- one message."""
    return stego_encode_batch([message], chunk_bytes=chunk_bytes, use_crc=use_crc, ecc=ecc, nsym=nsym,
                              quality=quality, seed_text=seed_text, lm=lm)[0]


def _assemble(packets: List[Packet]) -> bytes:
    by_seq: Dict[int, bytes] = {}
    msg_id = total = None
    for pkt in packets:
        if msg_id is None:
            msg_id, total = pkt.msg_id, pkt.total
        else:
            if pkt.msg_id != msg_id:
                raise ConfigurationError("decoded packet msg_id mismatch")
            if pkt.total != total:
                raise ConfigurationError("decoded packet total mismatch")
        if pkt.seq in by_seq:
            raise ConfigurationError(f"duplicate packet sequence {pkt.seq}")
        by_seq[pkt.seq] = pkt.payload
    if total is None:
        return b""
    present = sorted(by_seq)
    missing = sorted(set(range(total)) - set(by_seq))
    assembled = assemble_bytes(by_seq[i] for i in present)
    if missing:
        raise MissingChunksError(missing_indices=missing, partial_payload=assembled)
    return assembled


def stego_decode_batch(span_sets: Sequence[Iterable[List[int]]], *, use_crc: bool = True, ecc: Optional[str] = "rs",
                       nsym: int = 10, quality: Optional[Dict[str, float]] = None, seed_text: str = "", lm,
                       return_errors: bool = False) -> List[Any]:
    """Every message's spans -> its bytes, all spans decoded as one batch.  Errors (missing chunks, CRC, RS,
    cfg mismatch) raise for the first failing message, or are returned in its slot with
    ``return_errors=True``."""
    mode = normalise_ecc(ecc)
    expected = {"crc": bool(use_crc), "ecc": mode, "nsym": int(nsym if mode == "rs" else 0)}
    q = _quality_args(quality)
    flat: List[List[int]] = []
    owner: List[int] = []
    for mi, spans in enumerate(span_sets):
        for span in spans:
            flat.append([int(t) for t in span])
            owner.append(mi)
    context = list(lm.encode_seed(seed_text))
    bits = _decode_streams(lm, flat, context, q) if flat else []
    packets: List[List[Packet]] = [[] for _ in span_sets]
    errors: List[Optional[Exception]] = [None] * len(span_sets)
    for mi, b in zip(owner, bits):
        if errors[mi] is not None:
            continue
        try:
            packets[mi].append(parse_packet(packet_prefix(bits_to_bytes_lsb(b)), expected_cfg=expected))
        except Exception as exc:  # noqa: BLE001 - reported per message
            errors[mi] = exc
    out: List[Any] = []
    for mi in range(len(span_sets)):
        try:
            if errors[mi] is not None:
                raise errors[mi]
            out.append(_assemble(packets[mi]))
        except Exception as exc:  # noqa: BLE001
            if not return_errors:
                raise
            out.append(exc)
    return out


def stego_decode(spans: Iterable[List[int]], *, use_crc: bool = True, ecc: Optional[str] = "rs", nsym: int = 10,
                 quality: Optional[Dict[str, float]] = None, seed_text: str = "", lm) -> bytes:
    """``api.py:745`` -- one message."""
    return stego_decode_batch([list(spans)], use_crc=use_crc, ecc=ecc, nsym=nsym, quality=quality,
                              seed_text=seed_text, lm=lm)[0]


__all__ = ["EncodeMetadata", "EncodeResult", "stego_encode", "stego_decode", "stego_encode_batch",
           "stego_decode_batch", "DEFAULT_QUALITY", "bytes_to_bits_lsb", "bits_to_bytes_lsb", "packet_prefix"]
