"""Packet envelope of the api path (``src/neuralstego/codec/packet.py:68-160``, ``codec/chunker.py:14-38``),
restated for the batched front end.

A packet is compact, key-sorted JSON ``{"cfg", "msg_id", "payload", "seq", "total", "version": 1}`` whose
payload is base64 of ``RS(chunk [+ CRC32 big-endian])``; the byte layout is the reference's, so packets
built here parse there and vice versa.  Framing many packets at once batches the Reed-Solomon parity
(:func:`~neuralsteganography_amd.framing.rs.rs_encode_many`).
"""

from __future__ import annotations

import base64
import binascii
import json
import struct
import uuid
import zlib
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

from ..exceptions import ConfigurationError, PacketCRCError, PacketECCError
from .rs import RSDecodeError, rs_decode_checked, rs_encode_many


@dataclass(frozen=True)
class Packet:
    msg_id: str
    seq: int
    total: int
    cfg: Dict[str, Any]
    payload: bytes


def make_msg_id() -> str:
    return str(uuid.uuid4())


def chunk_bytes(data: bytes, *, chunk_size: int = 256) -> List[bytes]:
    """``codec/chunker.py:14``: fixed-size slices; an empty message is one empty chunk."""
    if chunk_size <= 0:
        raise ValueError("chunk_size must be positive")
    data = bytes(data)
    return [data[i:i + chunk_size] for i in range(0, len(data), chunk_size)] or [b""]


def assemble_bytes(chunks) -> bytes:
    return b"".join(bytes(c) for c in chunks)


def normalise_cfg(cfg: Dict[str, Any]) -> Dict[str, Any]:
    return {"chunk_bytes": cfg.get("chunk_bytes"), "crc": bool(cfg.get("crc", False)),
            "ecc": cfg.get("ecc", "none"), "nsym": int(cfg.get("nsym", 0))}


def crc32_append(data: bytes) -> bytes:
    return data + struct.pack(">I", zlib.crc32(data) & 0xFFFFFFFF)


def crc32_strip(data: bytes) -> bytes:
    if len(data) < 4:
        raise PacketCRCError("payload too small to contain CRC32")
    body, tail = data[:-4], data[-4:]
    if struct.pack(">I", zlib.crc32(body) & 0xFFFFFFFF) != tail:
        raise PacketCRCError("CRC32 mismatch detected")
    return body


def build_packets(chunks: Sequence[bytes], *, msg_id: str, cfg: Dict[str, Any], seqs: Optional[Sequence[int]] = None,
                  total: Optional[int] = None) -> List[bytes]:
    """Packets for ``chunks`` (sequence numbers ``seqs``, default 0..n-1, of ``total``), RS batched."""
    c = normalise_cfg(cfg)
    total = len(chunks) if total is None else int(total)
    seqs = list(range(len(chunks))) if seqs is None else [int(s) for s in seqs]
    for s in seqs:
        if s < 0 or total <= 0 or s >= total:
            raise ValueError("invalid sequence/total combination")
    framed = [crc32_append(bytes(ch)) if c["crc"] else bytes(ch) for ch in chunks]
    if c["ecc"] == "rs":
        if c["nsym"] <= 0:
            raise ValueError("nsym must be positive when ecc='rs'")
        framed = rs_encode_many(framed, c["nsym"])
    elif c["ecc"] not in ("none", None):
        raise ConfigurationError(f"unsupported ecc mode: {c['ecc']}")
    out = []
    for s, body in zip(seqs, framed):
        obj = {"version": 1, "msg_id": msg_id, "seq": s, "total": total, "cfg": c,
               "payload": base64.b64encode(body).decode("ascii")}
        out.append(json.dumps(obj, separators=(",", ":"), sort_keys=True).encode("utf-8"))
    return out


def build_packet(payload: bytes, *, msg_id: str, seq: int, total: int, cfg: Dict[str, Any]) -> bytes:
    return build_packets([payload], msg_id=msg_id, cfg=cfg, seqs=[seq], total=total)[0]


def parse_packet(packet: bytes, *, expected_cfg: Optional[Dict[str, Any]] = None) -> Packet:
    """``codec/packet.py:116``: envelope checks, cfg check, RS correction, CRC verification."""
    try:
        obj = json.loads(bytes(packet).decode("utf-8"))
    except (ValueError, UnicodeDecodeError) as exc:
        raise PacketECCError("invalid packet encoding") from exc
    if not isinstance(obj, dict):
        raise PacketECCError("packet is not a JSON object")
    need = {"msg_id", "seq", "total", "cfg", "payload"}
    if not need.issubset(obj):
        raise PacketECCError("missing packet keys: " + ", ".join(sorted(need - set(obj))))
    c = normalise_cfg(obj["cfg"])
    for key, value in (expected_cfg or {}).items():
        if key in c and value is not None and c[key] != value:
            raise ConfigurationError(f"packet cfg mismatch for {key}: expected {value}, got {c[key]}")
    try:
        body = base64.b64decode(obj["payload"], validate=True)
    except (ValueError, TypeError, binascii.Error) as exc:
        raise PacketECCError("payload is not valid base64") from exc
    if c["ecc"] == "rs":
        try:
            body = rs_decode_checked(body, c["nsym"])
        except RSDecodeError as exc:
            raise PacketECCError("Reed-Solomon decoding failed") from exc
    elif c["ecc"] not in ("none", None):
        raise ConfigurationError(f"unsupported ecc mode: {c['ecc']}")
    if c["crc"]:
        body = crc32_strip(body)
    return Packet(msg_id=obj["msg_id"], seq=int(obj["seq"]), total=int(obj["total"]), cfg=c, payload=body)


__all__ = ["Packet", "make_msg_id", "chunk_bytes", "assemble_bytes", "build_packet", "build_packets",
           "parse_packet", "crc32_append", "crc32_strip", "normalise_cfg"]
