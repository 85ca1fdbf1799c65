"""CPU: the batched framing front end (neuralsteganography_amd/stego.py, framing/) -- host logic.

Mirrors the reference's tests/framing (test_ecc.py, test_crc.py, test_api_end_to_end.py,
test_fault_injection.py), which skip their Reed-Solomon cases here because reedsolo is absent; the RS
restatement is pinned to reedsolo's documented RSCodec(10).encode outputs instead.
"""

import json
import os
import zlib
from copy import deepcopy

import pytest

from neuralsteganography_amd.exceptions import MissingChunksError, PacketCRCError, PacketECCError
from neuralsteganography_amd.framing import packets
from neuralsteganography_amd.framing.rs import generator_poly, rs_decode, rs_encode, rs_encode_many
from neuralsteganography_amd.lm.mock import MockLM
from neuralsteganography_amd.stego import stego_decode, stego_decode_batch, stego_encode, stego_encode_batch


def test_rs_matches_reedsolo_documented_outputs():
    # reedsolo README: RSCodec(10).encode(...) (prim 0x11d, generator 2, fcr 0)
    assert rs_encode(b"hello world", 10) == b"hello world\xed%T\xc4\xfd\xfd\x89\xf3\xa8\xaa"
    assert rs_encode(bytes([1, 2, 3, 4]), 10) == b"\x01\x02\x03\x04,\x9d\x1c+=\xf8h\xfa\x98M"
    assert len(generator_poly(10)) == 11


def test_rs_roundtrip_and_corrections():  # reference tests/framing/test_ecc.py
    ok, dec = rs_decode(rs_encode(b"neural stego", 8), 8)
    assert ok and dec == b"neural stego"
    enc = bytearray(rs_encode(b"0123456789abcdef", 8))
    enc[0] ^= 0x01
    enc[3] ^= 0x01
    enc[5] ^= 0x02
    assert rs_decode(bytes(enc), 8) == (True, b"0123456789abcdef")
    enc = bytearray(rs_encode(b"another block", 4))
    enc[0] ^= 0x01
    enc[1] ^= 0x02
    enc[2] ^= 0x04
    assert rs_decode(bytes(enc), 4) == (False, b"")


def test_rs_multi_block_and_batched_parity():
    msgs = [os.urandom(n) for n in (1, 245, 246, 600, 0, 17)]
    batch = rs_encode_many(msgs, 10)
    for m, e in zip(msgs, batch):
        assert e == rs_encode(m, 10)
        assert len(e) == len(m) + 10 * ((len(m) + 244) // 245)
        bad = bytearray(e)
        for blk in range(0, len(bad), 255):
            for k in range(min(5, len(bad) - blk)):
                bad[blk + k] ^= 0x5A
        ok, dec = rs_decode(bytes(bad), 10)
        assert ok and dec == m


def test_crc32_known_value_and_detection():  # reference tests/framing/test_crc.py
    assert zlib.crc32(b"hello") == 0x3610A686
    blob = packets.crc32_append(b"payload")
    assert packets.crc32_strip(blob) == b"payload"
    bad = bytearray(blob)
    bad[0] ^= 0xFF
    with pytest.raises(PacketCRCError):
        packets.crc32_strip(bytes(bad))


def test_packet_bytes_layout():
    pkt = packets.build_packet(b"hi", msg_id="m", seq=0, total=1, cfg={"chunk_bytes": 256, "crc": True,
                                                                         "ecc": "rs", "nsym": 10})
    obj = json.loads(pkt)
    assert list(obj) == sorted(obj) and obj["version"] == 1
    assert pkt == json.dumps(obj, separators=(",", ":"), sort_keys=True).encode()
    assert packets.parse_packet(pkt).payload == b"hi"
    with pytest.raises(PacketECCError):
        packets.parse_packet(b"not json")


@pytest.mark.parametrize("cfg", [{"ecc": "none", "use_crc": False, "nsym": 0},
                                 {"ecc": "none", "use_crc": True, "nsym": 0},
                                 {"ecc": "rs", "use_crc": True, "nsym": 10}])
def test_end_to_end_mock_lm(cfg):  # reference tests/framing/test_api_end_to_end.py
    data = os.urandom(4096)
    lm = MockLM()
    res = stego_encode(data, chunk_bytes=256, quality={"precision": 8}, seed_text="seed.", lm=lm, **cfg)
    assert res.metadata.total == len(res) == 16
    assert stego_decode(list(res), quality={"precision": 8}, seed_text="seed.", lm=lm, **cfg) == data


def _corrupt_payload_symbol(span):
    pkt = json.loads(bytes(span).decode("utf-8"))
    p = bytearray(pkt["payload"].encode("ascii"))
    p[0] = ord("B") if p[0] != ord("B") else ord("A")
    pkt["payload"] = p.decode("ascii")
    return list(json.dumps(pkt, separators=(",", ":"), sort_keys=True).encode("utf-8"))


def test_fault_injection_rs_corrects_and_unprotected_changes():  # reference test_fault_injection.py
    data = os.urandom(4096)
    lm = MockLM()
    res = stego_encode(data, quality={"precision": 8}, lm=lm)
    spans = deepcopy(list(res))
    spans[0] = _corrupt_payload_symbol(spans[0])
    assert stego_decode(spans, quality={"precision": 8}, lm=lm) == data
    res = stego_encode(data, use_crc=False, ecc="none", nsym=0, quality={"precision": 8}, lm=lm)
    spans = deepcopy(list(res))
    spans[0] = _corrupt_payload_symbol(spans[0])
    assert stego_decode(spans, use_crc=False, ecc="none", nsym=0, quality={"precision": 8}, lm=lm) != data


def test_missing_span_reported_with_partial_payload():
    data = os.urandom(4096)
    lm = MockLM()
    res = stego_encode(data, lm=lm)
    spans = list(res)
    gone = len(spans) // 2
    spans.pop(gone)
    with pytest.raises(MissingChunksError) as ei:
        stego_decode(spans, lm=lm)
    assert ei.value.missing_indices == [gone]
    chunks = packets.chunk_bytes(data, chunk_size=256)
    assert ei.value.partial_payload == b"".join(c for i, c in enumerate(chunks) if i != gone)


def test_batched_messages_and_per_message_errors():
    lm = MockLM()
    msgs = [os.urandom(n) for n in (0, 1, 255, 256, 1000, 3000)]
    results = stego_encode_batch(msgs, chunk_bytes=200, lm=lm)
    assert [r.metadata.total for r in results] == [max(1, -(-len(m) // 200)) for m in msgs]
    assert len({r.metadata.msg_id for r in results}) == len(msgs)
    assert stego_decode_batch([list(r) for r in results], lm=lm) == msgs
    broken = [list(r) for r in results]
    broken[4] = broken[4][1:]
    out = stego_decode_batch(broken, lm=lm, return_errors=True)
    assert isinstance(out[4], MissingChunksError) and out[4].missing_indices == [0]
    assert [o for i, o in enumerate(out) if i != 4] == [m for i, m in enumerate(msgs) if i != 4]
