"""Reed-Solomon over GF(2^8) in the byte format of ``reedsolo.RSCodec(nsym)`` (its defaults: primitive
polynomial 0x11d, generator 2, first consecutive root 0, codeword length 255).

``reedsolo`` is what the reference's packet framing calls (``src/neuralstego/codec/packet.py:29-63``,
``framing/ecc.py``); it is not installed in this image, so with the reference as shipped ``ecc="rs"``
(the api default) cannot run.  This module restates the published algorithm:

* encode: the message is cut into blocks of 255 - nsym bytes; each block is followed by the nsym-byte
  remainder of block(x) * x^nsym modulo g(x) = prod_{i<nsym} (x - 2^i) (systematic code, the block's first
  byte is the highest-degree coefficient);
* decode: blocks of 255 bytes (the last may be shorter); syndromes S_j = r(2^j); Berlekamp-Massey for the
  error locator; Chien search; Forney magnitudes; a block with more than nsym/2 errors is reported.

Encoding is vectorised over all equal-length blocks with numpy table lookups (the batched front end frames
thousands of packets at once); decoding is per block and only runs its locator search when a syndrome is
nonzero.
"""

from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

PRIM = 0x11D
NSIZE = 255

_EXP = np.zeros(512, dtype=np.int64)
_LOG = np.zeros(256, dtype=np.int64)
_x = 1
for _i in range(255):
    _EXP[_i] = _x
    _LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= PRIM
_EXP[255:510] = _EXP[0:255]


class RSDecodeError(ValueError):
    """More errors than the code can correct (or an uncorrectable pattern)."""


def gf_mul(a: int, b: int) -> int:
    if a == 0 or b == 0:
        return 0
    return int(_EXP[_LOG[a] + _LOG[b]])


def gf_div(a: int, b: int) -> int:
    if b == 0:
        raise ZeroDivisionError("division by zero in GF(256)")
    if a == 0:
        return 0
    return int(_EXP[(_LOG[a] - _LOG[b]) % 255])


def gf_pow2(e: int) -> int:
    return int(_EXP[e % 255])


def generator_poly(nsym: int) -> List[int]:
    """g(x) = prod_{i<nsym} (x + 2^i), highest degree first."""
    g = [1]
    for i in range(nsym):
        root = gf_pow2(i)
        nxt = g + [0]
        for j in range(len(g)):
            nxt[j + 1] ^= gf_mul(g[j], root)
        g = nxt
    return g


def _encode_blocks(blocks: np.ndarray, nsym: int) -> np.ndarray:
    """Parity of every row of ``blocks`` ([n, k] uint8) -> [n, nsym] (LFSR division by g, vectorised)."""
    g = np.asarray(generator_poly(nsym)[1:], dtype=np.int64)
    glog = _LOG[g]
    rem = np.zeros((blocks.shape[0], nsym), dtype=np.int64)
    for j in range(blocks.shape[1]):
        fb = blocks[:, j].astype(np.int64) ^ rem[:, 0]
        rem[:, :-1] = rem[:, 1:]
        rem[:, -1] = 0
        nz = fb != 0
        if nz.any():
            prod = _EXP[(_LOG[fb[nz]][:, None] + glog[None, :])]
            prod[:, g == 0] = 0
            rem[nz] ^= prod
    return rem.astype(np.uint8)


def rs_encode_many(messages: Sequence[bytes], nsym: int) -> List[bytes]:
    """reedsolo ``RSCodec(nsym).encode`` of every message (blocks of 255 - nsym bytes, parity appended)."""
    if not 0 < nsym < NSIZE:
        raise ValueError("nsym must be within (0, 255)")
    k = NSIZE - nsym
    # group blocks by length so each group is one vectorised division
    pieces: List[List[bytes]] = []
    groups = {}
    for mi, msg in enumerate(messages):
        msg = bytes(msg)
        blocks = [msg[i:i + k] for i in range(0, len(msg), k)] or []
        pieces.append(blocks)
        for bi, blk in enumerate(blocks):
            groups.setdefault(len(blk), []).append((mi, bi))
    parity = {}
    for length, where in groups.items():
        arr = np.frombuffer(b"".join(pieces[mi][bi] for mi, bi in where), dtype=np.uint8).reshape(len(where), length)
        par = _encode_blocks(arr, nsym)
        for row, (mi, bi) in enumerate(where):
            parity[(mi, bi)] = par[row].tobytes()
    return [b"".join(blk + parity[(mi, bi)] for bi, blk in enumerate(blocks)) for mi, blocks in enumerate(pieces)]


def rs_encode(data: bytes, nsym: int) -> bytes:
    return rs_encode_many([data], nsym)[0]


def _poly_eval_bytes(block: Sequence[int], x: int) -> int:
    y = 0
    for c in block:
        y = gf_mul(y, x) ^ int(c)
    return y


def _decode_block(block: bytearray, nsym: int) -> bytearray:
    n = len(block)
    synd = [_poly_eval_bytes(block, gf_pow2(j)) for j in range(nsym)]
    if not any(synd):
        return block
    # Berlekamp-Massey: error locator C(x) = 1 + C1 x + ..., ascending powers
    C, B = [1], [1]
    L, m, b = 0, 1, 1
    for r in range(nsym):
        d = synd[r]
        for i in range(1, L + 1):
            if i < len(C):
                d ^= gf_mul(C[i], synd[r - i])
        if d == 0:
            m += 1
            continue
        coef = gf_div(d, b)
        shifted = [0] * m + [gf_mul(coef, v) for v in B]
        T = list(C)
        if len(shifted) > len(C):
            C = C + [0] * (len(shifted) - len(C))
        for i, v in enumerate(shifted):
            C[i] ^= v
        if 2 * L <= r:
            L, B, b, m = r + 1 - L, T, d, 1
        else:
            m += 1
    while len(C) > 1 and C[-1] == 0:
        C.pop()
    if L * 2 > nsym or len(C) - 1 != L:
        raise RSDecodeError("too many errors to correct")
    # Chien search over the n byte positions: byte i sits at power n-1-i, locator X = 2^(n-1-i)
    positions = []
    for i in range(n):
        xinv = gf_pow2(-(n - 1 - i))
        acc = 0
        for k in range(len(C) - 1, -1, -1):
            acc = gf_mul(acc, xinv) ^ C[k]
        if acc == 0:
            positions.append(i)
    if len(positions) != L:
        raise RSDecodeError("error locator has roots outside the block")
    # Forney (first root 2^0): e = X * Omega(X^-1) / C'(X^-1), Omega = S(x) C(x) mod x^nsym
    omega = [0] * nsym
    for i, s in enumerate(synd):
        for j, c in enumerate(C):
            if i + j < nsym:
                omega[i + j] ^= gf_mul(s, c)
    for i in positions:
        X = gf_pow2(n - 1 - i)
        xinv = gf_pow2(-(n - 1 - i))
        om = 0
        for k in range(nsym - 1, -1, -1):
            om = gf_mul(om, xinv) ^ omega[k]
        der = 0
        for k in range(1, len(C), 2):  # formal derivative: odd powers
            der ^= gf_mul(C[k], gf_pow2(_LOG[xinv] * (k - 1)) if xinv else 0)
        if der == 0:
            raise RSDecodeError("degenerate error locator")
        block[i] ^= gf_mul(X, gf_div(om, der))
    if any(_poly_eval_bytes(block, gf_pow2(j)) for j in range(nsym)):
        raise RSDecodeError("could not correct the block")
    return block


def rs_decode_checked(data: bytes, nsym: int) -> bytes:
    """reedsolo ``RSCodec(nsym).decode(data)[0]``: the corrected message; raises :class:`RSDecodeError`."""
    if not 0 < nsym < NSIZE:
        raise ValueError("nsym must be within (0, 255)")
    out = bytearray()
    for i in range(0, len(data), NSIZE):
        blk = bytearray(data[i:i + NSIZE])
        if len(blk) <= nsym:
            raise RSDecodeError("block shorter than its parity")
        out += _decode_block(blk, nsym)[:-nsym]
    return bytes(out)


def rs_decode(data: bytes, nsym: int) -> Tuple[bool, bytes]:
    """``framing/ecc.py`` form: ``(ok, message)``, ``(False, b"")`` when uncorrectable."""
    try:
        return True, rs_decode_checked(data, nsym)
    except RSDecodeError:
        return False, b""


__all__ = ["RSDecodeError", "generator_poly", "rs_encode", "rs_encode_many", "rs_decode", "rs_decode_checked"]
