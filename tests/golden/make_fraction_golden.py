"""Golden outcomes of the reference's exact-rational coder (src/neuralstego/codec/arithmetic.py encode_bits /
decode_bits, row a12 of SURVEY §8), produced by RUNNING it here: tokens, per-token consumption and the decode
result, or the exception each call raises.  Distributions are regenerated from (V, seed) by
``dists(V, seed, n)`` below, so the fixture holds no arrays.
usage (this container only): python tests/golden/make_fraction_golden.py
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent

CASES = [(p, V) for p in ["00", "000000", "ff", "ffff", "80", "55", "01", "0000000000000000", "", "0001"]
         for V in (2, 4, 16)]


def dists(V: int, seed: int, n: int = 200, as_dict: bool = False):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        p = rng.random(V)
        p[rng.integers(0, V)] = 0.0 if V > 2 else p[0]  # a zero-probability token (dropped from the CDF)
        p /= p.sum()
        out.append({int(i): float(v) for i, v in enumerate(p)} if as_dict else p)
    return out


def main():
    sys.path.insert(0, str(REF / "src"))
    from neuralstego.codec import arithmetic as A

    out = []
    for payload_hex, V in CASES + [("000000", -4)]:
        as_dict = V < 0
        V = abs(V)
        payload = bytes.fromhex(payload_hex)
        ds = dists(V, 1000 + V, as_dict=as_dict)
        rec = {"payload": payload_hex, "V": V, "seed": 1000 + V, "as_dict": as_dict}
        state = {}
        try:
            toks = A.encode_bits(payload, iter(ds), state=state)
            rec["tokens"] = list(map(int, toks))
            rec["history"] = list(state["history"])
            rec["residual_bits"] = state["residual_bits"].hex()
            try:
                dec = A.decode_bits(toks, iter(ds), state=dict(state))
                rec["decoded"] = dec.hex()
            except Exception as exc:  # noqa: BLE001 - the exception class is the recorded outcome
                rec["decode_error"] = type(exc).__name__
        except Exception as exc:  # noqa: BLE001
            rec["encode_error"] = type(exc).__name__
        out.append(rec)
        print(rec, flush=True)
    (HERE / "fraction_golden.json").write_text(json.dumps(out, indent=0))


if __name__ == "__main__":
    main()
