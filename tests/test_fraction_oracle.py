"""CPU: the oracle's restatement of the reference's exact-rational coder (codec/arithmetic.py:234-550, row a12)
reproduces every outcome of the reference run in tests/golden/fraction_golden.json -- tokens, per-token
consumption, residual bit count, decoded bytes, and which call raises (mostly ArithmeticRangeError: the coder
is non-functional for general payloads; DESIGN.md §4, Fraction coder)."""

import json
from pathlib import Path

import pytest

from oracle import fraction_coder as fc
from tests.golden.make_fraction_golden import dists

G = json.loads((Path(__file__).resolve().parent / "golden" / "fraction_golden.json").read_text())


@pytest.mark.parametrize("rec", G, ids=[f"{r['payload'] or 'empty'}-V{r['V']}{'-dict' if r['as_dict'] else ''}" for r in G])
def test_fraction_coder_restatement_matches_reference(rec):
    ds = dists(rec["V"], rec["seed"], as_dict=rec["as_dict"])
    payload = bytes.fromhex(rec["payload"])
    if "encode_error" in rec:
        assert rec["encode_error"] == "ArithmeticRangeError"
        with pytest.raises(fc.RangeError):
            fc.encode(payload, ds)
        return
    toks, st = fc.encode(payload, ds)
    assert toks == rec["tokens"] and list(st["history"]) == rec["history"]
    assert st["residual_bits"].hex() == rec["residual_bits"]
    if "decode_error" in rec:
        with pytest.raises((fc.RangeError, fc.DivergenceError)):
            fc.decode(toks, ds, st)
    else:
        assert fc.decode(toks, ds, st).hex() == rec["decoded"]


def test_fraction_coder_is_mostly_non_functional():
    """The reference's coder cannot carry most payloads: most recorded cases end in ArithmeticRangeError
    (the kernel of row a12 reproduces that, tests/test_gpu_fraction.py)."""
    failed = sum("encode_error" in r for r in G)
    assert failed >= len(G) // 3
