"""CPU: the oracle restatement against the reference's own outputs (golden vectors) and known answers.

The golden vectors were produced by running ``code_base/arithmetic.py`` itself (tests/golden/make_golden.py);
the known answers of ``_select_cutoff_k`` are the reference's tests/codec/test_arithmetic_threshold.py:43-58.
"""

import math

import numpy as np
import pytest

from oracle import oracle
from tests import golden


@pytest.mark.parametrize("name", golden.names())
def test_oracle_matches_reference_golden(name):
    g = golden.load(name)
    m = g.meta
    for s in g.streams:
        row = lambda t, s=s: g.row(s.stream, t).astype(np.float32)
        sent_end = g.sent_end_table() if g.finish_sent else None
        toks, _ = oracle.encode_stream(row, s.msg, banned=m["banned"], temp=m["temp"], precision=m["precision"],
                                       topk=m["topk"], sent_end=sent_end)
        assert toks == s.tokens, f"{name} stream {s.stream}: encode tokens differ from the reference"
        bits, _ = oracle.decode_stream(row, s.tokens, banned=m["banned"], temp=m["temp"],
                                       precision=m["precision"], topk=m["topk"])
        assert bits == s.bits, f"{name} stream {s.stream}: decoded bits differ from the reference"
        assert bits[: len(s.msg)] == s.msg


def test_select_cutoff_k_known_answers():
    # tests/codec/test_arithmetic_threshold.py:43-58 of the reference
    assert oracle.select_cutoff_k([0.4, 0.35, 0.25], 0.1, 50) == 3
    assert oracle.select_cutoff_k([0.4, 0.35, 0.25], 0.1, 2) == 2
    # cutoff at index 0/1 is raised to 2 (code_base/arithmetic.py:75)
    assert oracle.select_cutoff_k([0.5, 0.05, 0.01], 0.1, 50) == 2
    assert oracle.select_cutoff_k([0.05, 0.04], 0.1, 50) == 2


def test_exp_canon_accuracy():
    rng = np.random.default_rng(3)
    for d in np.concatenate([-rng.exponential(20, 2000), [0.0, -1e-300, -0.5, -700.0]]):
        ref = math.exp(d)
        got = oracle.exp_canon(d)
        assert abs(got - ref) <= 4 * math.ulp(ref), (d, got, ref)
    assert oracle.exp_canon(-700.5) == 0.0
    assert oracle.exp_canon(float("nan")) == 0.0


def test_golden_fixtures_cover_the_configs():
    names = golden.names()
    assert len(names) >= 8
    assert any(golden.load(n).finish_sent for n in names)
    g = golden.load("g1_v50257_f32_p26_k300")
    assert g.meta["precision"] == 26 and g.meta["topk"] == 300 and g.meta["temp"] == 0.9
    # ragged payload lengths including 1 bit
    assert sorted(len(s.msg) for s in g.streams)[0] == 1
