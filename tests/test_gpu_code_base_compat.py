"""GPU: the code_base drop-in (neuralsteganography_amd/code_base.py) against the reference run.

Fixtures c* (tests/golden/make_golden.py) ran the reference's encode_arithmetic -> enc.decode -> its
decode_arithmetic through a toy greedy tokenizer whose re-tokenisation forces the BPE repair of
code_base/arithmetic.py:300-342 (including unrepairable tokens, which the reference decodes as rank 0) and
the '<eos>' stop of :207-210.  Tokens and decoded bits must be identical; statistics within rel 2e-5.
"""

from __future__ import annotations

import pytest

from neuralsteganography_amd import synthetic
from tests import golden
from tests.golden.toy_tokenizer import ToyTokenizer

pytestmark = pytest.mark.gpu


def _lm(g, streams):
    m = g.meta
    return synthetic.SyntheticBatchedLM(m["logit_seed"], m["vocab"], m["scale"], "f32", streams=streams,
                                        boost=g.boost)


@pytest.mark.parametrize("name", golden.compat_names())
def test_code_base_encode_matches_reference(name):
    from neuralsteganography_amd import code_base

    g = golden.load_compat(name)
    m = g.meta
    enc = ToyTokenizer(m["vocab"])
    res = code_base.encode_arithmetic_batch(_lm(g, [s.stream for s in g.streams]), enc, [s.msg for s in g.streams],
                                            m["context"], temp=m["temp"], precision=m["precision"], topk=m["topk"])
    for s, (toks, nll, kl, wpb, hq) in zip(g.streams, res):
        assert toks == s.tokens, f"{name} stream {s.stream}: tokens differ from the reference"
        for got, want in zip((nll, kl, wpb, hq), s.stats):
            assert got == pytest.approx(want, rel=2e-5, abs=2e-6)


@pytest.mark.parametrize("name", golden.compat_names())
def test_code_base_decode_with_bpe_repair_matches_reference(name):
    from neuralsteganography_amd import code_base

    g = golden.load_compat(name)
    m = g.meta
    enc = ToyTokenizer(m["vocab"])
    bits = code_base.decode_arithmetic_batch(_lm(g, [s.stream for s in g.streams]), enc, [s.text for s in g.streams],
                                             m["context"], temp=m["temp"], precision=m["precision"], topk=m["topk"])
    for s, b in zip(g.streams, bits):
        assert b == s.bits, f"{name} stream {s.stream}: decoded bits differ from the reference"


def test_code_base_single_stream_forms():
    """encode_arithmetic / decode_arithmetic / sample with the reference's signatures and return tuples."""
    from neuralsteganography_amd import code_base

    g = golden.load_compat("c1_toy_v700_repair")
    m = g.meta
    s = g.streams[1]
    enc = ToyTokenizer(m["vocab"])
    out = code_base.encode_arithmetic(_lm(g, [s.stream]), enc, s.msg, m["context"], temp=m["temp"],
                                      precision=m["precision"], topk=m["topk"])
    assert len(out) == 5 and out[0] == s.tokens
    bits = code_base.decode_arithmetic(_lm(g, [s.stream]), enc, s.text, m["context"], temp=m["temp"],
                                       precision=m["precision"], topk=m["topk"])
    assert bits == s.bits
    toks, nll, kl, hq = code_base.sample(_lm(g, [0]), enc, 10, m["context"], temperature=0.8, topk=50, seed=3)
    assert len(toks) == 10 and all(0 <= t < m["vocab"] for t in toks) and kl >= 0 and hq > 0
