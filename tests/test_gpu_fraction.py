"""GPU: the Fraction coder kernel (``ns_frac_encode_step`` / ``ns_frac_decode_step``, row a12) against the
reference's recorded outcomes (tests/golden/fraction_golden.json, produced by running its ``encode_bits`` /
``decode_bits``) and against the oracle restatement (``oracle/fraction_coder.py``, pinned by those outcomes) on
random batches: same tokens, same per-token consumption, same decoded bytes, same exception and message."""

import json
import random
from pathlib import Path

import numpy as np
import pytest

from oracle import fraction_coder as fc
from tests.golden.make_fraction_golden import dists

pytestmark = pytest.mark.gpu

G = json.loads((Path(__file__).resolve().parent / "golden" / "fraction_golden.json").read_text())


@pytest.fixture(scope="module")
def F():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from neuralsteganography_amd.codec import fraction

    return fraction


def _kind(exc):
    from neuralsteganography_amd.codec.errors import ArithmeticRangeError, DecodeDivergenceError

    if isinstance(exc, (fc.RangeError, ArithmeticRangeError)):
        return "range", str(exc)
    if isinstance(exc, (fc.DivergenceError, DecodeDivergenceError)):
        return "diverge", str(exc)
    return type(exc).__name__, str(exc)


def _oracle_encode(payload, ds):
    try:
        return fc.encode(payload, ds)
    except Exception as exc:  # noqa: BLE001 - the outcome under test
        return _kind(exc)


def _oracle_decode(toks, ds, state):
    try:
        return fc.decode(toks, ds, state)
    except Exception as exc:  # noqa: BLE001
        return _kind(exc)


@pytest.mark.parametrize("rec", G, ids=[f"{r['payload'] or 'empty'}-V{r['V']}{'-dict' if r['as_dict'] else ''}" for r in G])
def test_fraction_kernel_matches_reference_outcomes(F, rec):
    from neuralsteganography_amd.codec.errors import ArithmeticRangeError

    ds = dists(rec["V"], rec["seed"], as_dict=rec["as_dict"])
    payload = bytes.fromhex(rec["payload"])
    state = {}
    if "encode_error" in rec:
        with pytest.raises(ArithmeticRangeError):
            F.encode_bits(payload, iter(ds), state=state)
        return
    toks = F.encode_bits(payload, iter(ds), state=state)
    assert toks == rec["tokens"]
    assert list(state["history"]) == rec["history"]
    assert state["residual_bits"].hex() == rec["residual_bits"]
    assert F.decode_bits(toks, iter(ds), state=dict(state)).hex() == rec["decoded"]


def _random_dist(rng, V, as_dict):
    kind = rng.random()
    p = np.array([rng.random() for _ in range(V)])
    if kind < 0.2:
        p[rng.randrange(V)] = 0.0
    elif kind < 0.35:  # values below 2^-31: limit_denominator turns them into 0 or 2^-30
        p[rng.randrange(V)] = rng.choice([1e-12, 2.0 ** -31, 2.0 ** -31 * 1.0000001, 3e-10, 5e-324])
    elif kind < 0.45:  # unnormalised weights, integers and large values
        p = np.array([float(rng.randint(0, 9)) for _ in range(V)]) * rng.choice([1.0, 1e6, 2.0 ** 60])
        if not p.any():
            p[0] = 1.0
    elif kind < 0.55:  # short dyadic values (exact fractions, power-of-two denominators)
        p = np.array([rng.randint(1, 64) / 64 for _ in range(V)])
    if kind >= 0.55:
        p = p / p.sum()
    if as_dict:
        ids = rng.sample(range(5 * V + 7), V)
        return {int(i): float(v) for i, v in zip(ids, p)}
    return p


def test_fraction_kernel_batch_matches_oracle(F):
    rng = random.Random(5)
    payloads, streams = [], []
    for b in range(48):
        V = rng.choice([2, 3, 5, 16, 40, 130])
        as_dict = rng.random() < 0.3
        kind = rng.random()
        if kind < 0.45:
            payload = bytes(rng.choice([1, 2, 3, 6]))  # zeros: the payloads this coder can carry
        elif kind < 0.55:
            payload = b"\xff" * rng.choice([1, 2])
        elif kind < 0.6:
            payload = b""
        else:
            payload = bytes(rng.getrandbits(8) for _ in range(rng.choice([1, 2])))
        payloads.append(payload)
        streams.append([_random_dist(rng, V, as_dict) for _ in range(80)])
    states = [{} for _ in payloads]
    got = F.encode_bits_batch(payloads, [iter(s) for s in streams], states, return_exceptions=True)
    n_ok = 0
    dec_tok, dec_ds, dec_state, dec_want = [], [], [], []
    for payload, ds, st, g in zip(payloads, streams, states, got):
        want = _oracle_encode(payload, ds)
        if isinstance(want, tuple) and isinstance(want[0], str):
            assert isinstance(g, Exception) and _kind(g) == want, (payload, g, want)
            continue
        toks, wst = want
        assert g == toks and tuple(st["history"]) == tuple(wst["history"])
        assert st["residual_bits"] == wst["residual_bits"]
        n_ok += 1
        if toks:
            dec_tok.append(toks)
            dec_ds.append(ds)
            dec_state.append(dict(st))
            dec_want.append(_oracle_decode(toks, ds, dict(wst)))
    assert n_ok >= 15
    dec = F.decode_bits_batch(dec_tok, [iter(d) for d in dec_ds], dec_state, return_exceptions=True)
    for g, w in zip(dec, dec_want):
        if isinstance(w, tuple):
            assert isinstance(g, Exception) and _kind(g) == w
        else:
            assert g == w


def test_fraction_decode_arbitrary_tokens_matches_oracle(F):
    """Decode does not need an encodable payload: random tokens and consumption counts drive the interval and
    the prefix computation (ceil / floor divisions, the 'no prefix fits' and 'not present' branches)."""
    rng = random.Random(9)
    toks_l, ds_l, st_l, want = [], [], [], []
    for b in range(40):
        V = rng.choice([2, 4, 16, 64])
        as_dict = rng.random() < 0.3
        ds = [_random_dist(rng, V, as_dict) for _ in range(12)]
        T = rng.randint(1, 10)
        toks = []
        for t in range(T):
            keys = list(ds[t].keys()) if as_dict else list(range(V))
            toks.append(rng.choice(keys) if rng.random() < 0.95 else 10 ** 6)
        hist = tuple(rng.randint(0, 40) for _ in range(T))
        state = {"history": hist, "residual_bits": max(0, sum(hist) - rng.randint(0, 3) + (b % 5 == 0)).to_bytes(8, "big")}
        toks_l.append(toks)
        ds_l.append(ds)
        st_l.append(dict(state))
        want.append(_oracle_decode(toks, ds, dict(state)))
    got = F.decode_bits_batch(toks_l, [iter(d) for d in ds_l], st_l, return_exceptions=True)
    kinds = set()
    for g, w in zip(got, want):
        if isinstance(w, tuple):
            assert isinstance(g, Exception) and _kind(g) == w
            kinds.add(w[1].split()[0])
        else:
            assert g == w
            kinds.add("ok")
    assert "ok" in kinds and len(kinds) >= 2


def test_fraction_reference_error_behaviour(F):
    from neuralsteganography_amd.codec.errors import ArithmeticRangeError, DecodeDivergenceError

    with pytest.raises(ArithmeticRangeError, match="non-negative"):
        F.encode_bits(b"\x00", iter([np.array([0.5, -0.1, 0.6])]))
    with pytest.raises(ValueError):
        F.encode_bits(b"\x00", iter([np.array([0.5, np.nan])]))
    with pytest.raises(TypeError, match="Unsupported probability distribution type"):
        F.encode_bits(b"\x00", iter([[0.5, 0.5]]))
    with pytest.raises(ArithmeticRangeError, match="Insufficient probability distributions for encoding"):
        F.encode_bits(b"\x00\x00", iter([np.array([0.5, 0.5])]))
    with pytest.raises(ArithmeticRangeError, match="positive mass"):
        F.encode_bits(b"\x00", iter([np.zeros(3)]))
    with pytest.raises(ArithmeticRangeError, match="positive mass"):  # every value rounds to 0 / 1
        F.encode_bits(b"\x00", iter([np.array([1e-12, 2e-12])]))
    with pytest.raises(DecodeDivergenceError, match="history is required"):
        F.decode_bits([0], iter([np.array([0.5, 0.5])]), state={})
    st = {}
    assert F.encode_bits(b"", iter([]), state=st) == [] and st == {"history": (), "residual_bits": bytes(8)}
    assert F.decode_bits([], iter([])) == b""


def test_fraction_table_growth_and_capacity(F):
    """A 300-token step needs a cumulative table beyond the default 65,536 limbs (the lcm of 300 random 30-bit
    denominators): the step re-runs with a larger table and still matches the restatement; a tiny interval
    arena raises FractionCapacityError instead of writing past it."""
    rng = np.random.default_rng(4)
    p = rng.random(300)
    ds = [p / p.sum()]
    st = {}
    toks = F.encode_bits(b"\x00", iter(ds), state=st)
    want, wst = fc.encode(b"\x00", ds)
    assert toks == want and tuple(st["history"]) == tuple(wst["history"])
    assert F.decode_bits(toks, iter(ds), state=dict(st)) == b"\x00"
    with pytest.raises(F.FractionCapacityError):
        F.encode_bits_batch([bytes(8)], [iter(dists(16, 1016))], cap_limbs=8)


def test_fraction_table_growth_in_a_mixed_batch(F):
    """one stream's table re-run must not touch the others.  A batch mixing V = 300 rows (their
    steps re-run alone with a larger table, NS_FRAC_ERR_TABLE) and V = 16 rows (done in the first launch) gives
    every message the restatement's tokens, history and decoded bytes, over several steps."""
    rng = np.random.default_rng(11)
    payloads, streams = [], []
    for b in range(6):
        V = 300 if b in (1, 4) else 16
        rows = []
        for _ in range(40):
            p = rng.random(V)
            rows.append(p / p.sum())
        payloads.append(bytes(2))
        streams.append(rows)
    states = [{} for _ in payloads]
    got = F.encode_bits_batch(payloads, [iter(s) for s in streams], states, return_exceptions=True)
    for b, (payload, ds, st, g) in enumerate(zip(payloads, streams, states, got)):
        want = _oracle_encode(payload, ds)
        if isinstance(want, tuple) and isinstance(want[0], str):
            assert isinstance(g, Exception) and _kind(g) == want, (b, g, want)
            continue
        toks, wst = want
        assert g == toks, b
        assert tuple(st["history"]) == tuple(wst["history"]), b
    ok = [b for b, g in enumerate(got) if not isinstance(g, Exception)]
    assert {1, 4} & set(ok) and {0, 2} & set(ok)  # both kinds of stream really ran
    dec = F.decode_bits_batch([got[b] for b in ok], [iter(streams[b]) for b in ok], [dict(states[b]) for b in ok],
                              return_exceptions=True)
    for b, d in zip(ok, dec):
        assert d == payloads[b], b


def test_fraction_scratch_budget_splits_a_group_instead_of_failing_it(F, monkeypatch):
    """streams whose grown tables do not fit the scratch budget TOGETHER are launched in chunks
    that do (each fits alone), so every message still gets the restatement's tokens -- a message never fails because
    of what else is in its batch."""
    rng = np.random.default_rng(12)
    streams = [[(lambda p: p / p.sum())(rng.random(300)) for _ in range(12)] for _ in range(6)]
    payloads = [bytes([b]) for b in range(6)]  # every message encodes in the restatement (checked on the CPU)
    dv = F._Device(1, F.DEFAULT_CAP_LIMBS)
    one = int(dv.L.ns_frac_scratch_bytes(dv.ctx, 1, 300, 16, 8 * F.DEFAULT_TABLE_LIMBS))
    dv.close()
    assert one > 0
    monkeypatch.setattr(F, "SCRATCH_BUDGET_BYTES", one * 3 // 2)  # grown tables: one stream per launch
    got = F.encode_bits_batch(payloads, [iter(s) for s in streams], [{} for _ in payloads], return_exceptions=True)
    for b, (payload, ds, g) in enumerate(zip(payloads, streams, got)):
        want = _oracle_encode(payload, ds)
        if isinstance(want, tuple) and isinstance(want[0], str):
            assert isinstance(g, Exception) and _kind(g) == want, (b, g, want)
        else:
            assert g == want[0], b
    assert all(not isinstance(g, Exception) for g in got)  # before: all six failed with FractionCapacityError


def test_fraction_capacity_is_per_message(F):
    """an interval arena too small for one message's lcm (NS_FRAC_ERR_CAPACITY, which no table
    can cure) fails that message only, with FractionCapacityError, without growing any table."""
    rng = np.random.default_rng(3)
    big = [(lambda p: p / p.sum())(rng.random(3000)) for _ in range(2)]
    got = F.encode_bits_batch([b"\x00", b"\x00"], [iter(big), iter(dists(4, 1004))], [{}, {}], cap_limbs=64,
                              return_exceptions=True)
    assert isinstance(got[0], F.FractionCapacityError)
    assert got[1] == fc.encode(b"\x00", dists(4, 1004))[0]


def test_fraction_payload_bound(F):
    """Payloads beyond the device coder's bound raise FractionCapacityError for that message only."""
    got = F.encode_bits_batch([bytes(F.MAX_PAYLOAD_BITS // 8 + 1), b"\x00"],
                              [iter(dists(4, 1004)), iter(dists(4, 1004))], [{}, {}], return_exceptions=True)
    assert isinstance(got[0], F.FractionCapacityError)
    assert got[1] == fc.encode(b"\x00", dists(4, 1004))[0]
