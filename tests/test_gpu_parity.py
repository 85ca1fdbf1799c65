"""GPU parity: the HIP coder (through the C ABI) against the reference's golden vectors and the CPU oracle.

Bar: bit-exact tokens, bit-exact decoded bits, and identical per-step (k, k', sel, token) traces.
"""

from __future__ import annotations

import numpy as np
import pytest

from neuralsteganography_amd import synthetic
from neuralsteganography_amd.codec.errors import DecodeDivergenceError
from neuralsteganography_amd.exceptions import ConfigurationError
from oracle import oracle
from tests import golden

pytestmark = pytest.mark.gpu

KERNEL_GOLDEN = ["g1_v50257_f32_p26_k300", "g2_v50257_f16_p26_k100", "g3_v50257_f32_peaked_p26_k300",
                 "g4_v50257_f32_p16_k50000", "g5_v50257_f32_p40_k60000",  # wide (large top-k) path
                 "g6_v700_f32_p20_k500", "g7_v640_f32_p12_k1000",
                 "g8_v50257_f32_p26_k300_finish"]  # finish_sent=True


def _torch():
    import torch

    return torch


@pytest.fixture(autouse=True, params=["wave", "split"])
def coder_form(request):
    """Every test runs with both single-pass coder forms: one wave per stream, and the small-batch split form
    (one workgroup per stream, wave 0 merges) forced at every batch size."""
    from neuralsteganography_amd import _lib

    prev = _lib.set_split_max_batch(0 if request.param == "wave" else 1 << 30)
    yield request.param
    _lib.set_split_max_batch(prev)


def _ctx(params, B):
    from neuralsteganography_amd.coder import CoderContext

    return CoderContext(params, max_batch=B)


def _logits_fn(seed, streams, vocab, scale, dtype, ld):
    torch = _torch()
    npdt = np.float16 if dtype == "f16" else np.float32

    def fn(t, _last=None):
        arr = synthetic.logits_batch(seed, streams, t, vocab, scale, npdt, ld)
        return torch.from_numpy(arr).cuda()

    return fn


def _params_from_meta(m):
    from neuralsteganography_amd.coder import CoderParams

    return CoderParams(vocab=m["vocab"], precision=m["precision"], temp=m["temp"], topk=m["topk"],
                       dtype=m["dtype"], banned=m["banned"])


@pytest.mark.parametrize("force_exact", [False, True])
@pytest.mark.parametrize("name", KERNEL_GOLDEN)
def test_kernel_matches_reference_golden(name, force_exact):
    from neuralsteganography_amd.coder import decode_batch, encode_batch, row_stride

    g = golden.load(name)
    m = g.meta
    params = _params_from_meta(m)
    B = len(g.streams)
    ctx = _ctx(params, B)
    ld = row_stride(m["vocab"], m["dtype"])
    fn = _logits_fn(m["logit_seed"], [s.stream for s in g.streams], m["vocab"], m["scale"], m["dtype"], ld)
    if g.finish_sent:
        ctx.set_sentence_end(g.sent_end_table())
    toks = encode_batch(ctx, [s.msg for s in g.streams], fn, force_exact=force_exact, finish_sent=g.finish_sent)
    for s, tk in zip(g.streams, toks):
        assert tk == s.tokens, f"{name} stream {s.stream}: HIP tokens differ from the reference"
    bits = decode_batch(ctx, [s.tokens for s in g.streams], fn, force_exact=force_exact)
    for s, bt in zip(g.streams, bits):
        assert bt == s.bits, f"{name} stream {s.stream}: HIP decoded bits differ from the reference"


def test_wide_path_is_selected_beyond_single_pass_limit():
    from neuralsteganography_amd import _lib
    from neuralsteganography_amd.coder import CoderParams

    ctx = _ctx(CoderParams(vocab=50257, precision=16, topk=50000), 2)
    assert ctx.wide and ctx.K == 50000 > _lib.max_topk(_lib.NS_DTYPE_F32)
    assert not _ctx(CoderParams(vocab=50257, precision=26, topk=300), 2).wide


def _oracle_step_traces(seed, stream, bits, params, scale, nsteps_cap=None):
    row = lambda t: synthetic.logits_row(seed, stream, t, params.vocab, scale,
                                         np.float16 if params.dtype == "f16" else np.float32).astype(np.float32)
    toks, tr = oracle.encode_stream(row, bits, banned=params.banned_ids(), temp=params.temp,
                                    precision=params.precision, topk=params.topk)
    return toks, [(t.k, t.kprime, t.sel, t.n, t.token) for t in tr]


@pytest.mark.parametrize("dtype,scale,temp,precision,topk", [
    ("f32", 3.0, 0.9, 26, 300),
    ("f16", 3.0, 0.9, 26, 100),
    ("f32", 12.0, 1.0, 26, 300),   # peaked: the 1/R cutoff binds
    ("f32", 3.0, 1.0, 30, 768),    # the kernel's largest fp32 top-k
    ("f16", 1.0, 1.5, 20, 512),    # the kernel's largest fp16 top-k, flat rows
    ("f32", 0.05, 1.0, 26, 300),   # nearly uniform rows
    ("f32", 3.0, 1.0, 16, 50000),  # wide path: api defaults (precision 16, topk 50000)
    ("f16", 6.0, 0.9, 22, 2000),   # wide path, fp16, peaked: the cutoff binds inside the collected prefix
    ("f32", 3.0, 0.9, 40, 60000),  # wide path, message->bits mode (run_single.py:52-54)
])
def test_stepwise_traces_match_oracle(dtype, scale, temp, precision, topk):
    from neuralsteganography_amd.coder import CoderParams, EncodeSession, row_stride

    V, B, seed = 50257, 6, 11
    params = CoderParams(vocab=V, precision=precision, temp=temp, topk=topk, dtype=dtype)
    force = topk > 768  # the wide path also runs its exact-sum branch every other step
    ctx = _ctx(params, B)
    ld = row_stride(V, dtype)
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 12))[: 96 - 7 * s] for s in range(B)]
    expect = [_oracle_step_traces(seed, s, bits[s], params, scale) for s in range(B)]
    sess = EncodeSession(ctx, bits)
    sess.enable_trace()
    fn = _logits_fn(seed, list(range(B)), V, scale, dtype, ld)
    nmax = max(len(e[0]) for e in expect)
    for t in range(nmax):
        sess.step(fn(t), force_exact=force and t % 2 == 1)
        tr = sess.trace_rows()
        for s in range(B):
            if t < len(expect[s][1]):
                got = (int(tr.k[s]), int(tr.kprime[s]), int(tr.sel[s]), int(tr.n[s]), int(tr.token[s]))
                assert got == expect[s][1][t], f"stream {s} step {t}: kernel {got} oracle {expect[s][1][t]}"
    assert sess.all_done()
    assert sess.tokens() == [e[0] for e in expect]


@pytest.mark.parametrize("dtype,precision,topk", [
    ("f32", 26, 300),      # single-pass kernel
    ("f16", 26, 100),
    ("f32", 16, 50000),    # wide path
])
def test_finish_sent_matches_oracle(dtype, precision, topk):
    """finish_sent (code_base/arithmetic.py:114,134-137): after the payload, top-1 tokens until one is
    sentence-ending; ragged payloads so streams sit in different phases of the same launch."""
    from neuralsteganography_amd.coder import CoderParams, encode_batch, row_stride

    V, B, seed, scale = 50257, 5, 23, 3.0
    params = CoderParams(vocab=V, precision=precision, temp=0.9, topk=topk, dtype=dtype)
    ctx = _ctx(params, B)
    table = (np.arange(V) % 211 == 17).astype(np.uint8)   # sparse: long top-1 tails
    ctx.set_sentence_end(table)
    ld = row_stride(V, dtype)
    npdt = np.float16 if dtype == "f16" else np.float32
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 8))[: [64, 1, 0, 33, 7][s]] for s in range(B)]
    toks = encode_batch(ctx, bits, _logits_fn(seed, list(range(B)), V, scale, dtype, ld), finish_sent=True,
                        check_every=8)
    for s in range(B):
        row = lambda t, s=s: synthetic.logits_row(seed, s, t, V, scale, npdt).astype(np.float32)
        ref, _ = oracle.encode_stream(row, bits[s], banned=params.banned_ids(), temp=0.9, precision=precision,
                                      topk=topk, sent_end=table)
        assert toks[s] == ref, f"stream {s}: finish_sent tokens differ from the oracle"
        assert table[toks[s][-1]], f"stream {s}: the finish tail must end on a sentence-ending token"


def test_finish_sent_needs_table():
    from neuralsteganography_amd.coder import CoderParams, encode_batch, row_stride

    V = 50257
    ctx = _ctx(CoderParams(vocab=V, precision=26, temp=0.9, topk=300), 2)
    fn = _logits_fn(1, [0, 1], V, 3.0, "f32", row_stride(V, "f32"))
    with pytest.raises(ConfigurationError):
        encode_batch(ctx, [[1, 0], [1]], fn, finish_sent=True)


def test_roundtrip_large_batch_properties():
    """B=1024 streams x 64-byte payloads: decode(encode(x)) == x, the size-independent property."""
    from neuralsteganography_amd.coder import CoderParams, decode_batch, encode_batch, row_stride

    torch = _torch()
    V, B = 50257, 1024
    params = CoderParams(vocab=V, precision=26, temp=0.9, topk=300)
    ctx = _ctx(params, B)
    ld = row_stride(V, "f32")
    gen = torch.Generator(device="cuda")
    pool = []
    for i in range(8):
        gen.manual_seed(100 + i)
        pool.append(3.0 * torch.randn((B, ld), generator=gen, device="cuda", dtype=torch.float32))
    fn = lambda t, _l=None: pool[t % len(pool)]
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 64)) for s in range(B)]
    toks = encode_batch(ctx, bits, fn)
    out = decode_batch(ctx, toks, fn)
    for s in range(B):
        assert out[s][: len(bits[s])] == bits[s], f"stream {s} round trip failed"
    # spot-check a few streams against the oracle on the same rows
    pool_h = [p.cpu().numpy() for p in pool]
    for s in (0, 517, 1023):
        otoks, _ = oracle.encode_stream(lambda t: pool_h[t % len(pool_h)][s, :V], bits[s],
                                        banned=params.banned_ids(), temp=params.temp,
                                        precision=params.precision, topk=params.topk)
        assert otoks == toks[s]


def test_decode_divergence_is_reported():
    from neuralsteganography_amd.coder import CoderParams, decode_batch, row_stride

    V = 50257
    params = CoderParams(vocab=V, precision=26, temp=0.9, topk=300)
    ctx = _ctx(params, 2)
    fn = _logits_fn(5, [0, 1], V, 3.0, "f32", row_stride(V, "f32"))
    with pytest.raises(DecodeDivergenceError):
        decode_batch(ctx, [[628, 1, 2], [V - 1]], fn)  # banned ids can never be decoded


@pytest.mark.parametrize("topk", [300, 50000])  # single-pass kernel, wide path
@pytest.mark.parametrize("poison", ["nan", "inf"])
def test_non_finite_logits_are_reported(topk, poison):
    """A NaN row (what the attention kernel writes when a device-side cache length is out of range) or a +inf
    logit must surface as a range error, never as a token from a meaningless CDF."""
    from neuralsteganography_amd.codec.errors import ArithmeticRangeError
    from neuralsteganography_amd.coder import CoderParams, encode_batch, row_stride

    torch = _torch()
    V = 50257
    params = CoderParams(vocab=V, precision=16 if topk > 1000 else 26, temp=1.0, topk=topk)
    ctx = _ctx(params, 2)
    good = _logits_fn(3, [0, 1], V, 3.0, "f32", row_stride(V, "f32"))

    def fn(t, _last=None):
        x = good(t)
        if poison == "nan":
            x[1].fill_(float("nan"))
        else:
            x[1, 17] = float("inf")
        return x

    with pytest.raises(ArithmeticRangeError):
        encode_batch(ctx, [[1, 0, 1, 1] * 8, [0, 1, 1, 0] * 8], fn)
    torch.cuda.synchronize()


@pytest.mark.parametrize("dtype,topk,nfinite", [("f32", 300, 150), ("f32", 300, 2), ("f16", 100, 40),
                                                ("f32", 50000, 3000)])
def test_masked_rows_match_oracle(dtype, topk, nfinite):
    """Rows with fewer than topk finite logits (the rest -inf: a caller's mask, or the reference's -1e10 ban
    overflowing fp16): the -inf ids are ranks of probability 0, so tokens, traces and bits follow the oracle
    instead of reporting a range error.  NaN rows still do (test above)."""
    from neuralsteganography_amd.coder import CoderParams, EncodeSession, decode_batch, row_stride

    torch = _torch()
    V, B, seed = 50257, 3, 29
    npdt = np.float16 if dtype == "f16" else np.float32
    precision = 16 if topk > 1000 else 26
    params = CoderParams(vocab=V, precision=precision, temp=0.9, topk=topk, dtype=dtype)
    ctx = _ctx(params, B)
    ld = row_stride(V, dtype)

    def row(s, t):
        x = synthetic.logits_row(seed, s, t, V, 3.0, npdt).astype(np.float32)
        keep = np.random.default_rng([seed, s, t]).choice(V, size=nfinite + 7 * s, replace=False)
        out = np.full(V, -np.inf, np.float32)
        out[keep] = x[keep]
        return out

    def fn(t, _last=None):
        a = np.zeros((B, ld), npdt)
        for s in range(B):
            a[s, :V] = row(s, t)
        return torch.from_numpy(a).cuda()

    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 6))[: 48 - 5 * s] for s in range(B)]
    expect = []
    for s in range(B):
        toks, tr = oracle.encode_stream(lambda t, s=s: row(s, t), bits[s], banned=params.banned_ids(), temp=0.9,
                                        precision=precision, topk=topk)
        expect.append((toks, [(x.k, x.kprime, x.sel, x.n, x.token) for x in tr]))
    # two finite ids carry at most one bit per token: more tokens than the default history (2 x bits + 64)
    sess = EncodeSession(ctx, bits, max_tokens=max(len(e[0]) for e in expect) + 8)
    sess.enable_trace()
    for t in range(max(len(e[0]) for e in expect)):
        sess.step(fn(t))
        tr = sess.trace_rows()
        for s in range(B):
            if t < len(expect[s][1]):
                got = (int(tr.k[s]), int(tr.kprime[s]), int(tr.sel[s]), int(tr.n[s]), int(tr.token[s]))
                assert got == expect[s][1][t], f"stream {s} step {t}: kernel {got} oracle {expect[s][1][t]}"
    toks = sess.tokens()
    assert toks == [e[0] for e in expect]
    out = decode_batch(ctx, toks, fn)
    for s in range(B):
        assert out[s][: len(bits[s])] == bits[s]


def test_empty_and_single_bit_payloads():
    from neuralsteganography_amd.coder import CoderParams, decode_batch, encode_batch, row_stride

    V = 50257
    params = CoderParams(vocab=V, precision=26, temp=0.9, topk=300)
    ctx = _ctx(params, 3)
    fn = _logits_fn(9, [0, 1, 2], V, 3.0, "f32", row_stride(V, "f32"))
    bits = [[], [1], [0, 1, 1]]
    toks = encode_batch(ctx, bits, fn)
    assert toks[0] == []
    for s in (1, 2):
        otoks, _ = oracle.encode_stream(lambda t, s=s: synthetic.logits_row(9, s, t, V), bits[s],
                                        banned=params.banned_ids(), temp=0.9, precision=26, topk=300)
        assert toks[s] == otoks
    out = decode_batch(ctx, toks[1:], _logits_fn(9, [1, 2], V, 3.0, "f32", row_stride(V, "f32")))
    assert out[0][:1] == [1] and out[1][:3] == [0, 1, 1]


def _sample_ids(V, W=4):
    """Ids of the kernel's sample tiles (nsg_coder.hip, NSG_SAMPLE 64): 4,096 ids as whole 64*W-id tiles,
    tile s*space + space-1 for s < NSAMP, space = ntiles // NSAMP."""
    ts = 64 * W
    nsamp = 4096 // ts
    ntiles = (V + ts - 1) // ts
    space = ntiles // nsamp
    ids = []
    for s in range(nsamp):
        t = s * space + space - 1
        ids.extend(range(t * ts, min((t + 1) * ts, V)))
    return np.asarray(ids)


@pytest.mark.parametrize("mode", ["miss", "overflow", "ties", "outlier"])
def test_adversarial_rows_exercise_fallback_paths(mode):
    """Rows whose stratified sample is unrepresentative: 'miss' makes the speculative threshold too high
    (the wave must re-read its row), 'overflow' makes it far too low (many compactions).  'ties' quantises
    the logits to a few values (the histogram select falls back to bisection and the bucket rank to full
    counting); 'outlier' puts one huge logit in the row every other step (all other keys crowd into one
    bucket).  Tokens must still match the oracle exactly."""
    from neuralsteganography_amd.coder import CoderParams, EncodeSession, row_stride

    torch = _torch()
    V, B = 50257, 4
    params = CoderParams(vocab=V, precision=26, temp=0.9, topk=300)
    ctx = _ctx(params, B)
    ld = row_stride(V, "f32")
    samp = _sample_ids(V)

    def row(s, t):
        x = synthetic.logits_row(77, s, t, V, 1.0)
        if mode == "miss":
            x[samp] += 12.0
        elif mode == "overflow":
            x[samp] -= 12.0
        elif mode == "ties":
            x = np.round(x * 2.0) / 2.0
        elif t % 2 == 0:
            x[(97 * t + 13 * s) % (V - 2)] = 3.0e30
        return x.astype(np.float32)

    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 8)) for s in range(B)]
    expect = [oracle.encode_stream(lambda t, s=s: row(s, t), bits[s], banned=params.banned_ids(), temp=0.9,
                                   precision=26, topk=300)[0] for s in range(B)]
    sess = EncodeSession(ctx, bits)
    c0 = ctx.counters()
    for t in range(max(map(len, expect))):
        arr = np.zeros((B, ld), np.float32)
        for s in range(B):
            arr[s, :V] = row(s, t)
        sess.step(torch.from_numpy(arr).cuda())
    c1 = ctx.counters()
    assert sess.tokens() == expect
    if mode == "miss":
        assert c1[2] > c0[2], "speculation miss path was not exercised"
    elif mode == "overflow":
        assert c1[1] > c0[1], "overflow compaction path was not exercised"
    else:
        assert c1[3] > c0[3], "slow top-K selection path was not exercised"


def test_sample_tie_rows_admit_smaller_ids():
    """The sample tiles are offered before the stream.  Rows with one top value, held by half of the sample
    tiles' ids and 3 % of the others: the sample alone overflows the candidate buffer, and the compaction's K-th
    key then sits in a sample tile while the stream's EARLIER tiles hold ids of the same value with smaller ids
    -- they rank above it and must still be admitted (a strict x > K-th-value rule drops them).  Token by token against the oracle for a fixed number of
    steps (the reference's interval can stall at the midpoint on such flat rows, so runs are not taken to
    completion)."""
    from neuralsteganography_amd.coder import CoderParams, EncodeSession, row_stride

    torch = _torch()
    V, B, T = 50257, 4, 12
    params = CoderParams(vocab=V, precision=26, temp=0.9, topk=300)
    ctx = _ctx(params, B)
    ld = row_stride(V, "f32")
    samp = _sample_ids(V)

    def row(s, t):  # one top value: the top-K is the K smallest ids holding it
        u = np.random.default_rng([77, s, t]).random(V)
        x = np.where(u < 0.03, 2.0, 0.0)
        x[samp] = np.where(u[samp] < 0.5, 2.0, 0.0)
        return x.astype(np.float32)

    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 8)) for s in range(B)]
    expect = []
    for s in range(B):
        packed = np.packbits(np.asarray(bits[s], dtype=np.uint8), bitorder="little")
        st = oracle.new_state(26)
        toks = []
        for t in range(T):
            if st.bit_pos >= len(bits[s]):
                break
            rc, tok, _ = oracle.encode_step(row(s, t), st, packed, len(bits[s]), banned=params.banned_ids(),
                                            temp=0.9, precision=26, topk=300)
            assert rc == oracle.OR_OK
            toks.append(tok)
        expect.append(toks)
    sess = EncodeSession(ctx, bits)
    c0 = ctx.counters()
    for t in range(T):
        arr = np.zeros((B, ld), np.float32)
        for s in range(B):
            arr[s, :V] = row(s, t)
        sess.step(torch.from_numpy(arr).cuda())
    c1 = ctx.counters()
    assert sess.tokens() == expect
    assert c1[1] > c0[1], "overflow compaction path was not exercised"


@pytest.mark.parametrize("mode,dtype", [("plain", "f32"), ("ties", "f32"), ("outlier", "f32"), ("mixed", "f32"),
                                        ("ties", "f16"), ("mixed", "f16")])
def test_wide_lds_path_matches_oracle(mode, dtype):
    """The wide path's LDS sort (streams with <= 8,192 collected keys, api defaults precision 16 / topk 50,000):
    'plain' rows keep 2-5k keys (counting sort + in-bucket ranks), 'ties' quantises the logits so a few values
    hold thousands of keys each (over-full buckets -> bitonic sort), 'outlier' leaves the top two keys only (every other step),
    'mixed' puts streams of all three kinds and a flat row (> 8,192 keys: the device-wide sort) in one batch.
    Tokens must match the oracle and decode back to the payload."""
    from neuralsteganography_amd.coder import CoderParams, decode_batch, encode_batch, row_stride

    torch = _torch()
    V, B = 50257, 4
    params = CoderParams(vocab=V, precision=16, temp=1.0, topk=50000, dtype=dtype)
    ctx = _ctx(params, B)
    assert ctx.wide
    ld = row_stride(V, dtype)
    npdt = np.float16 if dtype == "f16" else np.float32
    kinds = {"plain": ["plain"] * B, "ties": ["ties"] * B, "outlier": ["outlier"] * B,
             "mixed": ["plain", "ties", "outlier", "flat"]}[mode]

    def row(s, t):
        kind = kinds[s]
        x = synthetic.logits_row(91, s, t, V, 0.5 if kind == "flat" else 3.0)
        if kind == "ties":
            x = np.round(x * 2.0) / 2.0
        elif kind == "outlier" and t % 2 == 0:  # (every step would carry no bits at all)
            x[(97 * t + 13 * s) % (V - 2)] = 6.0e4 if dtype == "f16" else 3.0e30
        return x.astype(npdt)

    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 6)) for s in range(B)]
    expect = [oracle.encode_stream(lambda t, s=s: row(s, t), bits[s], banned=params.banned_ids(), temp=1.0,
                                   precision=16, topk=50000)[0] for s in range(B)]

    def fn(t, _last=None):
        arr = np.zeros((B, ld), npdt)
        for s in range(B):
            arr[s, :V] = row(s, t)
        return torch.from_numpy(arr).cuda()

    c0 = ctx.counters()
    toks = encode_batch(ctx, bits, fn)
    assert toks == expect
    if "ties" in kinds:
        assert ctx.counters()[3] > c0[3], "the bitonic fallback of the LDS sort was not exercised"
    got = decode_batch(ctx, toks, fn)
    for s in range(B):
        assert got[s][: len(bits[s])] == bits[s]


def test_wide_list_kernel_grid_stride_over_many_streams():
    """More streams handed to the list kernel than it has workgroups (256): every step forces the exact row sum
    (so every stream is listed), and half the rows are flat enough to overflow
    the LDS path (device-wide sort).  Tokens must match the oracle for every stream."""
    from neuralsteganography_amd.coder import CoderParams, decode_batch, encode_batch, row_stride

    V, B = 50257, 258
    params = CoderParams(vocab=V, precision=16, temp=1.0, topk=50000)
    ctx = _ctx(params, B)
    ld = row_stride(V, "f32")
    seed = 23
    scales = [0.5 if s % 2 else 3.0 for s in range(B)]
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 2)) for s in range(B)]
    expect = [oracle.encode_stream(lambda t, s=s: synthetic.logits_row(seed, s, t, V, scales[s]), bits[s],
                                   banned=params.banned_ids(), temp=1.0, precision=16, topk=50000)[0]
              for s in range(B)]
    torch = _torch()

    def fn(t, _last=None):
        arr = np.zeros((B, ld), np.float32)
        for s in range(B):
            arr[s, :V] = synthetic.logits_row(seed, s, t, V, scales[s])
        return torch.from_numpy(arr).cuda()

    c0 = ctx.counters()
    toks = encode_batch(ctx, bits, fn, force_exact=True)
    assert toks == expect
    assert ctx.counters()[0] - c0[0] >= B, "the exact-sum path did not run for every stream"
    got = decode_batch(ctx, toks, fn)
    for s in range(B):
        assert got[s][: len(bits[s])] == bits[s]
