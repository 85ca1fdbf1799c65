"""GPU: the sampler (code_base/sample.py) and the encode statistics (code_base/arithmetic.py:193-217).

Sampler: tokens bit-exact against the oracle's canonical sampler (same counter-based draws); statistics
within rel 1e-4 of the oracle's float64 restatement (fp32 streaming sums on the GPU) and of the reference
run's deterministic KL / entropy.  Encode statistics: within rel 2e-5 of the reference's returned values
(golden fixtures), tokens still bit-exact.
"""

from __future__ import annotations

import numpy as np
import pytest

from neuralsteganography_amd import synthetic
from oracle import oracle
from tests import golden

pytestmark = pytest.mark.gpu


def _logits_fn(seed, streams, vocab, scale, dtype, ld):
    import torch

    npdt = np.float16 if dtype == "f16" else np.float32

    def fn(t, _last=None):
        return torch.from_numpy(synthetic.logits_batch(seed, streams, t, vocab, scale, npdt, ld)).cuda()

    return fn


def _ctx(vocab, dtype, topk, B, precision=26, temp=0.9):
    from neuralsteganography_amd.coder import CoderContext, CoderParams

    return CoderContext(CoderParams(vocab=vocab, precision=precision, temp=temp,
                                    topk=topk if topk > 0 else vocab, dtype=dtype), max_batch=B)


@pytest.mark.parametrize("vocab,dtype,topk,temp,scale", [
    (50257, "f32", 300, 0.9, 3.0),     # single-pass kernel
    (50257, "f16", 100, 0.9, 3.0),
    (50257, "f32", 768, 1.2, 2.0),     # largest single-pass top-k
    (50257, "f32", 2000, 1.0, 3.0),    # wide path
    (50257, "f32", -1, 1.0, 3.0),      # every id (wide path; the reference cannot run topk <= 0)
    (700, "f32", 690, 0.7, 2.0),
])
def test_sampler_matches_oracle(vocab, dtype, topk, temp, scale):
    from neuralsteganography_amd.coder import row_stride, sample_batch

    B, L, seed, off = 5, 12, 0xC0FFEE, 3
    ctx = _ctx(vocab, dtype, topk, B, temp=temp)
    ld = row_stride(vocab, dtype)
    streams = list(range(B))
    toks, stats = sample_batch(ctx, B, L, _logits_fn(17, streams, vocab, scale, dtype, ld), seed=seed, topk=topk,
                               temp=temp, stream_offset=off)
    npdt = np.float16 if dtype == "f16" else np.float32
    banned = [vocab - 1, 628]
    for s in range(B):
        row = lambda t, s=s: synthetic.logits_row(17, s, t, vocab, scale, npdt).astype(np.float32)
        acc = np.zeros(4)
        ref, _ = oracle.sample_stream(row, L, banned=banned, temp=temp, topk=topk, seed=seed, gid=off + s, stats=acc)
        assert toks[s] == ref, f"stream {s}: sampled tokens differ from the oracle"
        want = oracle.stats_summary(acc)
        for k in ("avg_NLL", "avg_KL", "avg_Hq"):
            assert stats[s][k] == pytest.approx(want[k], rel=1e-4, abs=1e-5), (s, k)


@pytest.mark.parametrize("name", golden.sample_names())
def test_sampler_statistics_match_reference_run(name):
    """KL and entropy of sample() depend only on the rows: the kernel's equal the reference run's."""
    from neuralsteganography_amd.coder import row_stride, sample_batch

    g = golden.load_sample(name)
    m = g.meta
    B = len(g.streams)
    L = max(len(s.tokens) for s in g.streams)
    ctx = _ctx(m["vocab"], m["dtype"], m["topk"], B, temp=m["temp"])
    ld = row_stride(m["vocab"], m["dtype"])
    toks, stats = sample_batch(ctx, B, L, _logits_fn(m["logit_seed"], [s.stream for s in g.streams], m["vocab"],
                                                     m["scale"], m["dtype"], ld),
                               seed=1, topk=m["topk"], temp=m["temp"])
    rel = 1e-3 if m["dtype"] == "f16" else 1e-4
    for s in g.streams:
        if len(s.tokens) != L:
            continue
        assert stats[s.stream]["avg_KL"] == pytest.approx(s.stats[1], rel=rel, abs=rel / 10)
        assert stats[s.stream]["avg_Hq"] == pytest.approx(s.stats[2], rel=rel, abs=rel / 10)


def test_sampler_is_shardable_by_stream_offset():
    """Stream b of a batch with offset o draws exactly as stream o+b of a larger batch (multi-GPU sharding)."""
    from neuralsteganography_amd.coder import row_stride, sample_batch

    V, L = 50257, 6
    ld = row_stride(V, "f32")
    ctx = _ctx(V, "f32", 300, 6)
    full, _ = sample_batch(ctx, 6, L, _logits_fn(5, list(range(6)), V, 3.0, "f32", ld), seed=42, topk=300, temp=0.9)
    part, _ = sample_batch(ctx, 2, L, _logits_fn(5, [4, 5], V, 3.0, "f32", ld), seed=42, topk=300, temp=0.9,
                           stream_offset=4)
    assert part == full[4:6]


@pytest.mark.parametrize("name", [n for n in golden.names() if not n.endswith("_finish")])
def test_encode_statistics_match_reference(name):
    from neuralsteganography_amd.coder import CoderContext, CoderParams, encode_batch, row_stride

    g = golden.load(name)
    m = g.meta
    params = CoderParams(vocab=m["vocab"], precision=m["precision"], temp=m["temp"], topk=m["topk"],
                         dtype=m["dtype"], banned=m["banned"])
    B = len(g.streams)
    ctx = CoderContext(params, max_batch=B)
    ld = row_stride(m["vocab"], m["dtype"])
    fn = _logits_fn(m["logit_seed"], [s.stream for s in g.streams], m["vocab"], m["scale"], m["dtype"], ld)
    toks, stats = encode_batch(ctx, [s.msg for s in g.streams], fn, return_stats=True)
    for s, tk, st in zip(g.streams, toks, stats):
        assert tk == s.tokens
        ref = dict(zip(["avg_NLL", "avg_KL", "words_per_bit", "avg_Hq"], s.stats))
        for k, v in ref.items():
            assert st[k] == pytest.approx(v, rel=2e-5, abs=2e-6), (name, s.stream, k)
