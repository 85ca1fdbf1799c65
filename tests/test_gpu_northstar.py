"""GPU: round trips at the north-star configurations (BASELINE.json ``configs``).

The north star asks for 100 % bit-exact payload recovery at batch 4096 with emitted tokens bit-exact against
the CPU reference on identical logits.  These tests run the product path (batched GPT-2 decode step on the HIP
kernels, hipGraph-replayed token loop, HIP coder) at the stated sizes:

* C3: GPT-2-small (random-init, fp16 compute and logits), B = 4096 streams x 1 KiB payloads, encode -> decode,
  every stream's payload recovered bit for bit; a sample of streams is re-run alone on the eager loop with every
  step's logits captured, which must give the same tokens (the decode step is batch-invariant) and which the
  CPU oracle (``oracle/nsg_oracle.c``, pinned by the reference's own outputs) replays token for token.
* C4: the same at the gpt2-fa geometry (V = 42,001): one GPU's 4,096-stream share of C4's 32,768.
* C2: GPT-2-small, B = 1, 1 KiB: every step's logits captured, oracle replay of the whole stream, graph-replayed
  loop equal to the eager loop, decode round trip.
* C5-like: GPT-2-medium fp16, topk 100, temp 0.9, finish_sent, quality guard ON (the api's default guard, the
  regeneration schedule of ``api.py:496-523``) over 1024 secrets in one ``cover_generate_batch``; every secret
  either passes and is revealed from its cover TEXT, or is rejected after the whole schedule.  Payloads are
  short (the guard's unigram perplexity grows with the cover length), not C5's coder parameters.
"""

import time

import numpy as np
import pytest
import torch

from neuralsteganography_amd import synthetic
from oracle import oracle

pytestmark = pytest.mark.gpu

Q_C3 = {"temp": 0.9, "precision": 26, "topk": 300}  # run_single.py:21-24


def _record_eager(lm, bit_lists, context, quality):
    """encode_batch on the eager loop (all messages in their own slots from the start, no compaction, so row j is
    message j throughout) with every step's logits copied to the host (fp32 view of the f16 rows)."""
    seen = []
    orig_static, orig_prefill = lm.lm.step_static, lm.lm.prefill

    def rec_prefill(*a, **k):
        out = orig_prefill(*a, **k)
        seen.append(out[:, : lm.vocab].float().cpu().numpy())
        return out

    def rec_static(tok):
        out = orig_static(tok)
        seen.append(out[:, : lm.vocab].float().cpu().numpy())
        return out

    lm.lm.prefill, lm.lm.step_static = rec_prefill, rec_static
    lm.slot_compaction = False
    try:
        toks = lm.encode_batch(bit_lists, context, quality=quality, graphs=False)
    finally:
        lm.lm.prefill, lm.lm.step_static = orig_prefill, orig_static
        lm.slot_compaction = True
    return toks, seen


def _oracle_replay(seen, s, bits, V, quality, traces=False):
    o, tr = oracle.encode_stream(lambda t: seen[t][s], bits, banned=[V - 1, 628], temp=quality["temp"],
                                 precision=quality["precision"], topk=quality["topk"])
    return (o, tr) if traces else o


def _free_cache(lm):
    lm.lm.release_cache()
    torch.cuda.empty_cache()


def _b4096_roundtrip(name, label, *, B=4096, nbytes=1024, quality=Q_C3, logit_scale=1.0, sample=None):
    """B streams (default 4096) x nbytes encoded on the hipGraph-replayed product loop, decoded, every payload
    recovered; three streams re-run alone (eager, logits captured) must give the same tokens, which the oracle
    replays.  Returns (tokens, the oracle's per-step traces of the sampled streams)."""
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    m = random_gpt2(name, seed=1234)
    lm = HipArithmeticLM(m, None, logits_dtype="f16", max_batch=B, logit_scale=logit_scale)
    # [<|endoftext|>] + 31 ids; the end-of-text id is the vocabulary's last (gpt2-fa: 42,000)
    ctx = [lm.vocab - 1] + list(synthetic.DEFAULT_CONTEXT[1:])
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, nbytes)) for s in range(B)]
    t0 = time.perf_counter()
    toks = lm.encode_batch(bits, ctx, quality=quality)
    t1 = time.perf_counter()
    print(f"{label} encode done: {t1 - t0:.1f} s, schedule {lm.last_schedule}", flush=True)
    _free_cache(lm)
    out = lm.decode_batch(toks, ctx, quality=quality)
    t2 = time.perf_counter()
    bad = [s for s in range(B) if out[s][: len(bits[s])] != bits[s]]
    assert not bad, f"{label}: {len(bad)} of {B} streams did not round-trip (first: {bad[:8]})"
    ntok = sum(map(len, toks))
    print(f"{label} round trip: V={lm.vocab}, {B} x {nbytes} B, {ntok} tokens ({8 * nbytes * B / ntok:.2f} bits/token), "
          f"encode {t1 - t0:.1f} s, decode {t2 - t1:.1f} s", flush=True)
    _free_cache(lm)
    # oracle replay: a sample of streams alone, eager, logits captured (batch-invariant step => same logits)
    sample = sample or [0, B // 2 - 271, B - 1]
    sub, seen = _record_eager(lm, [bits[s] for s in sample], ctx, quality)
    traces = []
    for j, s in enumerate(sample):
        assert sub[j] == toks[s], f"{label} stream {s}: alone (eager) != inside the B={B} graph-replayed batch"
        o, tr = _oracle_replay(seen, j, bits[s], lm.vocab, quality, traces=True)
        assert o == toks[s], f"{label} stream {s}: HIP coder != oracle"
        traces.append(tr)
    _free_cache(lm)
    return toks, traces


@pytest.mark.timeout(900)
def test_c3_gpt2_small_b4096_1kib_roundtrip_bit_exact():
    _b4096_roundtrip("gpt2", "C3")


@pytest.mark.timeout(900)
def test_c4_gpt2_fa_b4096_share_1kib_roundtrip_bit_exact():
    """C4 = gpt2-fa, 32,768 streams over 8 GPUs: one GPU's share (4,096 streams) at the gpt2-fa geometry
    (GPT-2-small layers, V = 42,001, end-of-text 42,000 banned with 628; random-init weights, no checkpoint
    offline) -- encode -> decode with every payload recovered, and the oracle replay."""
    _b4096_roundtrip("gpt2-fa", "C4")


@pytest.mark.timeout(900)
def test_c5_gpt2_medium_topk100_b1024_1kib_roundtrip_bit_exact():
    """C5's coder parameters: GPT-2-medium (random-init, fp16), topk 100, temp 0.9, precision 26,
    one GPU's 1,024-stream share of C5's 8,192, 1 KiB payloads -- encode -> decode with every payload recovered and a
    3-stream oracle replay (quality guard off: the guard-on path is the next test)."""
    _b4096_roundtrip("gpt2-medium", "C5", B=1024, quality={"temp": 0.9, "precision": 26, "topk": 100})


@pytest.mark.timeout(1100)
def test_trained_entropy_rows_b4096_roundtrip_and_cutoff_path():
    """random-init GPT-2 rows are near-uniform (~8.1 bits/token, k = topk every step).  With
    the head scaled (logit_scale 6: ~4.2 bits/token measured, tools/trained_probe.py) the rows peak like a trained
    LM's, so covers are longer and uneven in length, and the 1/R cutoff (code_base/arithmetic.py:140-165) binds on
    some steps (k < topk in the oracle's traces).  C3's geometry, 4,096 streams x 1 KiB: round trip + 3-stream oracle
    replay.  The paged KV cache holds live tokens only (a finished stream's pages go back to the pool; the youngest
    streams are re-queued if the device fills), so the long tail of a few low-entropy covers no longer multiplies
    by B -- the dense lockstep cache of round 5 ran out of memory here."""
    toks, traces = _b4096_roundtrip("gpt2", "trained-entropy", B=4096, nbytes=1024, logit_scale=6.0)
    bpt = 8 * 1024 * len(toks) / sum(map(len, toks))
    assert 2.5 < bpt < 6.0, bpt
    ks = [t.k for tr in traces for t in tr]
    assert min(ks) < Q_C3["topk"], "the 1/R cutoff never bound"


@pytest.mark.timeout(600)
def test_c2_gpt2_small_b1_1kib_oracle_replay_every_step():
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    m = random_gpt2("gpt2", seed=1234)
    lm = HipArithmeticLM(m, None, logits_dtype="f16", max_batch=1)
    ctx = synthetic.DEFAULT_CONTEXT
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(7, 1024))]
    toks_e, seen = _record_eager(lm, bits, ctx, Q_C3)
    assert len(seen) >= len(toks_e[0])  # prefill + one logits row per later token (+ steps up to the done check)
    assert _oracle_replay(seen, 0, bits[0], lm.vocab, Q_C3) == toks_e[0]
    toks_g = lm.encode_batch(bits, ctx, quality=Q_C3)  # the hipGraph-replayed product loop
    assert toks_g == toks_e
    for graphs in (True, False):
        out = lm.decode_batch(toks_g, ctx, quality=Q_C3, graphs=graphs)
        assert out[0][: len(bits[0])] == bits[0]


_IdTokenizer = synthetic.IdTokenizer


@pytest.mark.timeout(900)
def test_c5_like_gpt2_medium_topk100_guard_on_1024_secrets():
    from neuralsteganography_amd.cover import (_ensure_guard, cover_generate_batch, cover_reveal_batch,
                                               iter_attempts, prepare_gate_thresholds)
    from neuralsteganography_amd.stego import normalise_quality
    from neuralsteganography_amd.exceptions import QualityGateError
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    n = 1024
    m = random_gpt2("gpt2-medium", seed=77)
    lm = HipArithmeticLM(m, _IdTokenizer(50257), logits_dtype="f16", max_batch=2 * n)
    q = {"temp": 0.9, "precision": 26, "topk": 100, "finish_sent": True}
    # secrets of 0..255 bytes (one packet each); the gate's perplexity threshold is the median of an ungated
    # first pass over the same secrets, so roughly half the covers pass at attempt 1 and the regeneration
    # schedule (seed pool, top_k 80 / 70, temp 0.8 / 0.7) runs for the rest
    secrets = [synthetic.payload_bytes(s, s % 256) for s in range(n)]
    seed = "w11. w12. w13"
    first = cover_generate_batch(secrets, seed_text=seed, quality=q, ecc="rs", lm=lm, quality_gate=False)
    guard = _ensure_guard(None)
    ppl = sorted(v.metrics["ppl"] for v in guard.evaluate_batch(first, prepare_gate_thresholds(None)))
    gate = {"max_ppl": float(ppl[n // 2])}
    # the reference's schedule (api.py:496-523: top_k 80 / 70, temp 0.8 / 0.7) with a seed pool the test
    # tokenizer can spell, so that each cover's text tells which attempt made it
    strategy = {"seed_pool": ["w21. w22. w23", "w31. w32. w33"]}
    out = cover_generate_batch(secrets, seed_text=seed, quality=q, ecc="rs", lm=lm, quality_gate=True,
                               gate_thresholds=gate, regen_attempts=2, regen_strategy=strategy, return_errors=True)
    passed = [i for i, t in enumerate(out) if isinstance(t, str)]
    failed = [i for i, t in enumerate(out) if isinstance(t, QualityGateError)]
    assert len(passed) + len(failed) == n
    assert passed and failed, (len(passed), len(failed), gate)
    for i in failed:
        assert out[i].reasons  # rejected by the last attempt of the schedule, with its reasons
    # a cover reveals with the seed and quality of the attempt that made it (as in the reference, cover_reveal
    # takes them from the caller)
    attempts = list(iter_attempts(seed, 2, strategy))
    by_attempt = {}
    for i in passed:
        a = next(j for j, att in enumerate(attempts) if out[i].startswith(att.seed_text))
        by_attempt.setdefault(a, []).append(i)
    assert 0 in by_attempt, {a: len(v) for a, v in by_attempt.items()}
    for a, idx in sorted(by_attempt.items()):
        aq = dict(normalise_quality(q), **attempts[a].overrides)
        got = cover_reveal_batch([out[i] for i in idx], seed_text=attempts[a].seed_text, quality=aq, ecc="rs", lm=lm)
        wrong = [i for i, g in zip(idx, got) if g != secrets[i]]
        assert not wrong, f"attempt {a + 1}: {len(wrong)} of {len(idx)} covers did not reveal (first: {wrong[:8]})"
    print(f"C5-like: {n} secrets, gate {gate}, passed and revealed per attempt "
          f"{ {a + 1: len(v) for a, v in sorted(by_attempt.items())} }, {len(failed)} rejected")
