"""CPU: the quality guard, regeneration schedule and cover generation against the reference run's outputs
(tests/golden/guard_golden.json, made by tests/golden/make_guard_golden.py): text statistics, the fallback
LM metrics, guard verdicts and messages, attempt schedules, threshold preparation and complete
cover_generate runs (MockLM, deterministic msg_id) including QualityGateError after every attempt."""

import json
import math
from pathlib import Path

import pytest

from neuralsteganography_amd import cover, metrics, stego
from neuralsteganography_amd.detect import QualityGuard
from neuralsteganography_amd.exceptions import ConfigurationError, QualityGateError
from neuralsteganography_amd.lm.mock import MockLM

G = json.loads((Path(__file__).resolve().parent / "golden" / "guard_golden.json").read_text())


def _close(a, b):
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return a == b or (isinstance(a, (int, float)) and abs(a - b) <= 1e-12 * max(1.0, abs(b)))


@pytest.mark.parametrize("i", range(len(G["texts"])))
def test_text_metrics_match_reference(i):
    t, want = G["texts"][i], G["metrics"][i]
    assert metrics.ngram_repeat_ratio(t) == want["ngram_repeat_ratio"]
    assert metrics.type_token_ratio(t) == want["type_token_ratio"]
    assert metrics.avg_sentence_len(t) == want["avg_sentence_len"]
    sc = metrics.LMScorer(prefer_transformers=False)
    got = sc.score(t)
    assert set(got) == set(want["score"]) and all(_close(got[k], want["score"][k]) for k in got)
    assert _close(metrics.avg_entropy(t, sc), want["avg_entropy"])


def test_guard_verdicts_match_reference():
    guard = QualityGuard(lm_scorer=metrics.LMScorer(prefer_transformers=False))
    for rec in G["guard"]:
        r = guard.evaluate(rec["text"], rec["thresholds"])
        assert r.passed == rec["passed"] and r.reasons == rec["reasons"], rec["text"]
        assert set(r.metrics) == set(rec["metrics"])
        assert all(_close(r.metrics[k], rec["metrics"][k]) for k in r.metrics)
    # the batched form gives the same verdicts
    th = G["guard"][0]["thresholds"]
    batch = guard.evaluate_batch(G["texts"], th)
    single = [guard.evaluate(t, th) for t in G["texts"]]
    assert [(b.passed, b.reasons) for b in batch] == [(s.passed, s.reasons) for s in single]


def test_threshold_preparation_and_attempt_schedule_match_reference():
    for rec in G["thresholds"]:
        assert cover.prepare_gate_thresholds(rec["overrides"]) == rec["prepared"]
    with pytest.raises(ConfigurationError):
        cover.prepare_gate_thresholds({"max_ppl": "not a number"})
    for rec in G["attempts"]:
        got = [{"seed_text": a.seed_text, "overrides": a.overrides, "seed_variant": a.seed_variant}
               for a in cover.iter_attempts(rec["seed_text"], rec["regen_attempts"], rec["strategy"] or {})]
        assert got == rec["schedule"]


@pytest.mark.parametrize("i", range(len(G["covers"])))
def test_cover_generate_matches_reference(i, monkeypatch):
    rec = G["covers"][i]
    counter = {"n": 0}

    def fixed_msg_id():
        counter["n"] += 1
        return f"00000000-0000-4000-8000-{counter['n']:012d}"

    monkeypatch.setattr(stego, "make_msg_id", fixed_msg_id)
    secret = bytes(rec["secret"])
    if rec["secret_is_str"]:
        secret = secret.decode()
    kw = dict(seed_text=rec["seed_text"], ecc="none", lm=MockLM(), gate_thresholds=rec["thresholds"],
              regen_attempts=rec["regen_attempts"], chunk_bytes=rec.get("chunk_bytes", 256))
    res = rec["result"]
    if "error" in res:
        with pytest.raises(QualityGateError) as ei:
            cover.cover_generate(secret, **kw)
        assert ei.value.cover_text == res["cover_text"] and ei.value.reasons == res["reasons"]
        assert all(_close(ei.value.metrics[k], res["metrics"][k]) for k in res["metrics"])
    else:
        assert cover.cover_generate(secret, **kw) == res["text"]


def test_cover_generate_batch_mixed_outcomes(monkeypatch):
    """Many secrets through one schedule: passing ones return text, failing ones their QualityGateError."""
    monkeypatch.setattr(stego, "make_msg_id", lambda: "00000000-0000-4000-8000-000000000001")
    out = cover.cover_generate_batch(["a", "b" * 30, "c"], seed_text="x y", ecc="none", lm=MockLM(),
                                     gate_thresholds={"max_ppl": 1.5}, regen_attempts=1, return_errors=True)
    assert len(out) == 3 and all(isinstance(o, (str, QualityGateError)) for o in out)
    single = []
    for s in ["a", "b" * 30, "c"]:
        try:
            single.append(cover.cover_generate(s, seed_text="x y", ecc="none", lm=MockLM(),
                                               gate_thresholds={"max_ppl": 1.5}, regen_attempts=1))
        except QualityGateError as exc:
            single.append(exc)
    assert [type(o) for o in out] == [type(o) for o in single]
    assert [o if isinstance(o, str) else o.reasons for o in out] == \
           [o if isinstance(o, str) else o.reasons for o in single]


def test_cover_reveal_from_spans_payload():
    lm = MockLM()
    spans = stego.stego_encode(b"reveal me", ecc="none", seed_text="s", lm=lm)
    assert cover.cover_reveal(json.dumps([list(s) for s in spans]), seed_text="s", ecc="none", lm=lm) == b"reveal me"
    assert cover.cover_reveal(json.dumps({"spans": [list(s) for s in spans]}), seed_text="s", ecc="none",
                              lm=lm) == b"reveal me"
    from neuralsteganography_amd.codec.errors import DecodeDivergenceError

    with pytest.raises(DecodeDivergenceError):  # a text that does not start with the seed
        cover.cover_reveal("plain text cover", seed_text="s", ecc="none", lm=lm)


def test_cover_text_round_trip_through_text_to_spans():
    """cover_generate -> text -> cover_reveal: the spans are recovered from the TEXT (the reference's
    text_to_spans is a NotImplementedError placeholder, codec/textio.py:58-63).  Mock provider: identity
    coder, packets are the tokens."""
    from neuralsteganography_amd.codec.textio import seed_to_ids, text_to_spans

    lm = MockLM()
    secrets = [b"short", bytes(range(32, 127)) * 3, b"x"]
    texts = cover.cover_generate_batch(secrets, seed_text="A seed. ", ecc="none", lm=lm, quality_gate=False,
                                       chunk_bytes=40)
    assert cover.cover_reveal_batch(texts, seed_text="A seed. ", ecc="none", lm=lm) == secrets
    assert cover.cover_reveal(texts[1], seed_text="A seed. ", ecc="none", lm=lm) == secrets[1]
    spans = stego.stego_encode(secrets[1], ecc="none", seed_text="A seed. ", lm=lm, chunk_bytes=40)
    got = text_to_spans(texts[1], seed_to_ids("A seed. ", lm.tokenizer), lm.tokenizer, lm=lm, seed_text="A seed. ")
    assert len(got) == len(spans) == 8  # 285 bytes in 40-byte chunks
    with pytest.raises(NotImplementedError):  # no provider: the reference's placeholder behaviour
        text_to_spans(texts[1], [], lm.tokenizer)
