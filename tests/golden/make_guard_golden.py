"""Golden vectors for the quality guard and the regeneration loop, produced by RUNNING the reference here.

Records (tests/golden/guard_golden.json):
  * text metrics: ngram_repeat_ratio / type_token_ratio / avg_sentence_len (metrics/text_stats.py), the
    fallback LMScorer.score and avg_entropy (metrics/lm_scorer.py, metrics/entropy.py) on a set of texts;
  * QualityGuard(LMScorer(prefer_transformers=False)).evaluate under several threshold sets
    (detect/guard.py): passed, reasons, metrics;
  * api._iter_attempts schedules and api._prepare_gate_thresholds results (api.py:451-523);
  * api.cover_generate with the reference MockLM (lm/mock.py), ecc="none" and a deterministic msg_id:
    the returned cover text, or the QualityGateError's text / reasons / metrics.
usage (this container only; /root/reference is read-only input): python tests/golden/make_guard_golden.py
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent

TEXTS = [
    "",
    "   ",
    "hello",
    "hello world. this is a test! hello world again?",
    "the cat sat on the mat the cat sat on the mat the cat sat on the mat",
    "One two three. Four five six seven! Eight nine ten eleven twelve?\nThirteen",
    "Repeat repeat REPEAT repeat. repeat",
    "...",
    "a b c d e f g h i j k l m n o p",
    "در یک گفت‌وگوی کوتاه درباره‌ی فناوری صحبت می‌کنیم. آیا این درست است؟ بله",
    "x y x y x y x y. z",
    "Mixed   whitespace\tand\nnewlines  here .  end",
]

THRESHOLDS = [
    None,
    {"max_ppl": 3.0},
    {"min_ttr": 0.9, "max_ngram_repeat": 0.1},
    {"max_avg_entropy": 1.0, "min_avg_sentence_len": 4.0},
    {"max_ppl": None, "min_avg_sentence_len": "2.5"},
]

ATTEMPTS = [
    ("base seed", 2, None),
    ("base seed", 4, None),
    ("s", 3, {"seed_pool": ["p1"], "top_k_steps": ["90", 40.0], "temperature_steps": [1]}),
    ("s", 0, {}),
    ("s", 2, {"seed_pool": None, "top_k_steps": []}),
]

COVERS = [
    dict(secret="secret message", seed_text="hello world.", thresholds=None, regen_attempts=2),
    dict(secret=b"\x00\x01binary\xff", seed_text="A seed. With two sentences.", thresholds={"max_ppl": 1.0},
         regen_attempts=2),
    dict(secret="x" * 40, seed_text="short", thresholds={"min_avg_sentence_len": 3.0}, regen_attempts=3),
    dict(secret="another secret", seed_text="base", thresholds={"min_ttr": 0.99}, regen_attempts=1),
    dict(secret="chunked " * 10, seed_text="seed text here", thresholds={"max_ngram_repeat": 0.5}, regen_attempts=2,
         chunk_bytes=16),
    dict(secret="repetitive seed", seed_text="a a a a a a a a a a a a a a", thresholds=None, regen_attempts=2),
    dict(secret="rep", seed_text="b b b b b b b b b b", thresholds={"max_ppl": 6.0}, regen_attempts=2),
]


def main():
    sys.path.insert(0, str(REF / "src"))
    from neuralstego import api
    from neuralstego.detect.guard import QualityGuard
    from neuralstego.exceptions import QualityGateError
    from neuralstego.lm.mock import MockLM
    from neuralstego.metrics import LMScorer, avg_entropy, avg_sentence_len, ngram_repeat_ratio, type_token_ratio

    scorer = LMScorer(prefer_transformers=False)
    guard = QualityGuard(lm_scorer=scorer)
    out = {"texts": TEXTS, "metrics": [], "guard": [], "attempts": [], "thresholds": [], "covers": []}
    for t in TEXTS:
        out["metrics"].append({"ngram_repeat_ratio": ngram_repeat_ratio(t), "type_token_ratio": type_token_ratio(t),
                               "avg_sentence_len": avg_sentence_len(t), "score": scorer.score(t),
                               "avg_entropy": avg_entropy(t, scorer)})
    for th in THRESHOLDS:
        prepared = api._prepare_gate_thresholds(th)
        out["thresholds"].append({"overrides": th, "prepared": prepared})
        for t in TEXTS:
            r = guard.evaluate(t, dict(prepared))
            out["guard"].append({"text": t, "thresholds": prepared, "passed": r.passed, "reasons": r.reasons,
                                 "metrics": r.metrics})
    for seed, n, strat in ATTEMPTS:
        sched = [{"seed_text": a.seed_text, "overrides": a.overrides, "seed_variant": a.seed_variant}
                 for a in api._iter_attempts(seed, n, strat or {})]
        out["attempts"].append({"seed_text": seed, "regen_attempts": n, "strategy": strat, "schedule": sched})
    counter = {"n": 0}

    def fixed_msg_id():
        counter["n"] += 1
        return f"00000000-0000-4000-8000-{counter['n']:012d}"

    api.make_msg_id = fixed_msg_id
    for case in COVERS:
        counter["n"] = 0
        rec = dict(case)
        secret = case["secret"]
        rec["secret"] = list(secret.encode() if isinstance(secret, str) else secret)
        rec["secret_is_str"] = isinstance(secret, str)
        try:
            text = api.cover_generate(secret, seed_text=case["seed_text"], ecc="none", lm=MockLM(),
                                      gate_thresholds=case["thresholds"], regen_attempts=case["regen_attempts"],
                                      chunk_bytes=case.get("chunk_bytes", 256))
            rec["result"] = {"text": text}
        except QualityGateError as exc:
            rec["result"] = {"error": "QualityGateError", "cover_text": exc.cover_text, "reasons": exc.reasons,
                             "metrics": exc.metrics}
        out["covers"].append(rec)
        print(case["seed_text"], "->", "error" if "error" in rec["result"] else "text", flush=True)
    (HERE / "guard_golden.json").write_text(json.dumps(out, ensure_ascii=False, indent=1))
    print("wrote", HERE / "guard_golden.json")


if __name__ == "__main__":
    main()
