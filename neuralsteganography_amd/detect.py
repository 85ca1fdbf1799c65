"""Rule-based cover-text quality guard (``src/neuralstego/detect/guard.py:18-86``, ``detect/features.py``).

:meth:`QualityGuard.evaluate_batch` scores many covers at once: on the transformers branch the LM metrics of
every text come from one batched GPU forward (:class:`~neuralsteganography_amd.metrics.HipLMScorer`); the rules
and messages are the reference's.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Mapping, Optional, Sequence

from .metrics import LMScorer, avg_entropy, avg_sentence_len, ngram_repeat_ratio, type_token_ratio

EXPECTED_FEATURES = ("ppl", "avg_nll", "avg_entropy", "ngram_repeat_ratio", "type_token_ratio", "avg_sentence_len")


def extract_features(metrics: Mapping[str, float]) -> Dict[str, float]:
    """``detect/features.py``: the six guard features, 0.0 when absent."""
    return {k: float(metrics.get(k, 0.0)) for k in EXPECTED_FEATURES}


@dataclass
class GuardResult:
    passed: bool
    reasons: List[str]
    metrics: Dict[str, float]
    detector_score: Optional[float] = None


def _rule_reasons(f: Mapping[str, float], th: Mapping[str, float]) -> List[str]:
    """``guard.py:44-67``: the threshold rules in the reference's order and wording."""
    out: List[str] = []
    if "max_ppl" in th and f["ppl"] > th["max_ppl"]:
        out.append(f"ppl {f['ppl']:.2f} exceeds max {th['max_ppl']:.2f}")
    if "max_ngram_repeat" in th and f["ngram_repeat_ratio"] > th["max_ngram_repeat"]:
        out.append(f"ngram repeat ratio {f['ngram_repeat_ratio']:.2f} exceeds {th['max_ngram_repeat']:.2f}")
    if "min_ttr" in th and f["type_token_ratio"] < th["min_ttr"]:
        out.append(f"type-token ratio {f['type_token_ratio']:.2f} below {th['min_ttr']:.2f}")
    if "max_avg_entropy" in th and f["avg_entropy"] > th["max_avg_entropy"]:
        out.append(f"avg entropy {f['avg_entropy']:.2f} exceeds {th['max_avg_entropy']:.2f}")
    if "min_avg_sentence_len" in th and f["avg_sentence_len"] < th["min_avg_sentence_len"]:
        out.append(f"avg sentence length {f['avg_sentence_len']:.2f} below {th['min_avg_sentence_len']:.2f}")
    return out


@dataclass
class QualityGuard:
    lm_scorer: LMScorer = field(default_factory=LMScorer)
    classifier: Optional[object] = None

    def _text_stats(self, text: str) -> Dict[str, float]:
        return {"ngram_repeat_ratio": ngram_repeat_ratio(text), "type_token_ratio": type_token_ratio(text),
                "avg_sentence_len": avg_sentence_len(text)}

    def _collect_metrics(self, text: str) -> Dict[str, float]:
        """``guard.py:33-42``: LM metrics, then the text statistics and the average entropy."""
        m = dict(self.lm_scorer.score(text))
        m.update(self._text_stats(text))
        m["avg_entropy"] = avg_entropy(text, self.lm_scorer)
        return m

    def _finish(self, metrics: Dict[str, float], thresholds: Mapping[str, float]) -> GuardResult:
        feats = extract_features(metrics)
        reasons = _rule_reasons(feats, thresholds)
        score = None
        if self.classifier is not None and hasattr(self.classifier, "predict_proba"):
            score = float(self.classifier.predict_proba(feats))
            metrics["detector_score"] = score
            if "max_detector_score" in thresholds and score > thresholds["max_detector_score"]:
                reasons.append(f"detector score {score:.2f} exceeds {thresholds['max_detector_score']:.2f}")
        return GuardResult(not reasons, reasons, metrics, score)

    def evaluate(self, text: str, thresholds: Mapping[str, float]) -> GuardResult:
        return self._finish(self._collect_metrics(text), thresholds)

    def evaluate_batch(self, texts: Sequence[str], thresholds: Mapping[str, float]) -> List[GuardResult]:
        """:meth:`evaluate` for every text; the LM metrics of all texts in one scorer call."""
        if not hasattr(self.lm_scorer, "metrics_batch"):
            return [self.evaluate(t, thresholds) for t in texts]
        lm = self.lm_scorer.metrics_batch(list(texts))
        out = []
        for text, m in zip(texts, lm):
            ent = m.get("avg_entropy", 0.0)
            metrics = {k: m[k] for k in ("ppl", "avg_nll", "token_count")}
            metrics.update(self._text_stats(text))
            metrics["avg_entropy"] = ent
            out.append(self._finish(metrics, thresholds))
        return out


__all__ = ["QualityGuard", "GuardResult", "extract_features", "EXPECTED_FEATURES"]
