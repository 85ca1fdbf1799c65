"""Cover generation with the quality gate and regeneration loop (``src/neuralstego/api.py:418-705``),
batched (SURVEY §8(f) 2, config C5 "quality-guard on").

``cover_generate`` / ``cover_reveal`` keep the reference's signatures, defaults (``DEFAULT_GATE_THRESHOLDS``,
``DEFAULT_REGEN_STRATEGY``, ``api.py:89-104``), attempt schedule (``_iter_attempts``, ``:491-523``: attempt 1
uses the caller's seed and quality, later attempts pop the next seed of the pool, ``top_k`` and ``temp``
overrides), guard (``QualityGuard(LMScorer(prefer_transformers=False))`` by default, ``:118-127``) and errors
(``QualityGateError`` with the last attempt's text, reasons and metrics).

``cover_generate_batch`` runs the same schedule for MANY secrets: attempt r encodes every still-rejected
secret in ONE lockstep batch (all their packets are streams of one GPT-2 + HIP-coder loop,
``stego_encode_batch``), the guard scores all the resulting covers at once (one batched GPU forward on the
transformers branch), and only the rejected secrets go on to attempt r+1.
"""

from __future__ import annotations

import json
import logging
from collections import deque
from copy import deepcopy
from dataclasses import dataclass
from typing import Any, Dict, Iterable, List, Mapping, Optional, Sequence

from .codec.textio import seed_to_ids, spans_to_text, text_to_spans
from .detect import GuardResult, QualityGuard
from .exceptions import ConfigurationError, QualityGateError
from .metrics import LMScorer
from .stego import normalise_quality, stego_decode, stego_encode_batch

log = logging.getLogger(__name__)

DEFAULT_GATE_THRESHOLDS: Dict[str, float] = {  # api.py:89-94
    "max_ppl": 120.0,
    "max_ngram_repeat": 0.35,
    "min_ttr": 0.25,
    "max_avg_entropy": 5.5,
}

DEFAULT_REGEN_STRATEGY: Dict[str, Any] = {  # api.py:97-104 (the reference's Persian seed pool)
    "seed_pool": [
        "در یک گفت‌وگوی کوتاه درباره‌ی فناوری صحبت می‌کنیم.",
        "در یک گفت‌وگوی دوستانه درباره‌ی فرهنگ و هنر صحبت می‌کنیم.",
    ],
    "top_k_steps": [80, 70, 60],
    "temperature_steps": [0.8, 0.7],
}

_DEFAULT_GUARD: Optional[QualityGuard] = None


@dataclass
class Attempt:
    """``api.py:74-78`` ``_AttemptConfig``."""

    seed_text: str
    overrides: Dict[str, Any]
    seed_variant: str


def _ensure_guard(guard: Optional[QualityGuard]) -> QualityGuard:
    global _DEFAULT_GUARD
    if guard is not None:
        return guard
    if _DEFAULT_GUARD is None:
        _DEFAULT_GUARD = QualityGuard(lm_scorer=LMScorer(prefer_transformers=False))
    return _DEFAULT_GUARD


def prepare_gate_thresholds(overrides: Optional[Mapping[str, float]]) -> Dict[str, float]:
    """``api.py:451-465``: defaults updated by the non-None overrides (floats, else ConfigurationError)."""
    out = dict(DEFAULT_GATE_THRESHOLDS)
    for key, value in (overrides or {}).items():
        if value is None:
            continue
        try:
            out[str(key)] = float(value)
        except (TypeError, ValueError) as exc:
            raise ConfigurationError(f"invalid threshold value for {key!s}: {value!r}") from exc
    return out


def prepare_regen_strategy(strategy: Optional[Mapping[str, Any]]) -> Dict[str, Any]:
    """``api.py:468-479``."""
    merged = deepcopy(DEFAULT_REGEN_STRATEGY)
    for key, value in (strategy or {}).items():
        if value is not None:
            merged[str(key)] = value
    for key in ("seed_pool", "top_k_steps", "temperature_steps"):
        merged[key] = list(merged.get(key, []))
    return merged


def _as_int(value: Any) -> int:
    try:
        return int(value)
    except (TypeError, ValueError):
        return int(float(value))


def _as_float(value: Any) -> float:
    try:
        return float(value)
    except (TypeError, ValueError):
        raise ConfigurationError(f"invalid numeric value for regeneration strategy: {value!r}")


def iter_attempts(seed_text: str, regen_attempts: int, strategy: Optional[Mapping[str, Any]]) -> Iterable[Attempt]:
    """``api.py:496-523``: attempt 0 = the caller's seed, no overrides; attempt i > 0 = next pool seed (or the
    caller's once the pool is empty), next ``top_k`` step, next ``temp`` step."""
    cfg = prepare_regen_strategy(strategy)
    seeds = deque(str(s) for s in cfg.get("seed_pool", []))
    ks = deque(cfg.get("top_k_steps", []))
    temps = deque(cfg.get("temperature_steps", []))
    for i in range(max(regen_attempts, 0) + 1):
        if i == 0:
            yield Attempt(seed_text, {}, "base")
            continue
        seed = str(seeds.popleft()) if seeds else seed_text
        over: Dict[str, Any] = {}
        if ks:
            over["top_k"] = _as_int(ks.popleft())
        if temps:
            over["temp"] = _as_float(temps.popleft())
        yield Attempt(seed, over, f"alt-{i}")


def _normalise_secret(secret) -> bytes:
    if isinstance(secret, bytes):
        return secret
    if isinstance(secret, str):
        return secret.encode("utf-8")
    raise TypeError("secret must be bytes or string")


def _tokenizer_of(lm) -> Any:
    tok = getattr(lm, "tokenizer", None)
    if tok is None:
        raise ConfigurationError("language model tokenizer unavailable for cover rendering")
    return tok


def _ensure_cover_lm(lm):
    if lm is not None:
        return lm
    from .lm import load_lm

    try:
        return load_lm("gpt2-fa")  # api.py:391-395 default provider
    except Exception as exc:
        raise ConfigurationError("failed to load default language model") from exc


def _render_covers(payloads: Sequence[bytes], *, seed_text: str, quality: Mapping[str, Any], chunk_bytes: int,
                   use_crc: bool, ecc: str, nsym: int, lm) -> List[str]:
    """``_generate_cover_once`` (``api.py:526-562``) for many payloads: one batched stego_encode."""
    results = stego_encode_batch(list(payloads), chunk_bytes=chunk_bytes, use_crc=use_crc, ecc=ecc, nsym=nsym,
                                 quality=dict(quality), seed_text=seed_text, lm=lm)
    tok = _tokenizer_of(lm)
    seed_ids = seed_to_ids(seed_text, tok)
    return [spans_to_text([list(map(int, s)) for s in res], seed_ids, tok) for res in results]


def cover_generate_batch(secrets: Sequence[Any], *, seed_text: str, quality: Optional[Mapping[str, object]] = None,
                         chunk_bytes: int = 256, use_crc: bool = True, ecc: str = "rs", nsym: int = 10, lm=None,
                         quality_gate: bool = True, gate_thresholds: Optional[Mapping[str, float]] = None,
                         regen_attempts: int = 2, regen_strategy: Optional[Mapping[str, Any]] = None,
                         quality_guard: Optional[QualityGuard] = None, return_errors: bool = False) -> List[Any]:
    """One cover text per secret.  A secret whose every attempt is rejected raises ``QualityGateError`` (the
    first such, in input order), or leaves the error in its slot with ``return_errors=True``."""
    payloads = [_normalise_secret(s) for s in secrets]
    provider = _ensure_cover_lm(lm)
    q = normalise_quality(quality)
    kw = dict(chunk_bytes=chunk_bytes, use_crc=use_crc, ecc=ecc, nsym=nsym, lm=provider)
    if not quality_gate:
        return _render_covers(payloads, seed_text=seed_text, quality=q, **kw)
    thresholds = prepare_gate_thresholds(gate_thresholds)
    guard = _ensure_guard(quality_guard)
    total = max(regen_attempts, 0) + 1
    out: List[Any] = [None] * len(payloads)
    last: Dict[int, tuple] = {}
    pending = list(range(len(payloads)))
    for idx, att in enumerate(iter_attempts(seed_text, regen_attempts, regen_strategy or {}), start=1):
        if not pending:
            break
        aq = dict(q)
        aq.update(att.overrides)
        texts = _render_covers([payloads[i] for i in pending], seed_text=att.seed_text, quality=aq, **kw)
        verdicts: List[GuardResult] = guard.evaluate_batch(texts, thresholds)
        rejected = []
        for i, text, v in zip(pending, texts, verdicts):
            status = "PASS" if v.passed else "REJECT"
            log.info("quality attempt %d/%d (%s) message %d -> %s %s", idx, total, att.seed_variant, i, status,
                     "; ".join(v.reasons))
            if v.passed:
                out[i] = text
            else:
                last[i] = (text, v)
                rejected.append(i)
        pending = rejected
    for i in pending:
        text, v = last[i]
        err = QualityGateError(text, list(v.reasons), dict(v.metrics))
        if not return_errors:
            raise err
        out[i] = err
    return out


def cover_generate(secret, *, seed_text: str, quality: Optional[Mapping[str, object]] = None, chunk_bytes: int = 256,
                   use_crc: bool = True, ecc: str = "rs", nsym: int = 10, lm=None, quality_gate: bool = True,
                   gate_thresholds: Optional[Mapping[str, float]] = None, regen_attempts: int = 2,
                   regen_strategy: Optional[Mapping[str, Any]] = None,
                   quality_guard: Optional[QualityGuard] = None) -> str:
    """``api.py:565-662``: one secret."""
    return cover_generate_batch([secret], seed_text=seed_text, quality=quality, chunk_bytes=chunk_bytes,
                                use_crc=use_crc, ecc=ecc, nsym=nsym, lm=lm, quality_gate=quality_gate,
                                gate_thresholds=gate_thresholds, regen_attempts=regen_attempts,
                                regen_strategy=regen_strategy, quality_guard=quality_guard)[0]


def _parse_spans_payload(payload: str) -> List[List[int]]:
    """``api.py:426-448``: a JSON list of int lists (or ``{"spans": [...]}``)."""
    try:
        obj = json.loads(payload)
    except json.JSONDecodeError as exc:
        raise ConfigurationError("cover text parsing not implemented; provide spans JSON input") from exc
    if isinstance(obj, Mapping):
        obj = obj.get("spans")
    if not isinstance(obj, Sequence):
        raise ConfigurationError("spans payload must be a sequence")
    spans = []
    for entry in obj:
        if not isinstance(entry, Sequence):
            raise ConfigurationError("span entry must be a sequence of integers")
        spans.append([int(v) for v in entry])
    return spans


def _span_end(bits, counts, toks, finish, sent_end) -> Optional[int]:
    """Index of the last token of the span that starts at ``toks[0]``, from the decoder's output for the
    remaining tokens: the packet (``bits`` read up to the JSON's closing brace) is complete after the first
    token whose cumulative bit count covers it (t*); with ``finish_sent`` the encoder then emitted top-1 tokens
    up to and including the first sentence-ending one AFTER t* (``code_base/arithmetic.py:114,134-137``: the
    test runs only on tail tokens).  None while the decoded prefix does not yet settle it."""
    from .exceptions import PacketECCError
    from .stego import bits_to_bytes_lsb, packet_prefix

    try:
        need = 8 * len(packet_prefix(bits_to_bytes_lsb(bits)))
    except PacketECCError:
        return None
    tstar = next((t for t, c in enumerate(counts) if c >= need), None)
    if tstar is None:
        return None
    if not finish:
        return tstar
    for t in range(tstar + 1, len(counts)):
        if sent_end[int(toks[t])]:
            return t
    if len(counts) == len(toks):  # the text ends inside the tail (stripped / truncated cover)
        return len(toks) - 1
    return None


def _split_double_newlines(ids: List[int], tok) -> List[int]:
    """``code_base/arithmetic.py:233-242``: a re-tokenised "\\n\\n" (GPT-2 id 628, which the coder never emits:
    it is banned) is split back into two "\\n" (id 198) -- applied when the tokenizer has those pieces."""
    if 628 not in ids:
        return ids
    try:
        if tok.decode([628]) != "\n\n" or tok.decode([198]) != "\n":
            return ids
    except Exception:  # noqa: BLE001 - a vocabulary without those ids
        return ids
    out: List[int] = []
    for t in ids:
        out.extend((198, 198) if t == 628 else (t,))
    return out


def _cover_ids(text: str, seed_text: str, seed_ids: List[int], tok) -> Optional[List[int]]:
    """The cover's token ids after the seed: the text's ids minus the seed's, or -- when the seed's last token
    merged with the first cover token on re-tokenisation -- the ids of the text after the decoded seed."""
    ids = seed_to_ids(text, tok)
    if ids[: len(seed_ids)] == seed_ids:
        return ids[len(seed_ids):]
    seed_str = spans_to_text([], seed_ids, tok)
    if seed_str and text.startswith(seed_str):
        return seed_to_ids(text[len(seed_str):], tok) if text[len(seed_str):] else []
    return None


def texts_to_spans(texts: Sequence[str], *, seed_text: str, lm, quality: Optional[Mapping[str, object]] = None
                   ) -> List[List[List[int]]]:
    """Recover the token spans of many cover texts (the inverse of ``spans_to_text``, which the reference leaves
    unimplemented, ``codec/textio.py:58-63``).  The text is re-tokenised, the seed's ids are stripped, and the
    spans are found one per round: every cover's next span is decoded as one stream of a lockstep batch, the
    packet completes at a known token and the span ends there or, with ``finish_sent``, at the following
    sentence end.  A text that re-tokenises differently from the emitted ids (GPT-2 BPE merges, also across
    span boundaries) is repaired while decoding with the reference's heuristics (``code_base/arithmetic.py:
    233-242,300-342``, the provider's ``decode_counted_repair``): the spans are the repaired ids."""
    from .codec.errors import DecodeDivergenceError
    from .lm.mock import MockLM
    from .stego import _quality_args

    tok = _tokenizer_of(lm)
    seed_ids = seed_to_ids(seed_text, tok)
    q = _quality_args(quality)
    finish = bool(q.get("finish_sent")) and hasattr(lm, "sentence_end_table")
    sent_end = lm.sentence_end_table() if finish else None
    rest: List[List[int]] = []
    for i, text in enumerate(texts):
        ids = _cover_ids(text, seed_text, seed_ids, tok)
        if ids is None:
            raise DecodeDivergenceError(f"cover {i} does not start with the seed text")
        rest.append(_split_double_newlines(ids, tok))
    context = list(lm.encode_seed(seed_text))
    spans: List[List[List[int]]] = [[] for _ in texts]
    active = [i for i in range(len(texts)) if rest[i]]
    while active:
        lists = [rest[i] for i in active]

        def settled(bits_l, counts_l, toks_l=None):
            toks_l = lists if toks_l is None else toks_l
            return all(_span_end(b, c, l, finish, sent_end) is not None for b, c, l in zip(bits_l, counts_l, toks_l))

        edits_l = [[] for _ in lists]
        orig = [list(l) for l in lists]
        if hasattr(lm, "decode_counted_repair"):
            bits_l, counts_l, lists, edits_l = lm.decode_counted_repair(lists, context, quality=q, done=settled)
        elif hasattr(lm, "decode_counted"):
            bits_l, counts_l = lm.decode_counted(lists, context, quality=q, done=settled)
        elif isinstance(lm, MockLM):  # identity coder: 8 bits per token
            bits_l = [lm.decode_arithmetic(l, context, quality=q) for l in lists]
            counts_l = [[8 * (t + 1) for t in range(len(l))] for l in lists]
        else:
            raise NotImplementedError("text_to_spans needs a provider with decode_counted (or the mock)")
        nxt = []
        for i, l, b, c, ed, o in zip(active, lists, bits_l, counts_l, edits_l, orig):
            end = _span_end(b, c, l, finish, sent_end)
            if end is None:
                raise DecodeDivergenceError(f"cover {i}: no complete packet in the remaining {len(l)} tokens")
            # the list as it stood after the last repair inside the span (later "repairs" decoded the next span's
            # tokens out of context); a repair at the span's end may have split a cross-boundary merge, whose
            # suffix tokens start the next span
            l = next((snap for p, snap in reversed(ed) if p <= end), o)
            spans[i].append([int(t) for t in l[: end + 1]])
            rest[i] = l[end + 1:]
            if rest[i]:
                nxt.append(i)
        active = nxt
    return spans


def _looks_like_spans_json(text: str) -> bool:
    try:
        _parse_spans_payload(text)
        return True
    except ConfigurationError:
        return False


def cover_reveal_batch(cover_texts: Sequence[str], *, seed_text: str, quality: Optional[Mapping[str, object]] = None,
                       use_crc: bool = True, ecc: str = "rs", nsym: int = 10, lm=None,
                       return_errors: bool = False) -> List[Any]:
    """:func:`cover_reveal` for many covers: spans of all texts recovered round by round in lockstep batches,
    then one batched ``stego_decode``."""
    from .stego import stego_decode_batch

    provider = _ensure_cover_lm(lm)
    q = normalise_quality(quality)
    span_sets: List[Any] = [None] * len(cover_texts)
    plain = []
    for i, text in enumerate(cover_texts):
        if _looks_like_spans_json(text):
            span_sets[i] = _parse_spans_payload(text)
        else:
            plain.append(i)
    if plain:
        for i, sp in zip(plain, texts_to_spans([cover_texts[i] for i in plain], seed_text=seed_text, lm=provider,
                                                quality=q)):
            span_sets[i] = sp
    return stego_decode_batch(span_sets, use_crc=use_crc, ecc=ecc, nsym=nsym, quality=q, seed_text=seed_text,
                              lm=provider, return_errors=return_errors)


def cover_reveal(cover_text: str, *, seed_text: str, quality: Optional[Mapping[str, object]] = None,
                 use_crc: bool = True, ecc: str = "rs", nsym: int = 10, lm=None) -> bytes:
    """``api.py:665-704``: a JSON spans payload is decoded as in the reference; a cover TEXT has its spans
    recovered by :func:`texts_to_spans` (the reference's ``text_to_spans`` raises ``NotImplementedError``,
    after which it can only parse JSON), then ``stego_decode``."""
    provider = _ensure_cover_lm(lm)
    q = normalise_quality(quality)
    if _looks_like_spans_json(cover_text):
        spans = _parse_spans_payload(cover_text)
    else:
        tok = getattr(provider, "tokenizer", None)
        try:
            if tok is None:
                raise NotImplementedError
            spans = text_to_spans(cover_text, seed_to_ids(seed_text, tok), tok, lm=provider, quality=q,
                                  seed_text=seed_text)
        except NotImplementedError:
            spans = _parse_spans_payload(cover_text)
    return stego_decode(spans, use_crc=use_crc, ecc=ecc, nsym=nsym, quality=q, seed_text=seed_text, lm=provider)


__all__ = ["cover_generate", "cover_generate_batch", "cover_reveal", "cover_reveal_batch", "texts_to_spans",
           "iter_attempts", "prepare_gate_thresholds",
           "prepare_regen_strategy", "DEFAULT_GATE_THRESHOLDS", "DEFAULT_REGEN_STRATEGY", "Attempt"]
