"""ctypes front end of the CPU oracle (``oracle/nsg_oracle.c``).  TEST INFRASTRUCTURE ONLY.

Imported only by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, always as
the checker or the timed CPU baseline, never as the thing measured or shipped.

The per-stream loops below restate the reference drivers: ``encode_stream`` is the
``while i < len(message)`` loop of ``code_base/arithmetic.py:112-210`` and ``decode_stream`` the
``while i < len(inp)`` loop of ``code_base/arithmetic.py:254-371`` (without the BPE-repair heuristics of
``:300-342``: a received token outside the kept top-k is reported as a divergence).
"""

from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path
from typing import Callable, List, Sequence, Tuple

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "libnsgoracle.so"

OR_OK, OR_ERR_CONFIG, OR_ERR_RANGE, OR_ERR_DIVERGE = 0, -1, -2, -3


class OrState(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64), ("bit_pos", ctypes.c_int64),
                ("ntokens", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class OrRankQuality(ctypes.Structure):
    _fields_ = [("top_k", ctypes.c_int32), ("top_p", ctypes.c_double), ("min_prob", ctypes.c_double),
                ("cap_bits", ctypes.c_int32), ("prob_temp", ctypes.c_double)]


def rank_quality(quality) -> OrRankQuality:
    """src codec quality keys (codec/arithmetic.py:345-362) -> the oracle struct (off = <=0 / <0)."""
    q = dict(quality or {})
    return OrRankQuality(int(q.get("top_k") or 0), float(q.get("top_p") or 0.0),
                         float(q["min_prob"]) if q.get("min_prob") is not None else -1.0,
                         int(q.get("cap_per_token_bits") or 0), float(q.get("prob_temp") or 0.0))


class OrTrace(ctypes.Structure):
    _fields_ = [("k", ctypes.c_int32), ("kprime", ctypes.c_int32), ("sel", ctypes.c_int32),
                ("n", ctypes.c_int32), ("token", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("S", ctypes.c_double)]


_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        fp = ctypes.POINTER(ctypes.c_float)
        i32p = ctypes.POINTER(ctypes.c_int32)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.or_exp_canon.restype = ctypes.c_double
        L.or_exp_canon.argtypes = [ctypes.c_double]
        L.or_select_cutoff_k.restype = ctypes.c_int
        L.or_select_cutoff_k.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_double,
                                         ctypes.c_int]
        L.or_init_state.argtypes = [ctypes.POINTER(OrState), ctypes.c_int]
        L.or_encode_step.restype = ctypes.c_int
        L.or_encode_step.argtypes = [fp, ctypes.c_int, i32p, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                     ctypes.c_int, u8p, ctypes.c_int64, ctypes.POINTER(OrState), i32p,
                                     ctypes.POINTER(OrTrace)]
        L.or_decode_step.restype = ctypes.c_int
        L.or_decode_step.argtypes = [fp, ctypes.c_int, i32p, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int32, ctypes.c_int, ctypes.POINTER(OrState), u8p,
                                     ctypes.POINTER(OrTrace)]
        L.or_row_sum.restype = ctypes.c_double
        L.or_row_sum.argtypes = [fp, ctypes.c_int, i32p, ctypes.c_int, ctypes.c_double, ctypes.c_double]
        dp = ctypes.POINTER(ctypes.c_double)
        L.or_encode_step_stats.restype = ctypes.c_int
        L.or_encode_step_stats.argtypes = [fp, ctypes.c_int, i32p, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                           ctypes.c_int, u8p, ctypes.c_int64, ctypes.POINTER(OrState), i32p,
                                           ctypes.POINTER(OrTrace), dp]
        L.or_rand64.restype = ctypes.c_uint64
        L.or_rand64.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64]
        L.or_sample_step.restype = ctypes.c_int
        L.or_sample_step.argtypes = [fp, ctypes.c_int, i32p, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                     ctypes.c_uint64, ctypes.c_int64, ctypes.POINTER(OrState), i32p,
                                     ctypes.POINTER(OrTrace), dp]
        L.or_rank_step.restype = ctypes.c_int
        L.or_rank_step.argtypes = [fp, ctypes.c_int, ctypes.c_double, ctypes.POINTER(OrRankQuality), ctypes.c_int,
                                   u8p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(OrState),
                                   i32p, i32p, u8p, i32p]
        L.or_np_sum.restype = ctypes.c_double
        L.or_np_sum.argtypes = [dp, ctypes.c_int64]
        L.or_rank_step64.restype = ctypes.c_int
        L.or_rank_step64.argtypes = [dp, ctypes.c_int, i32p, ctypes.c_int, ctypes.POINTER(OrRankQuality), ctypes.c_int,
                                     u8p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(OrState),
                                     i32p, i32p, u8p, i32p]
        L.or_encode_batch.restype = ctypes.c_int
        L.or_encode_batch.argtypes = [fp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, i32p, ctypes.c_int,
                                      ctypes.c_double, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_int64,
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(OrState), i32p]
        _lib = L
    return _lib


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _i32(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _u8(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def exp_canon(d: float) -> float:
    return lib().or_exp_canon(float(d))


def select_cutoff_k(probs: Sequence[float], threshold: float, topk: int) -> int:
    p = np.ascontiguousarray(probs, dtype=np.float64)
    return lib().or_select_cutoff_k(p.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), p.size,
                                   float(threshold), int(topk))


def new_state(precision: int) -> OrState:
    st = OrState()
    lib().or_init_state(ctypes.byref(st), int(precision))
    return st


def encode_step(row: np.ndarray, st: OrState, payload: np.ndarray, nbits: int, *, banned, temp: float,
                precision: int, topk: int, stats: np.ndarray = None) -> Tuple[int, int, OrTrace]:
    """One encode step; ``stats`` (float64[4], optional) accumulates (sum log p(sel), sum KL bits,
    sum entropy bits, steps) as code_base/arithmetic.py:193-199 defines them."""
    x = np.ascontiguousarray(row, dtype=np.float32)
    b = np.ascontiguousarray(banned, dtype=np.int32)
    pl = np.ascontiguousarray(payload, dtype=np.uint8)
    if pl.size == 0:
        pl = np.zeros(1, np.uint8)
    tok = ctypes.c_int32(-1)
    tr = OrTrace()
    if stats is None:
        rc = lib().or_encode_step(_fptr(x), x.size, _i32(b), b.size, 1.0 / float(temp), int(precision), int(topk),
                                  _u8(pl), int(nbits), ctypes.byref(st), ctypes.byref(tok), ctypes.byref(tr))
    else:
        rc = lib().or_encode_step_stats(_fptr(x), x.size, _i32(b), b.size, 1.0 / float(temp), int(precision),
                                        int(topk), _u8(pl), int(nbits), ctypes.byref(st), ctypes.byref(tok),
                                        ctypes.byref(tr), stats.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return rc, tok.value, tr


def decode_step(row: np.ndarray, st: OrState, token: int, is_last: bool, out_bits: np.ndarray, *, banned,
                temp: float, precision: int, topk: int) -> Tuple[int, OrTrace]:
    x = np.ascontiguousarray(row, dtype=np.float32)
    b = np.ascontiguousarray(banned, dtype=np.int32)
    tr = OrTrace()
    rc = lib().or_decode_step(_fptr(x), x.size, _i32(b), b.size, 1.0 / float(temp), int(precision), int(topk),
                              int(token), int(bool(is_last)), ctypes.byref(st), _u8(out_bits), ctypes.byref(tr))
    return rc, tr


RowFn = Callable[[int], np.ndarray]


def stats_summary(acc: np.ndarray, bits_consumed: int = None) -> dict:
    """(sum log p, sum KL, sum H, n) -> the reference's averages (arithmetic.py:212-215, sample.py:50-52)."""
    n = acc[3]
    out = {"avg_NLL": -acc[0] / n, "avg_KL": acc[1] / n, "avg_Hq": acc[2] / n}
    if bits_consumed is not None:
        out["words_per_bit"] = n / bits_consumed
    return out


def encode_stream(row_fn: RowFn, bits: Sequence[int], *, banned, temp: float, precision: int, topk: int,
                  max_steps: int = 1 << 20, sent_end=None, stats: np.ndarray = None) -> Tuple[List[int], List[OrTrace]]:
    """Encode one bit list (``code_base/arithmetic.py:112-210`` loop); ``row_fn(t)`` gives step t's logits.

    ``sent_end`` (a per-id boolean table) enables finish_sent (``:114,134-137``): after the payload, the
    top-1 token (max logit, lowest id, banned excluded) is emitted until one is sentence-ending."""
    nbits = len(bits)
    packed = np.packbits(np.asarray(bits, dtype=np.uint8), bitorder="little") if nbits else np.zeros(1, np.uint8)
    st = new_state(precision)
    toks, traces = [], []
    t = 0
    while st.bit_pos < nbits:
        if t >= max_steps:
            raise RuntimeError("oracle encode did not terminate")
        rc, tok, tr = encode_step(row_fn(t), st, packed, nbits, banned=banned, temp=temp, precision=precision,
                                  topk=topk, stats=stats)
        if rc != OR_OK:
            raise RuntimeError(f"oracle encode step {t} failed rc={rc}")
        toks.append(tok)
        traces.append(tr)
        t += 1
    if sent_end is not None:
        while True:
            if t >= max_steps:
                raise RuntimeError("oracle finish_sent did not terminate")
            row = np.asarray(row_fn(t), dtype=np.float32).copy()
            row[list(banned)] = -np.inf
            row = row + np.float32(0.0)  # -0 -> +0, as the canonical key
            tok = int(np.flatnonzero(row == row.max())[0])
            toks.append(tok)
            t += 1
            if sent_end[tok]:
                break
    return toks, traces


def encode_bits_consumed(row_fn: RowFn, bits: Sequence[int], **kw) -> int:
    """bit_pos after encoding ``bits`` (the reference's final ``i``, arithmetic.py:215)."""
    nbits = len(bits)
    packed = np.packbits(np.asarray(bits, dtype=np.uint8), bitorder="little") if nbits else np.zeros(1, np.uint8)
    st = new_state(kw["precision"])
    t = 0
    while st.bit_pos < nbits:
        rc, _, _ = encode_step(row_fn(t), st, packed, nbits, **kw)
        if rc != OR_OK:
            raise RuntimeError(f"oracle encode step {t} failed rc={rc}")
        t += 1
    return int(st.bit_pos)


def rand64(seed: int, gid: int, t: int) -> int:
    return int(lib().or_rand64(int(seed) & ((1 << 64) - 1), int(gid), int(t)))


def sample_step(row: np.ndarray, st: OrState, *, banned, temp: float, topk: int, seed: int, gid: int,
                stats: np.ndarray = None) -> Tuple[int, OrTrace]:
    x = np.ascontiguousarray(row, dtype=np.float32)
    b = np.ascontiguousarray(banned, dtype=np.int32)
    tok = ctypes.c_int32(-1)
    tr = OrTrace()
    sp = stats.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if stats is not None else None
    rc = lib().or_sample_step(_fptr(x), x.size, _i32(b), b.size, 1.0 / float(temp), int(topk),
                              int(seed) & ((1 << 64) - 1), int(gid), ctypes.byref(st), ctypes.byref(tok),
                              ctypes.byref(tr), sp)
    if rc != OR_OK:
        raise RuntimeError(f"oracle sample step failed rc={rc}")
    return tok.value, tr


def sample_stream(row_fn: RowFn, length: int, *, banned, temp: float, topk: int, seed: int, gid: int,
                  stats: np.ndarray = None) -> Tuple[List[int], List[OrTrace]]:
    """``length`` canonical sampler steps (code_base/sample.py:22-48 loop); ``row_fn(t)`` gives step t's logits."""
    st = new_state(1)
    toks, traces = [], []
    for t in range(length):
        tok, tr = sample_step(row_fn(t), st, banned=banned, temp=temp, topk=topk, seed=seed, gid=gid, stats=stats)
        toks.append(tok)
        traces.append(tr)
    return toks, traces


def sample_stats_for_tokens(row_fn: RowFn, tokens: Sequence[int], *, banned, temp: float, topk: int) -> dict:
    """The reference sampler's statistics (sample.py:31-48) for a GIVEN token sequence (e.g. the one torch
    sampled): KL and entropy depend only on the rows, NLL on the tokens."""
    acc = np.zeros(4)
    for t, tok in enumerate(tokens):
        x = np.asarray(row_fn(t), dtype=np.float64).copy()
        valid = np.ones(x.size, bool)
        valid[list(banned)] = False
        m = x[valid].max()
        lse1 = np.log(np.exp(x[valid] - m).sum())
        order = np.lexsort((np.arange(x.size), -x))
        order = order[valid[order]]
        K = order.size if topk <= 0 else min(topk, order.size)
        top = x[order[:K]] - m
        z = top / temp
        lq = z - np.log(np.exp(z).sum())
        q = np.exp(lq)
        acc[0] += (x[tok] - m) - lse1
        acc[1] += np.sum(np.where(q > 0, q * (lq - (top - lse1)), 0.0)) / 0.69315
        acc[2] += -np.sum(np.where(q > 0, q * lq, 0.0)) / 0.69315
        acc[3] += 1
    return stats_summary(acc)


def rank_encode_stream(row_fn: RowFn, payload: bytes, *, temp: float, quality) -> Tuple[List[int], List[int]]:
    """src ``encode_with_lm`` (codec/arithmetic.py:122-168): tokens and the bits each consumed."""
    pl = np.frombuffer(bytes(payload), dtype=np.uint8).copy() if payload else np.zeros(1, np.uint8)
    nbits = 8 * len(payload)
    rq = rank_quality(quality)
    st = new_state(1)
    toks, cons = [], []
    t = 0
    while st.bit_pos < nbits:
        x = np.ascontiguousarray(row_fn(t), dtype=np.float32)
        tok, c, cap = ctypes.c_int32(-1), ctypes.c_int32(0), ctypes.c_int32(0)
        rc = lib().or_rank_step(_fptr(x), x.size, 1.0 / float(temp), ctypes.byref(rq), 0, _u8(pl), nbits, -1, 0,
                                ctypes.byref(st), ctypes.byref(tok), ctypes.byref(c), None, ctypes.byref(cap))
        if rc != OR_OK:
            raise RuntimeError(f"oracle rank encode step {t} failed rc={rc}")
        toks.append(tok.value)
        cons.append(c.value)
        t += 1
    return toks, cons


def rank_decode_stream(row_fn: RowFn, tokens: Sequence[int], consumed: Sequence[int], nbits: int, *, temp: float,
                       quality) -> bytes:
    """src ``decode_with_lm`` (codec/arithmetic.py:171-231) given the consumption history."""
    rq = rank_quality(quality)
    st = new_state(1)
    out = np.zeros(max(1, (sum(consumed) + 7) // 8 + 8), dtype=np.uint8)
    for t, tok in enumerate(tokens):
        x = np.ascontiguousarray(row_fn(t), dtype=np.float32)
        cap = ctypes.c_int32(0)
        rc = lib().or_rank_step(_fptr(x), x.size, 1.0 / float(temp), ctypes.byref(rq), 1, None, 0, int(tok),
                                int(consumed[t]), ctypes.byref(st), None, None, _u8(out), ctypes.byref(cap))
        if rc != OR_OK:
            raise RuntimeError(f"oracle rank decode step {t} failed rc={rc}")
    return out.tobytes()[: nbits // 8]


def np_sum(a: np.ndarray) -> float:
    """numpy's float64 ``sum`` restated (or_np_sum): 8192-element chunks of pairwise sums, left to right."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().or_np_sum(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), a.size)


def dist_arrays(dist):
    """A ProbDist as ``_dist_to_arrays`` sees it (codec/arithmetic.py:388-398): (float64 values, int32 ids or
    None for an ndarray, dict flag)."""
    if isinstance(dist, dict):
        items = sorted(dist.items())
        return (np.array([float(p) for _, p in items], dtype=np.float64),
                np.array([int(t) for t, _ in items], dtype=np.int32), True)
    return np.ascontiguousarray(np.asarray(dist, dtype=np.float64).reshape(-1)), None, False


def _rank_step64(dist, rq, mode, pl, nbits, tok, keep, st, out_bits):
    v, ids, is_dict = dist_arrays(dist)
    otok, c, cap = ctypes.c_int32(-1), ctypes.c_int32(0), ctypes.c_int32(0)
    rc = lib().or_rank_step64(v.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), v.size,
                              _i32(ids) if ids is not None else None, int(is_dict), ctypes.byref(rq), mode,
                              _u8(pl) if pl is not None else None, nbits, tok, keep, ctypes.byref(st),
                              ctypes.byref(otok), ctypes.byref(c), _u8(out_bits) if out_bits is not None else None,
                              ctypes.byref(cap))
    return rc, otok.value, c.value


def _trim(ctx, window):
    return tuple(ctx[-window:]) if window is not None and len(ctx) > window else tuple(ctx)


def provider_encode_stream(provider, payload: bytes, *, context=(), quality=None, max_context=None):
    """``encode_with_lm`` over a ``next_token_probs`` provider (codec/arithmetic.py:122-169): each step queries
    the provider with the context trimmed to ``max_context`` (``_next_distribution``, :337-348) and ranks its
    float64 ProbDist with or_rank_step64.  Returns (tokens, bits consumed per token)."""
    pl = np.frombuffer(bytes(payload), dtype=np.uint8).copy() if payload else np.zeros(1, np.uint8)
    nbits = 8 * len(payload)
    rq = rank_quality(quality)
    st = new_state(1)
    ctx = [int(t) for t in context]
    toks, cons = [], []
    while st.bit_pos < nbits:
        rc, tok, c = _rank_step64(provider.next_token_probs(_trim(ctx, max_context)), rq, 0, pl, nbits, -1, 0, st,
                                  None)
        if rc != OR_OK:
            raise RuntimeError(f"oracle provider encode step {len(toks)} failed rc={rc}")
        toks.append(tok)
        cons.append(c)
        ctx.append(tok)
    return toks, cons


def provider_decode_stream(provider, tokens, consumed, nbits: int, *, context=(), quality=None, max_context=None):
    """``decode_with_lm`` over a provider (codec/arithmetic.py:172-231) given the consumption history."""
    rq = rank_quality(quality)
    st = new_state(1)
    out = np.zeros(max(1, (sum(consumed) + 7) // 8 + 8), dtype=np.uint8)
    ctx = [int(t) for t in context]
    for t, tok in enumerate(tokens):
        rc, _, _ = _rank_step64(provider.next_token_probs(_trim(ctx, max_context)), rq, 1, None, 0, int(tok),
                                int(consumed[t]), st, out)
        if rc != OR_OK:
            raise RuntimeError(f"oracle provider decode step {t} failed rc={rc}")
        ctx.append(int(tok))
    return out.tobytes()[: nbits // 8]


def decode_stream(row_fn: RowFn, tokens: Sequence[int], *, banned, temp: float, precision: int,
                  topk: int) -> Tuple[List[int], List[OrTrace]]:
    """Decode a token list (``code_base/arithmetic.py:254-371`` loop) into the full emitted bit list."""
    st = new_state(precision)
    out = np.zeros((len(tokens) * max(precision, 1) + 7) // 8 + 8, dtype=np.uint8)
    traces = []
    for t, tok in enumerate(tokens):
        rc, tr = decode_step(row_fn(t), st, int(tok), t == len(tokens) - 1, out, banned=banned, temp=temp,
                             precision=precision, topk=topk)
        if rc != OR_OK:
            raise RuntimeError(f"oracle decode step {t} failed rc={rc}")
        traces.append(tr)
    bits = np.unpackbits(out, bitorder="little")[: st.bit_pos].astype(np.int64).tolist()
    return bits, traces
