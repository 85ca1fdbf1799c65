"""Batched arithmetic-coding sessions on the HIP coder (``libnsgcoder.so``).

A session owns the device buffers of B independent streams and launches one coder step per call on the
current torch stream.  It is the batched replacement of the per-stream loops in
``code_base/arithmetic.py:112-210`` (encode) and ``:254-371`` (decode): the caller supplies the ``[B, ld]``
logits of each step (a GPT-2 forward, or synthetic rows) and the kernel does sort/softmax/CDF/interval
work for all B streams at once.

All device state lives in torch tensors (PyTorch is plumbing here); the arithmetic runs only in the HIP
kernel.  There is no CPU fallback.
"""

from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .codec.errors import ArithmeticRangeError, DecodeDivergenceError
from .exceptions import ConfigurationError


def _torch():
    import torch

    return torch


def _ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream_handle():
    torch = _torch()
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def row_stride(vocab: int, dtype: str) -> int:
    """Padded logits row stride the kernel wants: a multiple of 64 elements (16-byte vectors, 256-B rows)."""
    _ = dtype
    return ((vocab + 63) // 64) * 64


@dataclass(frozen=True)
class CoderParams:
    """Coder parameters of ``encode_arithmetic``/``decode_arithmetic`` (``code_base/arithmetic.py:78-88``)."""

    vocab: int
    precision: int = 26
    temp: float = 0.9
    topk: int = 300
    dtype: str = "f32"  # logits dtype: "f32" or "f16"; "f64": a provider's probability rows (rank coder only)
    banned: Optional[Sequence[int]] = None  # default: (vocab-1, 628) as arithmetic.py:124-125

    def banned_ids(self) -> List[int]:
        if self.banned is not None:
            return [int(b) for b in self.banned]
        return [self.vocab - 1, 628]

    @property
    def dtype_code(self) -> int:
        if self.dtype == "f32":
            return _lib.NS_DTYPE_F32
        if self.dtype == "f16":
            return _lib.NS_DTYPE_F16
        if self.dtype == "f64":
            return _lib.NS_DTYPE_F64
        raise ConfigurationError(f"unsupported logits dtype {self.dtype!r}")

    @property
    def torch_dtype(self):
        torch = _torch()
        return {"f16": torch.float16, "f64": torch.float64}.get(self.dtype, torch.float32)

    def validate(self) -> None:
        if self.vocab < 2:
            raise ConfigurationError("vocab must be >= 2")
        if not 1 <= self.precision <= 60:
            raise ConfigurationError("precision must be within [1, 60]")
        if not self.temp > 0:
            raise ConfigurationError("temperature must be positive")
        if self.topk < 1:
            raise ConfigurationError("topk must be positive")
        if len(self.banned_ids()) > _lib.NS_MAX_BANNED:
            raise ConfigurationError(f"at most {_lib.NS_MAX_BANNED} banned ids")


_DEFERRED: List[tuple] = []  # (device, handle) of contexts closed during a graph capture


def _destroy(device: int, h) -> None:
    torch = _torch()
    if torch.cuda.is_available():  # launches still queued may read the context's buffers
        torch.cuda.synchronize(device)
    _lib.lib().ns_destroy(h)


def _drain_deferred() -> None:
    torch = _torch()
    if not _DEFERRED or (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
        return
    while _DEFERRED:
        dev, h = _DEFERRED.pop()
        _destroy(dev, h)


class CoderContext:
    """Owns an ``ns_ctx`` (device, vocab, precision, dtype, max batch)."""

    def __init__(self, params: CoderParams, max_batch: int, device: Optional[int] = None):
        params.validate()
        torch = _torch()
        if not torch.cuda.is_available():
            raise _lib.NativeLibraryError("the HIP coder needs a ROCm GPU (torch.cuda.is_available() is False)")
        _drain_deferred()
        self.params = params
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.max_batch = int(max_batch)
        L = _lib.lib()
        vocab_valid = params.vocab - len({b for b in params.banned_ids() if 0 <= b < params.vocab})
        self.K = min(params.topk, vocab_valid)
        self.wide = self.K > L.ns_max_topk(params.dtype_code)  # large top-k: multi-kernel wide path
        handle = L.ns_create(self.device, self.max_batch, params.vocab, max(1, self.K), params.precision,
                             params.dtype_code)
        if not handle:
            raise _lib.NativeLibraryError(f"ns_create failed: {L.ns_last_error(None).decode()}")
        self._h = ctypes.c_void_p(handle)
        self._banned = (ctypes.c_int32 * max(1, len(params.banned_ids())))(*params.banned_ids())
        self._nbanned = len(params.banned_ids())

    def check(self, rc: int, what: str) -> None:
        if rc != _lib.NS_OK:
            msg = _lib.lib().ns_last_error(self._h).decode()
            if rc == _lib.NS_ERR_CONFIG:
                raise ConfigurationError(f"{what}: {msg}")
            raise _lib.NativeLibraryError(f"{what}: rc={rc}: {msg}")

    def set_sentence_end(self, table) -> None:
        """Register a device uint8 table [vocab] (nonzero = sentence-ending token) for finish_sent."""
        torch = _torch()
        if table is None:
            self._sent_end = None
            self.check(_lib.lib().ns_set_sentence_end(self._h, ctypes.c_void_p(0)), "ns_set_sentence_end")
            return
        t = torch.as_tensor(table, dtype=torch.uint8).to(torch.device("cuda", self.device)).contiguous()
        if t.numel() != self.params.vocab:
            raise ConfigurationError("sentence-end table must have one entry per vocabulary id")
        self._sent_end = t  # keep alive: the library holds the raw pointer
        self.check(_lib.lib().ns_set_sentence_end(self._h, _ptr(t)), "ns_set_sentence_end")

    def counters(self) -> List[int]:
        out = (ctypes.c_uint64 * 4)()
        self.check(_lib.lib().ns_read_counters(self._h, out), "ns_read_counters")
        return [int(v) for v in out]

    def close(self) -> None:
        """Release the context.  Launches still queued may read its buffers, so the device is synchronised
        first -- except while the current stream is capturing a hipGraph (a garbage-collected context during
        a capture): a device-wide sync or a free there would invalidate the capture, so the handle is parked
        and destroyed by the next close() or context creation outside a capture."""
        h = getattr(self, "_h", None)
        if not h:
            return
        self._h = None
        torch = _torch()
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            _DEFERRED.append((self.device, h))
            return
        _destroy(self.device, h)
        _drain_deferred()

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


def _check_logits(ctx: "CoderContext", B: int, logits) -> None:
    """Host-side validation before any launch that reads a logit matrix: dtype of the context, [B, ld] with
    unit column stride, ld >= vocab, on this context's device (a mismatch would make the kernel misread rows
    or read past their end)."""
    p = ctx.params
    if logits.dtype != p.torch_dtype or logits.dim() != 2 or logits.shape[0] != B:
        raise ConfigurationError(f"logits must be [{B}, ld] {p.dtype}")
    if logits.stride(1) != 1 or logits.shape[1] < p.vocab or logits.stride(0) < p.vocab or not logits.is_cuda:
        raise ConfigurationError("logits must be contiguous rows on the GPU with ld >= vocab")
    if logits.device.index != ctx.device:
        raise ConfigurationError(f"logits on cuda:{logits.device.index}, coder context on cuda:{ctx.device}")


def _rank_rows(ctx: "CoderContext", B: int, rows, q):
    """The device matrix a rank step reads: logits as they are (checked), or a provider step's
    :class:`~neuralsteganography_amd.codec.distribution.ProbRows` registered with ``ns_set_rank_rows`` (the
    reference's quality errors raised on the host first)."""
    if not getattr(rows, "prob_rows", False):
        if ctx.params.dtype == "f64":
            # an f64 context reads rk_count / rk_idmap registered for ProbRows: a plain matrix would leave it reading
            # an earlier step's (possibly freed) tensors
            raise ConfigurationError("a coder context of dtype 'f64' takes provider ProbRows only")
        _check_logits(ctx, B, rows)
        return rows
    if ctx.params.dtype != "f64":
        raise ConfigurationError("provider probability rows need a coder context of dtype 'f64'")
    if rows.ncols > ctx.params.vocab:
        raise ConfigurationError(f"a row of {rows.ncols} entries exceeds the context's {ctx.params.vocab}")
    rows.check_quality(q)
    _check_logits(ctx, B, rows.values)
    idm = rows.idmap
    ctx.check(_lib.lib().ns_set_rank_rows(ctx._h, _ptr(rows.count), _ptr(idm), idm.stride(0) if idm is not None else 0,
                                          int(rows.dict_rows)), "ns_set_rank_rows")
    return rows.values


def _state_tensor(B: int, device):
    torch = _torch()
    return torch.zeros((B, 4), dtype=torch.int64, device=device)


def _state_fields(state) -> dict:
    """Host view of [B,4] int64 state rows: lo, hi, bit_pos, ntokens, flags."""
    s = state.cpu().numpy()
    w32 = s.view(np.int32).reshape(s.shape[0], 8)
    return {"lo": s[:, 0].view(np.uint64), "hi": s[:, 1].view(np.uint64), "bit_pos": s[:, 2],
            "ntokens": w32[:, 6], "flags": w32[:, 7].view(np.uint32)}


def _stats_rows(acc: np.ndarray, bits_consumed: Optional[np.ndarray] = None) -> List[dict]:
    """[B, 4] accumulators (sum log p, sum KL bits, sum H bits, n) -> the reference's averages per stream
    (``code_base/arithmetic.py:212-215``, ``sample.py:50-52``); NaN where a stream had no counted step."""
    out = []
    for i in range(acc.shape[0]):
        n = acc[i, 3]
        d = {"avg_NLL": -acc[i, 0] / n if n else math.nan, "avg_KL": acc[i, 1] / n if n else math.nan,
             "avg_Hq": acc[i, 2] / n if n else math.nan}
        if bits_consumed is not None:
            d["words_per_bit"] = n / bits_consumed[i] if bits_consumed[i] else math.nan
        out.append(d)
    return out


def _bit_array(bits) -> np.ndarray:
    """A payload bit list as uint8 (nonzero = 1 after packing).  Python lists go through ``bytes`` (one C pass,
    ≈3x faster than numpy's per-object conversion: 4,096 KiB-payload lists are ≈1 s of host time otherwise)."""
    if isinstance(bits, (list, tuple)):
        try:
            return np.frombuffer(bytes(bits), dtype=np.uint8)
        except (ValueError, TypeError):
            pass
    return np.asarray(bits, dtype=np.uint8)


def _rows_to_lists(dev_rows, lengths) -> List[List[int]]:
    """Row i's first lengths[i] entries of a device [B, cap] int array as Python int lists: only the columns in
    use cross PCIe (the history buffer is sized for the KV budget, far wider than a finished job's tokens), and
    the rows become lists in one conversion."""
    lengths = np.asarray(lengths, dtype=np.int64)
    n = int(lengths.max(initial=0))
    if n == 0:
        return [[] for _ in range(dev_rows.shape[0])]
    rows = dev_rows[:, :n].cpu().numpy().tolist()
    return [r[:k] if k < n else r for r, k in zip(rows, lengths.tolist())]


def _bit_rows_to_lists(dev_bytes, nbits) -> List[List[int]]:
    """Row i's first nbits[i] bits (LSB-first bytes on the device) as Python int lists."""
    nbits = np.asarray(nbits, dtype=np.int64)
    nb = int(nbits.max(initial=0))
    if nb == 0:
        return [[] for _ in range(dev_bytes.shape[0])]
    host = dev_bytes[:, : (nb + 7) // 8].cpu().numpy()
    rows = np.unpackbits(host, axis=1, bitorder="little")[:, :nb].tolist()
    return [r[:k] if k < nb else r for r, k in zip(rows, nbits.tolist())]


class EncodeSession:
    """B streams being encoded; call :meth:`step` once per generated token with that step's logits.

    ``stats=True`` also accumulates the statistics ``encode_arithmetic`` returns (avg_NLL, avg_KL,
    words_per_bit, avg_Hq; ``code_base/arithmetic.py:193-217``) on the device -- within a float64
    tolerance of the reference, not bit-exact -- at the cost of a heavier kernel build."""

    def __init__(self, ctx: CoderContext, payload_bits: Sequence[Sequence[int]], max_tokens: Optional[int] = None,
                 stats: bool = False, payload_stride: Optional[int] = None):
        torch = _torch()
        self.ctx = ctx
        self.B = len(payload_bits)
        if self.B < 1 or self.B > ctx.max_batch:
            raise ConfigurationError(f"batch {self.B} outside [1, {ctx.max_batch}]")
        dev = torch.device("cuda", ctx.device)
        self.nbits_host = np.asarray([len(b) for b in payload_bits], dtype=np.int64)
        stride = max(1, int((self.nbits_host.max() + 7) // 8), int(payload_stride or 0))
        pl = np.zeros((self.B, stride), dtype=np.uint8)
        for i, bits in enumerate(payload_bits):
            if len(bits):
                packed = np.packbits(_bit_array(bits), bitorder="little")
                pl[i, : packed.size] = packed
        self.payload = torch.from_numpy(pl).to(dev)
        self.nbits = torch.from_numpy(self.nbits_host).to(dev)
        self.state = _state_tensor(self.B, dev)
        ctx.check(_lib.lib().ns_init_state(ctx._h, _ptr(self.state), self.B, _stream_handle()), "ns_init_state")
        self.out_token = torch.zeros(self.B, dtype=torch.int32, device=dev)
        cap = max_tokens if max_tokens is not None else int(2 * self.nbits_host.max() + 64)
        self.hist = torch.full((self.B, cap), -1, dtype=torch.int32, device=dev)
        self.trace = None
        self.steps = 0
        self.stats_acc = torch.zeros((self.B, 4), dtype=torch.float64, device=dev) if stats else None

    def enable_trace(self):
        torch = _torch()
        self.trace = torch.zeros((self.B, 4), dtype=torch.int64, device=self.state.device)
        return self.trace

    def stats(self) -> List[dict]:
        """Per-stream avg_NLL, avg_KL, words_per_bit, avg_Hq (as ``encode_arithmetic`` returns them)."""
        if self.stats_acc is None:
            raise ConfigurationError("the session was created without stats=True")
        return _stats_rows(self.stats_acc.cpu().numpy(), self.fields()["bit_pos"])

    def step(self, logits, *, force_exact: bool = False, finish_sent: bool = False, diag_flags: int = 0):
        """One coder step on ``logits`` ([B, ld] contiguous rows, ld = :func:`row_stride`).

        ``finish_sent``: once a stream's payload is consumed it keeps emitting top-1 tokens until a
        sentence-ending one (needs :meth:`CoderContext.set_sentence_end`).  ``diag_flags``
        (NS_STEP_DIAG_*) are for phase timing only: such a step advances no state."""
        p = self.ctx.params
        self._check_logits(logits)
        flags = (_lib.NS_STEP_FORCE_EXACT_SUM if force_exact else 0) | int(diag_flags)
        if finish_sent:
            flags |= _lib.NS_STEP_FINISH_SENT
        L = _lib.lib()
        if self.stats_acc is not None:
            self.ctx.check(L.ns_set_stats(self.ctx._h, _ptr(self.stats_acc)), "ns_set_stats")
        rc = L.ns_encode_step(
            self.ctx._h, _ptr(logits), logits.stride(0), self.B, _ptr(self.payload), self.payload.stride(0),
            _ptr(self.nbits), _ptr(self.state), _ptr(self.out_token), _ptr(self.hist), self.hist.shape[1],
            float(p.temp), int(p.topk), self.ctx._banned, self.ctx._nbanned, _ptr(self.trace), flags,
            _stream_handle())
        if self.stats_acc is not None:
            L.ns_set_stats(self.ctx._h, ctypes.c_void_p(0))
        self.ctx.check(rc, "ns_encode_step")
        self.steps += 1
        return self.out_token

    def _check_logits(self, logits) -> None:
        _check_logits(self.ctx, self.B, logits)

    def all_done(self) -> bool:
        return bool(np.all(_state_fields(self.state)["flags"] & _lib.NS_ST_DONE))

    def mark_done(self, streams: Sequence[int]) -> None:
        """Stop ``streams`` (host decision, e.g. the reference's '<eos>' text check, arithmetic.py:208-210)."""
        torch = _torch()
        idx = torch.tensor(list(streams), device=self.state.device, dtype=torch.long)
        w = self.state.view(torch.int32)
        w[idx, 7] = w[idx, 7] | _lib.NS_ST_DONE

    def ensure_history(self, steps_ahead: int) -> None:
        """Grow the device token history so ``steps_ahead`` more steps fit (finish_sent tails are unbounded)."""
        need = int(self.fields()["ntokens"].max(initial=0)) + int(steps_ahead)
        cap = self.hist.shape[1]
        if need <= cap:
            return
        torch = _torch()
        new = torch.full((self.B, max(need, 2 * cap)), -1, dtype=torch.int32, device=self.hist.device)
        new[:, :cap] = self.hist
        self.hist = new

    def fields(self) -> dict:
        return _state_fields(self.state)

    # ---------------------------------------------------------------- slots (lm/slots.py: refill, compaction)
    def load_slots(self, slots: Sequence[int], payload_bits: Sequence[Sequence[int]]) -> None:
        """Start new payloads in ``slots`` (rows of this session): payload row, bit count, a fresh coder state
        (``ns_init_state``'s values) and, with stats, zeroed accumulators.  The token history row is reused from
        position 0 (only the first ``ntokens`` entries of a row are ever read)."""
        torch = _torch()
        n = len(slots)
        if n == 0:
            return
        stride = self.payload.shape[1]
        pl = np.zeros((n, stride), dtype=np.uint8)
        nb = np.zeros(n, dtype=np.int64)
        for i, bits in enumerate(payload_bits):
            nb[i] = len(bits)
            if len(bits):
                packed = np.packbits(_bit_array(bits), bitorder="little")
                if packed.size > stride:
                    raise ConfigurationError("payload longer than the session's payload stride")
                pl[i, : packed.size] = packed
        dev = self.state.device
        idx = torch.as_tensor(np.asarray(slots, dtype=np.int64), device=dev)
        self.payload[idx] = torch.from_numpy(pl).to(dev)
        self.nbits[idx] = torch.from_numpy(nb).to(dev)
        self.nbits_host[np.asarray(slots)] = nb
        self.state[idx] = self.init_row().expand(n, 4)
        if self.stats_acc is not None:
            self.stats_acc[idx] = 0

    def init_row(self):
        """[1, 4] int64: the state ``ns_init_state`` writes (lo 0, hi 2^precision, bit_pos 0, ntokens | flags 0)."""
        torch = _torch()
        return torch.tensor([[0, 1 << self.ctx.params.precision, 0, 0]], dtype=torch.int64, device=self.state.device)

    def park_slots(self, slots: Sequence[int]) -> None:
        """Mark ``slots`` finished (NS_ST_DONE): the coder step and the decode attention skip them (empty slots)."""
        if len(slots) == 0:
            return
        torch = _torch()
        idx = torch.as_tensor(np.asarray(slots, dtype=np.int64), device=self.state.device)
        w = self.state.view(torch.int32)
        w[idx, 7] = w[idx, 7] | _lib.NS_ST_DONE

    def compact(self, keep: Sequence[int]) -> None:
        """Keep rows ``keep`` (in that order) of every per-stream buffer: the session now has len(keep) streams."""
        torch = _torch()
        idx = torch.as_tensor(np.asarray(keep, dtype=np.int64), device=self.state.device)
        for name in ("payload", "nbits", "state", "out_token", "hist", "stats_acc", "trace"):
            t = getattr(self, name)
            if t is not None:
                setattr(self, name, t.index_select(0, idx).contiguous())
        self.nbits_host = self.nbits_host[np.asarray(keep, dtype=np.int64)]
        self.B = len(keep)

    def raise_errors(self) -> None:
        f = self.fields()["flags"]
        bad = np.nonzero(f & _lib.NS_ST_ERR_RANGE)[0]
        if bad.size:
            raise ArithmeticRangeError(f"streams {bad.tolist()[:8]} found no CDF bucket for the payload index")

    def tokens(self) -> List[List[int]]:
        self.raise_errors()
        f = self.fields()
        if int(f["ntokens"].max(initial=0)) > self.hist.shape[1]:
            raise ConfigurationError("token history overflow: raise max_tokens")
        return _rows_to_lists(self.hist, f["ntokens"])

    def trace_rows(self) -> np.ndarray:
        """Last-step trace as a structured host array (k, kprime, sel, n, token, exact, S)."""
        raw = self.trace.cpu().numpy()
        w = raw.view(np.int32).reshape(self.B, 8)
        return np.rec.fromarrays([w[:, 0], w[:, 1], w[:, 2], w[:, 3], w[:, 4], w[:, 5], raw[:, 3].view(np.float64)],
                                 names="k,kprime,sel,n,token,exact,S")


class DecodeSession:
    """B received token streams (ragged) being decoded back to bits."""

    def __init__(self, ctx: CoderContext, token_lists: Sequence[Sequence[int]]):
        torch = _torch()
        self.ctx = ctx
        self.B = len(token_lists)
        if self.B < 1 or self.B > ctx.max_batch:
            raise ConfigurationError(f"batch {self.B} outside [1, {ctx.max_batch}]")
        dev = torch.device("cuda", ctx.device)
        self.lens = np.asarray([len(t) for t in token_lists], dtype=np.int64)
        self.T = int(self.lens.max(initial=0))
        tok = np.zeros((max(self.T, 1), self.B), dtype=np.int32)
        last = np.zeros((max(self.T, 1), self.B), dtype=np.uint8)
        act = np.zeros((max(self.T, 1), self.B), dtype=np.uint8)
        for i, tl in enumerate(token_lists):
            n = len(tl)
            if n:
                tok[:n, i] = np.asarray(tl, dtype=np.int32)
                last[n - 1, i] = 1
                act[:n, i] = 1
        self.tok = torch.from_numpy(tok).to(dev)
        self.last = torch.from_numpy(last).to(dev)
        self.act = torch.from_numpy(act).to(dev)
        P = ctx.params.precision
        self.out_stride = int((self.T * P + P + 7) // 8 + 8)
        self.out_bits = torch.zeros((self.B, self.out_stride), dtype=torch.uint8, device=dev)
        self.state = _state_tensor(self.B, dev)
        ctx.check(_lib.lib().ns_init_state(ctx._h, _ptr(self.state), self.B, _stream_handle()), "ns_init_state")
        self.trace = None
        self.t = 0

    def enable_trace(self):
        torch = _torch()
        self.trace = torch.zeros((self.B, 4), dtype=torch.int64, device=self.state.device)
        return self.trace

    def step(self, logits, *, force_exact: bool = False) -> None:
        p = self.ctx.params
        if self.t >= self.T:
            raise ConfigurationError("all tokens already decoded")
        t = self.t
        _check_logits(self.ctx, self.B, logits)
        flags = _lib.NS_STEP_FORCE_EXACT_SUM if force_exact else 0
        rc = _lib.lib().ns_decode_step(
            self.ctx._h, _ptr(logits), logits.stride(0), self.B, _ptr(self.tok[t]), _ptr(self.last[t]),
            _ptr(self.act[t]), _ptr(self.state), _ptr(self.out_bits), self.out_stride, float(p.temp),
            int(p.topk), self.ctx._banned, self.ctx._nbanned, _ptr(self.trace), flags, _stream_handle())
        self.ctx.check(rc, "ns_decode_step")
        self.t += 1

    def step_static(self, logits, *, force_exact: bool = False):
        """:meth:`step` with the token index on the device (``d_t``): the step's token / last / active rows are
        gathered into fixed buffers by the device, so one captured hipGraph serves every step.  Returns the
        token buffer (the LM's next input)."""
        torch = _torch()
        _check_logits(self.ctx, self.B, logits)
        if getattr(self, "d_t", None) is None:
            self.d_t = torch.full((1,), self.t, dtype=torch.long, device=self.state.device)
            self.tok_s = torch.empty((1, self.B), dtype=self.tok.dtype, device=self.state.device)
            self.last_s = torch.empty((1, self.B), dtype=self.last.dtype, device=self.state.device)
            self.act_s = torch.empty((1, self.B), dtype=self.act.dtype, device=self.state.device)
        torch.index_select(self.tok, 0, self.d_t, out=self.tok_s)
        torch.index_select(self.last, 0, self.d_t, out=self.last_s)
        torch.index_select(self.act, 0, self.d_t, out=self.act_s)
        p = self.ctx.params
        flags = _lib.NS_STEP_FORCE_EXACT_SUM if force_exact else 0
        rc = _lib.lib().ns_decode_step(
            self.ctx._h, _ptr(logits), logits.stride(0), self.B, _ptr(self.tok_s), _ptr(self.last_s),
            _ptr(self.act_s), _ptr(self.state), _ptr(self.out_bits), self.out_stride, float(p.temp),
            int(p.topk), self.ctx._banned, self.ctx._nbanned, _ptr(self.trace), flags, _stream_handle())
        self.ctx.check(rc, "ns_decode_step")
        self.d_t += 1
        return self.tok_s[0]

    def bits(self) -> List[List[int]]:
        f = _state_fields(self.state)
        bad = np.nonzero(f["flags"] & _lib.NS_ST_ERR_DIVERGE)[0]
        if bad.size:
            raise DecodeDivergenceError(f"streams {bad.tolist()[:8]}: received token outside the kept top-k")
        return _bit_rows_to_lists(self.out_bits, f["bit_pos"])


def encode_batch(ctx: CoderContext, payload_bits: Sequence[Sequence[int]], logits_fn, *, max_steps: int = 1 << 20,
                 check_every: int = 32, force_exact: bool = False, finish_sent: bool = False,
                 return_stats: bool = False):
    """Run encode steps until every stream has consumed its payload; ``logits_fn(step, last_tokens)``
    returns the ``[B, ld]`` logits of that step.  ``return_stats=True`` returns ``(tokens, stats)`` with the
    per-stream statistics of ``encode_arithmetic`` (see :meth:`EncodeSession.stats`)."""
    sess = EncodeSession(ctx, payload_bits, stats=return_stats)
    last = sess.out_token
    for t in range(max_steps):
        if t % check_every == 0:
            if sess.all_done():
                break
            sess.ensure_history(check_every)
        last = sess.step(logits_fn(t, last), force_exact=force_exact, finish_sent=finish_sent)
    else:
        raise ConfigurationError("encode did not finish within max_steps")
    if return_stats:
        return sess.tokens(), sess.stats()
    return sess.tokens()


def decode_batch(ctx: CoderContext, token_lists: Sequence[Sequence[int]], logits_fn, *,
                 force_exact: bool = False) -> List[List[int]]:
    sess = DecodeSession(ctx, token_lists)
    for t in range(sess.T):
        sess.step(logits_fn(t, sess.tok[t]), force_exact=force_exact)
    return sess.bits()


class SampleSession:
    """B independent non-stego sampling streams (``code_base/sample.py:22-48``), one HIP launch per token.

    Draws are counter based (``ns_sample_step``): token t of stream b uses splitmix64(seed, stream_offset + b,
    t), so a run is reproducible and shardable (a rank passes its first global stream id as
    ``stream_offset``).  ``topk <= 0`` samples from every id.  Statistics (avg_NLL, avg_KL, avg_Hq of
    ``sample()``) are accumulated on the device when ``stats=True``."""

    def __init__(self, ctx: CoderContext, B: int, *, seed: int, topk: int, temp: float, stream_offset: int = 0,
                 max_tokens: int = 1024, stats: bool = True):
        torch = _torch()
        if B < 1 or B > ctx.max_batch:
            raise ConfigurationError(f"batch {B} outside [1, {ctx.max_batch}]")
        if not temp > 0:
            raise ConfigurationError("temperature must be positive")
        self.ctx, self.B = ctx, int(B)
        self.seed = int(seed) & ((1 << 64) - 1)
        self.topk, self.temp, self.stream_offset = int(topk), float(temp), int(stream_offset)
        dev = torch.device("cuda", ctx.device)
        self.state = _state_tensor(self.B, dev)
        ctx.check(_lib.lib().ns_init_state(ctx._h, _ptr(self.state), self.B, _stream_handle()), "ns_init_state")
        self.out_token = torch.zeros(self.B, dtype=torch.int32, device=dev)
        self.hist = torch.full((self.B, int(max_tokens)), -1, dtype=torch.int32, device=dev)
        self.stats_acc = torch.zeros((self.B, 4), dtype=torch.float64, device=dev) if stats else None
        self.trace = None
        self.steps = 0

    def enable_trace(self):
        torch = _torch()
        self.trace = torch.zeros((self.B, 4), dtype=torch.int64, device=self.state.device)
        return self.trace

    def step(self, logits, *, diag_flags: int = 0):
        _check_logits(self.ctx, self.B, logits)
        if self.steps >= self.hist.shape[1]:
            raise ConfigurationError("token history full: raise max_tokens")
        rc = _lib.lib().ns_sample_step(
            self.ctx._h, _ptr(logits), logits.stride(0), self.B, ctypes.c_uint64(self.seed), self.stream_offset,
            _ptr(self.state), _ptr(self.out_token), _ptr(self.hist), self.hist.shape[1], self.temp, self.topk,
            self.ctx._banned, self.ctx._nbanned, _ptr(self.stats_acc), _ptr(self.trace), int(diag_flags),
            _stream_handle())
        self.ctx.check(rc, "ns_sample_step")
        self.steps += 1
        return self.out_token

    def trace_rows(self) -> np.ndarray:
        t = self.trace.cpu().numpy().view(np.int32).reshape(self.B, 8)
        return np.rec.fromarrays([t[:, 0], t[:, 1], t[:, 2], t[:, 3], t[:, 4]], names="k,kprime,sel,n,token")

    def tokens(self) -> List[List[int]]:
        n = min(self.steps, self.hist.shape[1])
        return _rows_to_lists(self.hist, np.full(self.B, n))

    def stats(self) -> List[dict]:
        if self.stats_acc is None:
            raise ConfigurationError("the session was created without stats=True")
        return _stats_rows(self.stats_acc.cpu().numpy())


def sample_batch(ctx: CoderContext, B: int, length: int, logits_fn, *, seed: int, topk: int, temp: float,
                 stream_offset: int = 0, stats: bool = True):
    """``length`` sampler steps for B streams; ``logits_fn(step, last_tokens)`` returns the ``[B, ld]``
    logits.  Returns ``(tokens, stats)`` (stats None when ``stats=False``)."""
    sess = SampleSession(ctx, B, seed=seed, topk=topk, temp=temp, stream_offset=stream_offset,
                         max_tokens=max(1, length), stats=stats)
    last = sess.out_token
    for t in range(length):
        last = sess.step(logits_fn(t, last))
    return sess.tokens(), (sess.stats() if stats else None)


class StreamingDecodeSession:
    """Decode with the received tokens supplied step by step by the host (``code_base/arithmetic.py:254-371``
    loop, where the token list can change mid-stream: the BPE repair of ``:300-342`` inserts and deletes
    tokens).  A stream whose token falls outside the kept top-k' is flagged NS_ST_ERR_DIVERGE with its state
    untouched and its ranked kept ids exported; :meth:`clear` re-arms it for a re-issued step."""

    def __init__(self, ctx: CoderContext, B: int, max_tokens: int):
        torch = _torch()
        if B < 1 or B > ctx.max_batch:
            raise ConfigurationError(f"batch {B} outside [1, {ctx.max_batch}]")
        self.ctx, self.B = ctx, int(B)
        dev = torch.device("cuda", ctx.device)
        self.dev = dev
        P = ctx.params.precision
        self.out_stride = int((max(1, max_tokens) * P + P + 7) // 8 + 8)
        self.out_bits = torch.zeros((self.B, self.out_stride), dtype=torch.uint8, device=dev)
        self.state = _state_tensor(self.B, dev)
        ctx.check(_lib.lib().ns_init_state(ctx._h, _ptr(self.state), self.B, _stream_handle()), "ns_init_state")
        self.rank_stride = int(ctx.K) + 1
        self.ranked = torch.full((self.B, self.rank_stride), -1, dtype=torch.int32, device=dev)

    def _grow(self, need_bits: int) -> None:
        torch = _torch()
        need = (need_bits + 7) // 8 + 8
        if need <= self.out_stride:
            return
        new = torch.zeros((self.B, max(need, 2 * self.out_stride)), dtype=torch.uint8, device=self.dev)
        new[:, : self.out_stride] = self.out_bits
        self.out_bits, self.out_stride = new, new.shape[1]

    def step(self, logits, tokens: Sequence[int], is_last: Sequence[bool], active: Sequence[bool]) -> None:
        torch = _torch()
        p = self.ctx.params
        _check_logits(self.ctx, self.B, logits)
        f = _state_fields(self.state)
        self._grow(int(f["bit_pos"].max(initial=0)) + 2 * p.precision)
        tok = torch.tensor(np.asarray(tokens, dtype=np.int32), device=self.dev)
        last = torch.tensor(np.asarray(is_last, dtype=np.uint8), device=self.dev)
        act = torch.tensor(np.asarray(active, dtype=np.uint8), device=self.dev)
        L = _lib.lib()
        self.ctx.check(L.ns_set_rank_export(self.ctx._h, _ptr(self.ranked), self.rank_stride), "ns_set_rank_export")
        rc = L.ns_decode_step(self.ctx._h, _ptr(logits), logits.stride(0), self.B, _ptr(tok), _ptr(last), _ptr(act),
                              _ptr(self.state), _ptr(self.out_bits), self.out_stride, float(p.temp), int(p.topk),
                              self.ctx._banned, self.ctx._nbanned, ctypes.c_void_p(0), 0, _stream_handle())
        L.ns_set_rank_export(self.ctx._h, ctypes.c_void_p(0), 0)
        self.ctx.check(rc, "ns_decode_step")

    def diverged(self) -> List[int]:
        f = _state_fields(self.state)["flags"]
        return np.nonzero(f & _lib.NS_ST_ERR_DIVERGE)[0].tolist()

    def ranked_ids(self, b: int) -> List[int]:
        row = self.ranked[b].cpu().numpy()
        end = np.nonzero(row < 0)[0]
        return row[: int(end[0]) if end.size else row.size].astype(np.int64).tolist()

    def clear(self, streams: Sequence[int]) -> None:
        """Drop the divergence / done flags of ``streams`` (their lo/hi/bit_pos were left untouched)."""
        if not streams:
            return
        torch = _torch()
        w = self.state.view(torch.int32)
        idx = torch.tensor(list(streams), device=self.dev, dtype=torch.long)
        keep = ~(_lib.NS_ST_ERR_DIVERGE | _lib.NS_ST_DONE)
        w[idx, 7] = w[idx, 7] & keep

    def bits(self) -> List[List[int]]:
        f = _state_fields(self.state)
        return _bit_rows_to_lists(self.out_bits, f["bit_pos"])


def rank_quality(quality) -> "_lib.NsRankQuality":
    """src codec quality (``lm/arithmetic.py:77-95`` ``_normalise_quality``: topk/top_k, top_p, min_prob,
    cap_per_token_bits / cap_bits_per_token) -> ``ns_rank_quality``."""
    q = {}
    for key, value in dict(quality or {}).items():
        if value is None:
            continue
        k = key.replace("-", "_").lower()
        if k in ("topk", "top_k"):
            q["top_k"] = int(value)
        elif k in ("topp", "top_p"):
            q["top_p"] = float(value)
        elif k in ("minprob", "min_prob"):
            q["min_prob"] = float(value)
        elif k in ("cap_per_token_bits", "cap_bits_per_token"):
            q["cap"] = int(value)
        elif k == "prob_temp":  # crypto quality LM (crypto/quality.py:57-64): temperature on probabilities
            q["prob_temp"] = float(value)
    if "top_k" in q and q["top_k"] <= 0:
        raise ConfigurationError("top_k must be positive")
    if "top_p" in q and not 0 < q["top_p"] <= 1:
        raise ConfigurationError("top_p must be within (0, 1]")
    if "min_prob" in q and q["min_prob"] < 0:
        raise ConfigurationError("min_prob must be non-negative")
    if "cap" in q and q["cap"] <= 0:
        raise ConfigurationError("cap_per_token_bits must be positive")
    if "prob_temp" in q and q["prob_temp"] <= 0:
        raise ConfigurationError("temperature must be positive")
    if "prob_temp" in q and ("cap" in q or "min_prob" in q):
        raise ConfigurationError("the crypto quality policy takes only top_k, top_p and temperature")
    return _lib.NsRankQuality(q.get("top_k", 0), q.get("cap", 0), q.get("top_p", 0.0), q.get("min_prob", -1.0),
                              q.get("prob_temp", 0.0))


class RankEncodeSession:
    """B payloads (bytes) encoded by the src rank coder (``codec/arithmetic.py:122-168``), one launch per
    token; :meth:`consumed` is the reference's ``state["history"]`` per stream."""

    def __init__(self, ctx: CoderContext, payloads: Sequence[bytes], *, temp: float, quality=None,
                 max_tokens: Optional[int] = None):
        torch = _torch()
        self.ctx, self.B = ctx, len(payloads)
        if self.B < 1 or self.B > ctx.max_batch:
            raise ConfigurationError(f"batch {self.B} outside [1, {ctx.max_batch}]")
        dev = torch.device("cuda", ctx.device)
        self.temp, self.q = float(temp), rank_quality(quality)
        self.nbytes = [len(bytes(pl)) for pl in payloads]
        stride = max(1, max(self.nbytes))
        buf = np.zeros((self.B, stride), dtype=np.uint8)
        for i, pl in enumerate(payloads):
            buf[i, : len(pl)] = np.frombuffer(bytes(pl), dtype=np.uint8)
        self.payload = torch.from_numpy(buf).to(dev)
        self.nbits = torch.tensor([8 * n for n in self.nbytes], dtype=torch.int64, device=dev)
        self.state = _state_tensor(self.B, dev)
        ctx.check(_lib.lib().ns_init_state(ctx._h, _ptr(self.state), self.B, _stream_handle()), "ns_init_state")
        cap = max_tokens if max_tokens is not None else 8 * stride + 16
        self.out_token = torch.zeros(self.B, dtype=torch.int32, device=dev)
        self.hist = torch.full((self.B, cap), -1, dtype=torch.int32, device=dev)
        self.cons = torch.zeros((self.B, cap), dtype=torch.int32, device=dev)

    def step(self, logits):
        logits = _rank_rows(self.ctx, self.B, logits, self.q)
        rc = _lib.lib().ns_rank_encode_step(
            self.ctx._h, _ptr(logits), logits.stride(0), self.B, _ptr(self.payload), self.payload.stride(0),
            _ptr(self.nbits), _ptr(self.state), _ptr(self.out_token), _ptr(self.hist), _ptr(self.cons),
            self.hist.shape[1], self.temp, ctypes.byref(self.q), ctypes.c_void_p(0), 0, _stream_handle())
        self.ctx.check(rc, "ns_rank_encode_step")
        return self.out_token

    def fields(self) -> dict:
        return _state_fields(self.state)

    def all_done(self) -> bool:
        f = self.fields()
        return bool(np.all((f["flags"] & _lib.NS_ST_DONE) != 0))

    def raise_errors(self) -> None:
        bad = np.nonzero(self.fields()["flags"] & _lib.NS_ST_ERR_RANGE)[0]
        if bad.size:
            raise ArithmeticRangeError(f"streams {bad.tolist()[:8]}: language model distribution provides no capacity")

    def tokens(self) -> List[List[int]]:
        self.raise_errors()
        n = self.fields()["ntokens"]
        h = self.hist.cpu().numpy()
        return [h[i, : int(n[i])].astype(np.int64).tolist() for i in range(self.B)]

    def consumed(self) -> List[List[int]]:
        n = self.fields()["ntokens"]
        c = self.cons.cpu().numpy()
        return [c[i, : int(n[i])].astype(np.int64).tolist() for i in range(self.B)]


class RankDecodeSession:
    """Decode of the rank coder (``codec/arithmetic.py:171-231``) given every stream's consumption history."""

    def __init__(self, ctx: CoderContext, token_lists: Sequence[Sequence[int]], histories: Sequence[Sequence[int]],
                 *, temp: float, quality=None):
        torch = _torch()
        self.ctx, self.B = ctx, len(token_lists)
        if self.B < 1 or self.B > ctx.max_batch:
            raise ConfigurationError(f"batch {self.B} outside [1, {ctx.max_batch}]")
        for tl, hs in zip(token_lists, histories):
            if len(hs) < len(tl):
                raise DecodeDivergenceError("Bit consumption history is required for decoding")
        dev = torch.device("cuda", ctx.device)
        self.temp, self.q = float(temp), rank_quality(quality)
        self.T = max((len(t) for t in token_lists), default=0)
        T1 = max(self.T, 1)
        tok = np.zeros((T1, self.B), np.int32)
        keep = np.zeros((T1, self.B), np.int32)
        act = np.zeros((T1, self.B), np.uint8)
        for i, (tl, hs) in enumerate(zip(token_lists, histories)):
            n = len(tl)
            tok[:n, i] = np.asarray(tl, np.int32)
            keep[:n, i] = np.asarray(list(hs)[:n], np.int32)
            act[:n, i] = 1
        self.tok, self.keep, self.act = (torch.from_numpy(a).to(dev) for a in (tok, keep, act))
        total = int(max((sum(list(h)[: len(t)]) for t, h in zip(token_lists, histories)), default=0))
        self.out_stride = (total + 7) // 8 + 8
        self.out_bits = torch.zeros((self.B, self.out_stride), dtype=torch.uint8, device=dev)
        self.state = _state_tensor(self.B, dev)
        ctx.check(_lib.lib().ns_init_state(ctx._h, _ptr(self.state), self.B, _stream_handle()), "ns_init_state")
        self.t = 0

    def step(self, logits) -> None:
        t = self.t
        logits = _rank_rows(self.ctx, self.B, logits, self.q)
        rc = _lib.lib().ns_rank_decode_step(
            self.ctx._h, _ptr(logits), logits.stride(0), self.B, _ptr(self.tok[t]), _ptr(self.keep[t]),
            _ptr(self.act[t]), _ptr(self.state), _ptr(self.out_bits), self.out_stride, self.temp,
            ctypes.byref(self.q), ctypes.c_void_p(0), 0, _stream_handle())
        self.ctx.check(rc, "ns_rank_decode_step")
        self.t += 1

    def payloads(self) -> List[bytes]:
        f = _state_fields(self.state)
        bad = np.nonzero(f["flags"] & _lib.NS_ST_ERR_DIVERGE)[0]
        if bad.size:
            raise DecodeDivergenceError(f"streams {bad.tolist()[:8]}: token not present in distribution")
        ob = self.out_bits.cpu().numpy()
        return [ob[i, : int(f["bit_pos"][i]) // 8].tobytes() for i in range(self.B)]
