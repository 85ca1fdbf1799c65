"""The src package's exact-rational arithmetic coder, selectable as ``encode_bits`` / ``decode_bits``
(``src/neuralstego/codec/arithmetic.py:234-325``, steps ``:408-550``) on the batched device kernel
``ns_frac_encode_step`` / ``ns_frac_decode_step`` (``include/nsg_fraction.h``, ``csrc/nsg_fraction.hip``).

Same names, arguments, state dict and exceptions as the reference; ``encode_bits_batch`` / ``decode_bits_batch``
run B independent messages in lockstep, one kernel launch per token step.  Host side (here): iterating the
ProbDist iterables, the reference's type / sign / NaN checks in its order, the payload bit expansion
(``BitReader``, MSB first, zero-padded by the kernel) and the ``BitWriter`` packing.  Every fraction, interval
and prefix computation is on the device; there is no CPU path (the library must load, a GPU must be present).

The reference computes with ``fractions.Fraction``; the kernel keeps the same rational values as integers
whose size grows with every token (by about the size of the lcm of the step's denominators).  Integers are
bounded by ``cap_limbs`` 32-bit limbs per stream (the cumulative table by ``table_limbs``, grown on demand);
a message that outgrows them raises :class:`FractionCapacityError` -- where the reference would keep going,
ever more slowly.
"""

from __future__ import annotations

from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .errors import ArithmeticRangeError, DecodeDivergenceError

NS_FRAC_OK, NS_FRAC_SKIPPED = 0, 1
NS_FRAC_ERR_NO_MASS, NS_FRAC_ERR_UNRESOLVED, NS_FRAC_ERR_NOT_PRESENT, NS_FRAC_ERR_NO_PREFIX = -1, -2, -3, -4
NS_FRAC_ERR_CAPACITY, NS_FRAC_ERR_TABLE = -5, -6

DEFAULT_CAP_LIMBS = 4096          # 131,072-bit interval integers per stream
DEFAULT_TABLE_LIMBS = 1 << 16     # cumulative numerators of one step, grown x8 on demand ...
MAX_TABLE_LIMBS = 1 << 24         # ... up to 64 MiB per stream
SCRATCH_BUDGET_BYTES = 8 << 30    # device scratch of one launch; a larger table than this allows fails the message
MAX_PAYLOAD_BITS = 1 << 16        # payloads above 8 KiB (and consumption entries above this + 64) are refused: a
#                                   failing step searches one depth per payload bit on ever longer integers
_INT32 = (-(1 << 31), (1 << 31) - 1)


class FractionCapacityError(ArithmeticRangeError):
    """A stream's exact integers outgrew the device arena (``cap_limbs`` / ``table_limbs``)."""


def _bytes_to_bits(payload: bytes) -> np.ndarray:
    """``BitReader`` bits (``codec/arithmetic.py:20-77``): MSB first."""
    return np.unpackbits(np.frombuffer(bytes(payload), dtype=np.uint8))


def _bits_to_bytes(bits: np.ndarray) -> bytes:
    """``BitWriter.to_bytes`` (``codec/arithmetic.py:100-119``): MSB first, the last byte zero-padded."""
    return np.packbits(np.asarray(bits, dtype=np.uint8)).tobytes() if len(bits) else b""


def _dist_row(dist) -> Tuple[np.ndarray, np.ndarray]:
    """(token ids, float64 values) in the reference's order (``_dist_to_sequences``, ``:490-500``: array index
    order, or the dict's sorted items), raising what its ``_to_fraction`` (``:545-550``) raises for the first
    value it cannot take: a negative value, then NaN / infinity (``Fraction.from_float``)."""
    if isinstance(dist, np.ndarray):
        if dist.ndim == 1 and dist.dtype.kind in "fiub":  # float(v) of each element, vectorised
            vals = dist.astype(np.float64)
        else:
            vals = np.asarray([float(v) for v in dist.tolist()], dtype=np.float64)
        ids = np.arange(vals.size, dtype=np.int64)
    elif isinstance(dist, dict):
        items = sorted(dist.items())
        ids = np.asarray([int(t) for t, _ in items], dtype=np.int64)
        vals = np.asarray([float(p) for _, p in items], dtype=np.float64)
    else:
        raise TypeError(f"Unsupported probability distribution type: {type(dist)!r}")
    bad = ~(np.isfinite(vals) & (vals >= 0.0))
    if bad.any():
        v = float(vals[int(np.argmax(bad))])
        if v < 0.0:
            raise ArithmeticRangeError("Probabilities must be non-negative")
        v.as_integer_ratio()  # NaN: ValueError, infinity: OverflowError -- Fraction.from_float's own errors
    if ids.size and (ids.min() < _INT32[0] or ids.max() > _INT32[1]):
        raise ValueError("token ids must fit in int32")
    return ids.astype(np.int32), vals


class _Device:
    """An ``ns_frac`` context for B streams plus the step's staging buffers."""

    def __init__(self, B: int, cap_limbs: int, device=None):
        import torch

        from .. import _lib

        if not torch.cuda.is_available():
            raise _lib.NativeLibraryError("the Fraction coder runs on the GPU (there is no CPU path)")
        self.torch = torch
        self.L = _lib.lib()
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.B = B
        self.ctx = self.L.ns_frac_create(B, int(cap_limbs), self.dev.index or 0)
        if not self.ctx:
            raise RuntimeError("ns_frac_create failed: " + self.L.ns_frac_last_error(None).decode())
        self.tables = np.full(B, DEFAULT_TABLE_LIMBS, dtype=np.int64)  # per stream: grown only where a step needs it

    def close(self) -> None:
        if self.ctx:
            self.L.ns_frac_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int, what: str) -> None:
        if rc != 0:
            raise RuntimeError(f"{what} failed ({rc}): {self.L.ns_frac_last_error(self.ctx).decode()}")

    def stream(self):
        return self.torch.cuda.current_stream(self.dev).cuda_stream

    def rows(self, rows: dict):
        """Stage {stream: (ids, values)} as [B, ld] device arrays; count -1 for the other streams."""
        torch = self.torch
        ld = max([1] + [len(v) for _, v in rows.values()])
        probs = np.zeros((self.B, ld), dtype=np.float64)
        ids = np.zeros((self.B, ld), dtype=np.int32)
        count = np.full(self.B, -1, dtype=np.int32)
        for i, (tid, vals) in rows.items():
            probs[i, :len(vals)] = vals
            ids[i, :len(tid)] = tid
            count[i] = len(vals)
        return (torch.from_numpy(probs).to(self.dev), torch.from_numpy(ids).to(self.dev), count, ld)

    def run(self, launch, count: np.ndarray, status_dev, ld: int, max_bits: int, collect) -> np.ndarray:
        """Run the step for the streams with ``count >= 0``: one launch per table size in use, each with scratch
        for its own streams only (``ns_frac_set_slots``).  A stream whose step needs a larger cumulative table
        (``NS_FRAC_ERR_TABLE``; its state is unchanged) re-runs with 8x the table -- kept for its later steps --
        until ``MAX_TABLE_LIMBS`` or the scratch budget, past which it fails with ``NS_FRAC_ERR_CAPACITY``.
        ``collect(mask)`` reads the per-stream outputs of the streams that ran in a launch before the next one.
        Returns the per-stream status."""
        torch = self.torch
        status = np.full(self.B, NS_FRAC_SKIPPED, dtype=np.int32)
        pending = count >= 0
        while pending.any():
            table = int(self.tables[pending].min())
            grp = pending & (self.tables == table)
            n = int(grp.sum())
            if self.L.ns_frac_scratch_bytes(self.ctx, n, ld, max_bits, table) > SCRATCH_BUDGET_BYTES:
                # over the scratch budget together: launch as many as fit (a stream fails only if it
                # cannot fit alone, never because of what else is in the batch); the rest stay pending
                one = int(self.L.ns_frac_scratch_bytes(self.ctx, 1, ld, max_bits, table))
                if one > SCRATCH_BUDGET_BYTES:
                    status[grp] = NS_FRAC_ERR_CAPACITY
                    pending &= ~grp
                    continue
                fit = max(1, SCRATCH_BUDGET_BYTES // one)
                while fit > 1 and \
                        self.L.ns_frac_scratch_bytes(self.ctx, fit, ld, max_bits, table) > SCRATCH_BUDGET_BYTES:
                    fit -= 1
                idx = np.nonzero(grp)[0]
                grp = np.zeros_like(grp)
                grp[idx[:fit]] = True
                n = int(fit)
            pending &= ~grp
            d_slot = torch.from_numpy(np.where(grp, np.cumsum(grp) - 1, -1).astype(np.int32)).to(self.dev)
            self.check(self.L.ns_frac_set_slots(self.ctx, d_slot.data_ptr(), n), "ns_frac_set_slots")
            try:
                launch(torch.from_numpy(np.where(grp, count, -1).astype(np.int32)).to(self.dev), table)
                st = status_dev.cpu().numpy()  # synchronises: d_slot is no longer read
            finally:
                self.check(self.L.ns_frac_set_slots(self.ctx, None, 0), "ns_frac_set_slots")
            collect(grp)
            status[grp] = st[grp]
            short = grp & (st == NS_FRAC_ERR_TABLE)
            grow = short & (self.tables < MAX_TABLE_LIMBS)
            status[short & ~grow] = NS_FRAC_ERR_CAPACITY
            self.tables[grow] = np.minimum(self.tables[grow] * 8, MAX_TABLE_LIMBS)
            pending |= grow
        return status


def _capacity_error() -> FractionCapacityError:
    return FractionCapacityError("the message's exact interval integers outgrew the device arena "
                                 "(raise cap_limbs); the reference would need ever larger fractions here too")


def encode_bits_batch(payloads: Sequence[bytes], probs: Sequence[Iterable], states: Optional[Sequence] = None, *,
                      cap_limbs: int = DEFAULT_CAP_LIMBS, device=None, return_exceptions: bool = False) -> list:
    """``encode_bits`` for B messages at once; ``probs[b]`` is message b's ProbDist iterable.  Errors are the
    reference's, per message: raised for the first failing message, or returned in its place with
    ``return_exceptions``."""
    B = len(payloads)
    if states is not None and len(states) != B:
        raise ValueError("one state per payload")
    bits = [_bytes_to_bits(p) for p in payloads]
    n = np.array([len(b) for b in bits], dtype=np.int64)
    out: list = [[] for _ in range(B)]
    used_hist: List[List[int]] = [[] for _ in range(B)]
    err: list = [None] * B
    for i in range(B):
        if n[i] > MAX_PAYLOAD_BITS:
            err[i] = FractionCapacityError(f"payload of {int(n[i])} bits: the device Fraction coder takes at most "
                                           f"{MAX_PAYLOAD_BITS} bits per message")
    live = [i for i in range(B) if n[i] > 0 and err[i] is None]
    if live:
        dv = _Device(B, cap_limbs, device)
        torch = dv.torch
        try:
            stride = max(1, max(int(n[i]) for i in live))
            host_bits = np.zeros((B, stride), dtype=np.uint8)
            for i in live:
                host_bits[i, :len(bits[i])] = bits[i]
            d_bits = torch.from_numpy(host_bits).to(dv.dev)
            n_live = np.where([err[i] is None for i in range(B)], n, 0).astype(np.int64)
            dv.check(dv.L.ns_frac_init(dv.ctx, B, n_live.ctypes.data, dv.stream()), "ns_frac_init")
            token = torch.empty(B, dtype=torch.int32, device=dv.dev)
            used = torch.empty(B, dtype=torch.int32, device=dv.dev)
            status = torch.empty(B, dtype=torch.int32, device=dv.dev)
            tok = np.full(B, -1, dtype=np.int32)
            use = np.zeros(B, dtype=np.int32)

            def collect(mask):
                tok[mask] = token.cpu().numpy()[mask]
                use[mask] = used.cpu().numpy()[mask]

            its = [iter(p) for p in probs]
            pos = np.zeros(B, dtype=np.int64)
            while live:
                rows = {}
                for i in live:
                    try:
                        dist = next(its[i])
                    except StopIteration:
                        err[i] = ArithmeticRangeError("Insufficient probability distributions for encoding")
                        continue
                    try:
                        rows[i] = _dist_row(dist)
                    except Exception as exc:  # the reference's own conversion errors, per message
                        err[i] = exc
                live = [i for i in live if err[i] is None]
                if not live:
                    break
                d_probs, d_ids, count, ld = dv.rows(rows)

                def launch(d_count, table):
                    dv.check(dv.L.ns_frac_encode_step(dv.ctx, B, d_probs.data_ptr(), d_ids.data_ptr(), ld,
                                                      d_count.data_ptr(), d_bits.data_ptr(), stride, stride, table,
                                                      token.data_ptr(), used.data_ptr(), status.data_ptr(),
                                                      dv.stream()), "ns_frac_encode_step")

                st = dv.run(launch, count, status, ld, stride, collect)
                for i in list(live):
                    s = int(st[i])
                    if s == NS_FRAC_OK:
                        out[i].append(int(tok[i]))
                        used_hist[i].append(int(use[i]))
                        pos[i] += min(int(use[i]), max(int(n[i] - pos[i]), 0))
                    elif s == NS_FRAC_ERR_NO_MASS:
                        err[i] = ArithmeticRangeError("Probability distribution must have positive mass")
                    elif s == NS_FRAC_ERR_UNRESOLVED:
                        err[i] = ArithmeticRangeError("Unable to resolve token interval with available bits")
                    elif s == NS_FRAC_ERR_CAPACITY:
                        err[i] = _capacity_error()
                    else:
                        err[i] = RuntimeError(f"ns_frac_encode_step: unexpected status {s}")
                live = [i for i in live if err[i] is None and pos[i] < n[i]]
        finally:
            dv.close()
    for i in range(B):
        if err[i] is None and states is not None and states[i] is not None:
            states[i]["history"] = tuple(used_hist[i])
            states[i]["residual_bits"] = int(n[i]).to_bytes(8, byteorder="big", signed=False)
    if not return_exceptions:
        for e in err:
            if e is not None:
                raise e
    return [err[i] if err[i] is not None else out[i] for i in range(B)]


def decode_bits_batch(token_lists: Sequence[Sequence[int]], probs: Sequence[Iterable],
                      states: Optional[Sequence] = None, *, cap_limbs: int = DEFAULT_CAP_LIMBS, device=None,
                      return_exceptions: bool = False) -> list:
    """``decode_bits`` for B token sequences at once (``probs[b]`` and ``states[b]`` are message b's)."""
    B = len(token_lists)
    if states is not None and len(states) != B:
        raise ValueError("one state per token list")
    res: list = [b"" for _ in range(B)]
    err: list = [None] * B
    toks = [list(t) for t in token_lists]
    cons: List[List[int]] = [[] for _ in range(B)]
    total: List[Optional[int]] = [None] * B
    live = []
    for i in range(B):
        if not toks[i]:
            continue
        state = states[i] if states is not None else None
        history = state.get("history") if state is not None else None
        if state is not None:
            residual = state.get("residual_bits")
            if residual:
                total[i] = int.from_bytes(residual, byteorder="big", signed=False)
        if history is None or len(history) < len(toks[i]):
            err[i] = DecodeDivergenceError("Bit consumption history is required for decoding")
            continue
        cons[i] = [int(c) for c in history[:len(toks[i])]]
        if max(cons[i]) > MAX_PAYLOAD_BITS + 64:
            err[i] = FractionCapacityError(f"a token consuming {max(cons[i])} bits: the device Fraction coder takes at "
                                           f"most {MAX_PAYLOAD_BITS + 64} per token")
            continue
        live.append(i)
    written = np.zeros(B, dtype=np.int64)
    if live:
        dv = _Device(B, cap_limbs, device)
        torch = dv.torch
        try:
            out_stride = max(1, max(sum(max(c, 0) for c in cons[i]) for i in live))
            max_used = max(max(max(c, 0) for c in cons[i]) for i in live)
            d_out = torch.zeros((B, out_stride), dtype=torch.uint8, device=dv.dev)
            d_pos = torch.zeros(B, dtype=torch.int64, device=dv.dev)
            status = torch.empty(B, dtype=torch.int32, device=dv.dev)
            dv.check(dv.L.ns_frac_init(dv.ctx, B, np.zeros(B, dtype=np.int64).ctypes.data, dv.stream()),
                     "ns_frac_init")
            its = [iter(probs[i]) if i in live else None for i in range(B)]
            t = 0
            while live:
                rows, tok_h, use_h = {}, np.zeros(B, dtype=np.int32), np.full(B, -1, dtype=np.int32)
                for i in live:
                    try:
                        dist = next(its[i])
                    except StopIteration:
                        err[i] = ArithmeticRangeError("Insufficient probability distributions for decoding")
                        continue
                    try:
                        row = _dist_row(dist)
                    except Exception as exc:
                        err[i] = exc
                        continue
                    tid = int(toks[i][t])
                    if not (_INT32[0] <= tid <= _INT32[1]):
                        err[i] = DecodeDivergenceError(f"Token {toks[i][t]} not present in distribution")
                        continue
                    rows[i] = row
                    tok_h[i] = tid
                    use_h[i] = max(cons[i][t], 0)
                live = [i for i in live if err[i] is None]
                if not live:
                    break
                d_probs, d_ids, count, ld = dv.rows(rows)
                d_tok = torch.from_numpy(tok_h).to(dv.dev)
                d_use = torch.from_numpy(use_h).to(dv.dev)

                def launch(d_count, table):
                    dv.check(dv.L.ns_frac_decode_step(dv.ctx, B, d_probs.data_ptr(), d_ids.data_ptr(), ld,
                                                      d_count.data_ptr(), d_tok.data_ptr(), d_use.data_ptr(),
                                                      max_used, table, d_out.data_ptr(), out_stride,
                                                      d_pos.data_ptr(), status.data_ptr(), dv.stream()),
                             "ns_frac_decode_step")

                st = dv.run(launch, count, status, ld, max_used, lambda mask: None)
                for i in list(live):
                    s = int(st[i])
                    if s == NS_FRAC_OK:
                        continue
                    if s == NS_FRAC_ERR_NO_MASS:
                        err[i] = ArithmeticRangeError("Probability distribution must have positive mass")
                    elif s == NS_FRAC_ERR_NOT_PRESENT:
                        err[i] = DecodeDivergenceError(f"Token {toks[i][t]} not present in distribution")
                    elif s == NS_FRAC_ERR_NO_PREFIX:
                        err[i] = DecodeDivergenceError("No binary prefix fits within the interval")
                    elif s == NS_FRAC_ERR_CAPACITY:
                        err[i] = _capacity_error()
                    else:
                        err[i] = RuntimeError(f"ns_frac_decode_step: unexpected status {s}")
                t += 1
                live = [i for i in live if err[i] is None and t < len(toks[i])]
            written = d_pos.cpu().numpy()
            host_out = d_out.cpu().numpy()
        finally:
            dv.close()
        for i in range(B):
            if err[i] is not None or not toks[i]:
                continue
            bits = host_out[i, :int(written[i])]
            state = states[i] if states is not None else None
            if state is not None:
                rest = list(state["history"][len(toks[i]):])
                if rest:
                    state["history"] = tuple(rest)
                else:
                    state.pop("history", None)
            n_total = total[i] if total[i] is not None else len(bits)
            if n_total > len(bits):
                err[i] = DecodeDivergenceError("Decoded bitstream shorter than expected")
                continue
            res[i] = _bits_to_bytes(bits[:n_total])
    if not return_exceptions:
        for e in err:
            if e is not None:
                raise e
    return [err[i] if err[i] is not None else res[i] for i in range(B)]


def encode_bits(bits: bytes, probs: Iterable, *, state=None) -> List[int]:
    """Encode a bitstream into a sequence of token identifiers (``codec/arithmetic.py:234-270``)."""
    return encode_bits_batch([bits], [probs], [state])[0]


def decode_bits(tokens: Sequence[int], probs: Iterable, *, state=None) -> bytes:
    """Decode a sequence of token identifiers back into the embedded bitstream (``codec/arithmetic.py:273-325``)."""
    return decode_bits_batch([tokens], [probs], [state])[0]


__all__ = ["encode_bits", "decode_bits", "encode_bits_batch", "decode_bits_batch", "FractionCapacityError"]
