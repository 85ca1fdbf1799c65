"""Synthetic workloads shared by the parity tests, the golden-vector generator and bench.py.

SURVEY.md §8(d) restates BASELINE.json's metric as synthetic inputs:

* stream ``s`` carries a payload from ``np.random.default_rng([20251010, s])``; bits are LSB-first per
  byte, the convention of ``src/neuralstego/api.py:153-157`` and ``lm/arithmetic.py:30-35``;
* context = ``[50256] + list(range(1000, 1031))``;
* coder-only logits: row ``(s, t)`` = ``scale * N(0, 1)`` drawn from ``default_rng([seed, s, t])``.

Nothing here touches the GPU; callers copy the arrays where they need them.
"""

from __future__ import annotations

from typing import List, Sequence

import numpy as np

PAYLOAD_SEED = 20251010
DEFAULT_CONTEXT: List[int] = [50256] + list(range(1000, 1031))
GPT2_VOCAB = 50257


def payload_bytes(stream: int, nbytes: int, seed: int = PAYLOAD_SEED) -> bytes:
    """Random payload of stream ``stream``."""
    return np.random.default_rng([seed, stream]).bytes(nbytes)


def bytes_to_bits_lsb(data: bytes) -> List[int]:
    """LSB-first bit list, as ``src/neuralstego/api.py:153-157`` builds it."""
    arr = np.frombuffer(bytes(data), dtype=np.uint8)
    return np.unpackbits(arr, bitorder="little").astype(np.int64).tolist()


def bits_to_bytes_lsb(bits: Sequence[int]) -> bytes:
    """Inverse of :func:`bytes_to_bits_lsb` (``api.py:160-170``); pads the last byte with zeros."""
    arr = np.asarray(list(bits), dtype=np.uint8)
    return np.packbits(arr, bitorder="little").tobytes()


def pack_bits_lsb(bits: Sequence[int]) -> np.ndarray:
    """Pack a bit list into the coder's payload byte layout: bit ``j`` is ``byte[j >> 3] >> (j & 7)``."""
    arr = np.asarray(list(bits), dtype=np.uint8)
    if arr.size == 0:
        return np.zeros(0, dtype=np.uint8)
    return np.packbits(arr, bitorder="little")


def unpack_bits_lsb(packed: np.ndarray, nbits: int) -> List[int]:
    bits = np.unpackbits(np.asarray(packed, dtype=np.uint8), bitorder="little")
    return bits[:nbits].astype(np.int64).tolist()


def logits_row(seed: int, stream: int, step: int, vocab: int, scale: float = 3.0,
               dtype=np.float32) -> np.ndarray:
    """One synthetic logit row; the same generator feeds the HIP kernel and the CPU oracle."""
    rng = np.random.default_rng([seed, stream, step])
    return (scale * rng.standard_normal(vocab)).astype(np.float32).astype(dtype)


def logits_batch(seed: int, streams: Sequence[int], step: int, vocab: int, scale: float = 3.0,
                 dtype=np.float32, ld: int | None = None) -> np.ndarray:
    """``[len(streams), ld]`` batch of rows; columns ``[vocab, ld)`` are zero padding."""
    ld = vocab if ld is None else ld
    out = np.zeros((len(streams), ld), dtype=dtype)
    for r, s in enumerate(streams):
        out[r, :vocab] = logits_row(seed, s, step, vocab, scale, dtype)
    return out


def top_region_tie_free(row: np.ndarray, topk: int, banned: Sequence[int]) -> bool:
    """True when the ``topk + 1`` largest non-banned values are pairwise distinct.

    The reference sorts with ``torch.sort(descending=True)`` (``code_base/arithmetic.py:127``), whose tie
    order is unspecified; fixtures are generated with a stable sort and this check documents which rows
    would be order-ambiguous under the unstable one.
    """
    vals = row.astype(np.float64).copy()
    vals[list(banned)] = -np.inf
    n = min(topk + 1, vals.size)
    top = np.sort(vals)[::-1][:n]
    return bool(np.all(top[:-1] != top[1:]))


class SyntheticBatchedLM:
    """Batched-logits provider with context-independent synthetic rows (the ``prefill``/``step`` protocol of
    :class:`~neuralsteganography_amd.lm.gpt2.BatchedGPT2`): call t (prefill = call 0) returns
    ``logits_row(seed, streams[b], t)`` for every stream b, whatever tokens were fed -- the same rows the
    golden generator's synthetic model hands the reference coder (tests/golden/make_golden.py)."""

    def __init__(self, seed: int, vocab: int, scale: float = 3.0, dtype: str = "f32", streams=None, boost=None):
        from types import SimpleNamespace

        self.boost = {int(k): int(v) for k, v in (boost or {}).items()}  # call index -> token id, +30 logit
        self.seed, self.vocab, self.scale = int(seed), int(vocab), float(scale)
        self.np_dtype = np.float16 if dtype == "f16" else np.float32
        self.ld = ((self.vocab + 63) // 64) * 64
        self.shape = SimpleNamespace(vocab=self.vocab, n_positions=1024)
        self.streams = None if streams is None else [int(s) for s in streams]
        self.t, self.B, self.fed = 0, 0, []

    def _rows(self):
        import torch

        ids = self.streams[: self.B] if self.streams is not None else list(range(self.B))
        arr = logits_batch(self.seed, ids, self.t, self.vocab, self.scale, self.np_dtype, self.ld)
        if self.t in self.boost:
            arr[:, self.boost[self.t]] += self.np_dtype(30.0)
        return torch.from_numpy(arr).cuda()

    def prefill(self, context, B: int, max_new: int):
        self.t, self.B, self.fed = 0, int(B), []
        return self._rows()

    def step(self, tokens):
        self.fed.append(tokens.detach().cpu().numpy().copy())
        self.t += 1
        return self._rows()


class IdTokenizer:
    """Synthetic tokenizer for random-init models (no vocabulary file offline): id i <-> " w<i>." (every id but 3
    ends a sentence), the last id = <|endoftext|>.  ``decode`` / ``encode`` round-trip every id sequence, so covers
    made with it are revealed from their TEXT (the C5 bench leg and its GPU test)."""

    def __init__(self, vocab: int):
        self.eos_id = vocab - 1

    def _piece(self, i: int) -> str:
        return "<|endoftext|>" if i == self.eos_id else f" w{i}" + ("." if i != 3 else "")

    def decode(self, ids, skip_special_tokens: bool = False) -> str:
        return "".join("" if (skip_special_tokens and int(i) == self.eos_id) else self._piece(int(i)) for i in ids)

    def encode(self, text: str, add_special_tokens: bool = False) -> List[int]:
        import re

        return [self.eos_id if mm.group(1) is None else int(mm.group(1))
                for mm in re.finditer(r"<\|endoftext\|>|w(\d+)", text)]

