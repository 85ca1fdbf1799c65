"""``HipArithmeticLM``: the drop-in provider behind the reference's plugin protocol.

Implements ``src/neuralstego/api.py:42-56`` (``LMProvider``: ``encode_arithmetic`` / ``decode_arithmetic`` /
``encode_seed``) plus the optional ``drain_states`` / ``load_states`` side channel probed by
``api.encode_text``/``decode_text`` (``api.py:850-854,996-1000``), mirroring ``ArithmeticLM``
(``src/neuralstego/lm/arithmetic.py:144-264``).  Unlike the reference provider (a fixed-width rank coder
that re-runs the whole context per token, ``codec/arithmetic.py:122-231``), this one runs the TRUE arithmetic
coder of ``code_base/arithmetic.py`` on the HIP kernel, batched over streams, with a KV-cached GPT-2.

Bits cross the boundary as LSB-first bit lists (``api.py:153-157``); ``encode_arithmetic`` returns token
ids; ``decode_arithmetic`` returns exactly the number of bits that were encoded (the count travels in the
state side channel as ``residual_bits`` = 8-byte big-endian bit count, the reference's CodecState format).
"""

from __future__ import annotations

from collections import deque
from typing import Deque, Dict, Iterable, List, Mapping, Optional, Sequence

from ..coder import CoderContext, CoderParams, DecodeSession, EncodeSession
from ..exceptions import ConfigurationError

CodecState = Dict[str, object]


def coder_params_from_quality(quality: Optional[Mapping[str, object]], vocab: int, logits_dtype: str,
                              banned: Optional[Sequence[int]] = None) -> CoderParams:
    """Map the api quality dict to coder parameters.

    Keys and defaults follow ``encode_arithmetic``'s signature (``code_base/arithmetic.py:78-88``) and the
    api's key aliases (``api.py:130-141``): temp/temperature (1.0), precision (16), topk/top_k (50000)."""
    q = dict(quality or {})

    def pick(*names, default=None):
        for n in names:
            if n in q and q[n] is not None:
                return q[n]
        return default

    temp = float(pick("temp", "temperature", default=1.0))
    precision = int(pick("precision", default=16))
    topk = int(pick("topk", "top_k", "top-k", default=50000))
    if temp <= 0:
        raise ConfigurationError("temperature must be positive")
    return CoderParams(vocab=vocab, precision=precision, temp=temp, topk=topk, dtype=logits_dtype, banned=banned)


def _bits_count_state(nbits: int) -> CodecState:
    return {"history": (), "residual_bits": int(nbits).to_bytes(8, byteorder="big", signed=False)}


class ByteTokenizer:
    """Tokenizer stand-in for random-init models (no vocabulary files offline): ids = UTF-8 bytes and
    ``<|endoftext|>`` = the last id of the vocabulary (50256 for GPT-2)."""

    def __init__(self, vocab: int = 50257):
        if vocab < 257:
            raise ConfigurationError("ByteTokenizer needs a vocabulary of at least 257 ids")
        self.eos_id = vocab - 1

    def encode(self, text: str, add_special_tokens: bool = False) -> List[int]:
        _ = add_special_tokens
        if text == "<|endoftext|>":
            return [self.eos_id]
        return list(text.encode("utf-8"))

    def decode(self, ids: Iterable[int]) -> str:
        return bytes(int(i) % 256 for i in ids).decode("utf-8", errors="ignore")


class HipArithmeticLM:
    """Arithmetic-coding provider: batched GPT-2 on PyTorch-ROCm + the HIP coder step."""

    def __init__(self, model, tokenizer=None, *, device: Optional[str] = None, logits_dtype: str = "f32",
                 compute_dtype=None, banned: Optional[Sequence[int]] = None, max_batch: int = 4096):
        import torch

        from .gpt2 import BatchedGPT2

        if not torch.cuda.is_available():
            from .._lib import NativeLibraryError

            raise NativeLibraryError("HipArithmeticLM needs a ROCm GPU (the coder has no CPU path)")
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        ldt = torch.float16 if logits_dtype == "f16" else torch.float32
        self.lm = BatchedGPT2(model, device=dev, compute_dtype=compute_dtype, logits_dtype=ldt)
        self.vocab = self.lm.shape.vocab
        self.tokenizer = tokenizer if tokenizer is not None else ByteTokenizer(self.vocab)
        self.logits_dtype = logits_dtype
        self.banned = list(banned) if banned is not None else None
        self.max_batch = int(max_batch)
        self.device = dev
        self._ctx_cache: Dict[tuple, CoderContext] = {}
        self._sent_end = None
        self._encode_states: List[CodecState] = []
        self._decode_states: Deque[CodecState] = deque()

    # ---------------------------------------------------------------- plumbing
    def _coder(self, params: CoderParams, B: int) -> CoderContext:
        key = (params.vocab, params.precision, params.temp, params.topk, params.dtype,
               tuple(params.banned_ids()), B)
        ctx = self._ctx_cache.get(key)
        if ctx is None:
            ctx = CoderContext(params, max_batch=max(B, 1), device=self.device.index)
            self._ctx_cache[key] = ctx
        return ctx

    def sentence_end_table(self):
        """Per-id table of sentence-ending tokens: ``'.' in t or '!' in t or '?' in t`` for the decoded
        text of each id (``code_base/utils.py:55-57``)."""
        if self._sent_end is None:
            import numpy as np

            tab = np.zeros(self.vocab, dtype=np.uint8)
            for i in range(self.vocab):
                try:
                    txt = self.tokenizer.decode([i])
                except Exception:
                    continue
                if "." in txt or "!" in txt or "?" in txt:
                    tab[i] = 1
            self._sent_end = tab
        return self._sent_end

    # ---------------------------------------------------------------- protocol
    def encode_seed(self, text: str) -> List[int]:
        """``<|endoftext|>`` + tokens of ``text`` (``src/neuralstego/lm/arithmetic.py:143-160``)."""
        tok = self.tokenizer
        try:
            bos = list(tok.encode("<|endoftext|>", add_special_tokens=False))
        except TypeError:
            bos = list(tok.encode("<|endoftext|>"))
        try:
            body = list(tok.encode(text, add_special_tokens=False))
        except TypeError:
            body = list(tok.encode(text))
        return [int(t) for t in bos + body]

    def encode_arithmetic(self, bits: List[int], context: List[int], *, quality: Mapping[str, object]) -> List[int]:
        toks = self.encode_batch([bits], context, quality=quality)[0]
        return toks

    def decode_arithmetic(self, tokens: List[int], context: List[int], *, quality: Mapping[str, object]) -> List[int]:
        state = self._decode_states.popleft() if self._decode_states else None
        if not tokens:
            return []
        nbits = None
        if state is not None and state.get("residual_bits"):
            nbits = int.from_bytes(bytes(state["residual_bits"]), byteorder="big", signed=False)
        out = self.decode_batch([tokens], context, quality=quality)[0]
        return out[:nbits] if nbits is not None else out

    def drain_states(self) -> List[CodecState]:
        states = [dict(s) for s in self._encode_states]
        self._encode_states.clear()
        return states

    def load_states(self, states: Iterable[CodecState]) -> None:
        self._decode_states = deque(dict(s) for s in states)

    # ---------------------------------------------------------------- batched entry points
    def encode_batch(self, bit_lists: Sequence[Sequence[int]], context: Sequence[int], *,
                     quality: Mapping[str, object], check_every: int = 16,
                     stall_steps: int = 4096) -> List[List[int]]:
        """Encode B independent bit lists in lockstep (one GPT-2 forward + one coder launch per token).

        The reference coder has no underflow handling: when the interval straddles the midpoint and one
        token takes the whole range, no bit is ever fixed and ``code_base/arithmetic.py:114`` loops
        forever.  Here a stream that fixes no payload bit for ``stall_steps`` tokens raises
        :class:`ArithmeticRangeError` instead of hanging."""
        B = len(bit_lists)
        if B == 0:
            return []
        params = coder_params_from_quality(quality, self.vocab, self.logits_dtype, self.banned)
        ctx = self._coder(params, B)
        finish = bool(dict(quality or {}).get("finish_sent", False))
        if finish:
            ctx.set_sentence_end(self.sentence_end_table())
        max_bits = max(len(b) for b in bit_lists)
        budget = 2 * max_bits + 64            # initial KV/history capacity (grows on demand)
        hard_cap = 64 * max_bits + 4096       # a stream fixing < 1/64 bit per token is reported, not looped
        logits = self.lm.prefill(context, B, budget)
        sess = EncodeSession(ctx, bit_lists, max_tokens=hard_cap)
        t = 0
        last_pos = None
        last_move = 0
        while True:
            if t % check_every == 0:
                f = sess.fields()
                if bool((f["flags"] & 1).all()):
                    break
                pos = f["bit_pos"].copy()
                if last_pos is None or (pos != last_pos).any():
                    last_pos, last_move = pos, t
                if t - last_move >= stall_steps or t >= hard_cap:
                    from ..codec.errors import ArithmeticRangeError

                    stuck = [i for i in range(B) if not (f["flags"][i] & 1)]
                    if all(f["bit_pos"][i] >= len(bit_lists[i]) for i in stuck):
                        raise ArithmeticRangeError(
                            f"finish_sent: streams {stuck[:8]} produced no sentence-ending token in "
                            f"{t - last_move} tokens (the reference would keep generating forever)")
                    raise ArithmeticRangeError(
                        f"streams {stuck[:8]} fixed no payload bit for {t - last_move} tokens: the interval "
                        "straddles the midpoint and one token takes the whole range (the reference coder "
                        "has no underflow handling and would loop forever)")
            tok = sess.step(logits, finish_sent=finish)
            logits = self.lm.step(tok)
            t += 1
        toks = sess.tokens()
        for b in bit_lists:
            st = _bits_count_state(len(b))
            self._encode_states.append(st)
            self._decode_states.append(dict(st))
        return toks

    def decode_batch(self, token_lists: Sequence[Sequence[int]], context: Sequence[int], *,
                     quality: Mapping[str, object]) -> List[List[int]]:
        """Decode B token lists (ragged) in lockstep; returns every emitted bit (callers truncate)."""
        import torch

        from ..codec.errors import DecodeDivergenceError

        B = len(token_lists)
        if B == 0:
            return []
        for tl in token_lists:  # received ids feed the embedding gather: validate on the host first
            if any((int(t) < 0 or int(t) >= self.vocab) for t in tl):
                raise DecodeDivergenceError(f"received token id outside [0, {self.vocab})")
        params = coder_params_from_quality(quality, self.vocab, self.logits_dtype, self.banned)
        ctx = self._coder(params, B)
        sess = DecodeSession(ctx, token_lists)
        logits = self.lm.prefill(context, B, max(sess.T, 1) + 1)
        for t in range(sess.T):
            sess.step(logits)
            if t + 1 < sess.T:
                logits = self.lm.step(sess.tok[t])
        return sess.bits()


__all__ = ["HipArithmeticLM", "ByteTokenizer", "coder_params_from_quality"]
