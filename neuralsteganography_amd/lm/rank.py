"""``HipRankLM``: the src package's own provider (``src/neuralstego/lm/arithmetic.py:115-264``, ``ArithmeticLM``)
on the GPU -- the uniform rank coder of ``codec/arithmetic.py:122-231`` (``encode_with_lm`` /
``decode_with_lm``) with its quality policies, over a KV-cached batched GPT-2 and the HIP rank kernel.

Same protocol and side channel as the reference: ``encode_arithmetic`` returns token ids and queues a
``{"history", "residual_bits"}`` state (bits consumed per token, payload bit count); ``decode_arithmetic``
pops one and needs it (the rank coder cannot decode without the history, ``codec/arithmetic.py:188-189``).
Quality keys follow ``lm/arithmetic.py:77-112``: temp / temperature, topk / top_k, top_p, min_prob,
cap_per_token_bits, max_context.

Without ``max_context`` the reference re-runs the whole context per token; this provider keeps a KV cache with
positions modulo ``n_positions`` -- the same logits while the context fits ``n_positions`` (the reference's forward
fails beyond it).  With ``max_context`` (``lm/arithmetic.py:50-51,106-112``) the trimmed window's positions shift
every token, so no cache applies: each step re-runs every stream's last ``max_context`` tokens from scratch
(:class:`WindowedLM`, the batched GPT-2's native causal sequence forward), exactly the reference's computation.
"""

from __future__ import annotations

from collections import deque
from typing import Deque, Dict, Iterable, List, Mapping, Optional, Sequence

from ..coder import CoderContext, CoderParams, RankDecodeSession, RankEncodeSession
from ..exceptions import ConfigurationError
from .arithmetic import ByteTokenizer

CodecState = Dict[str, object]


def _bits_to_bytes(bits: Sequence[int]) -> bytes:
    if len(bits) % 8:
        raise ConfigurationError("bit stream length must be a multiple of 8")
    out = bytearray(len(bits) // 8)
    for i in range(len(out)):
        out[i] = sum((int(bits[8 * i + k]) & 1) << k for k in range(8))
    return bytes(out)


def _bytes_to_bits(data: bytes) -> List[int]:
    return [(b >> k) & 1 for b in bytes(data) for k in range(8)]


def _temperature(quality: Optional[Mapping[str, object]]) -> float:
    for key in ("temp", "temperature"):
        if quality and quality.get(key) is not None:
            t = float(quality[key])
            if t <= 0:
                raise ConfigurationError("temperature must be positive")
            return t
    return 1.0


def _max_context(quality: Optional[Mapping[str, object]]) -> Optional[int]:
    """``_quality_max_context`` (``lm/arithmetic.py:106-112``)."""
    if not quality:
        return None
    for key in ("max_context", "maxContext"):
        if key in quality and quality[key] is not None:
            return int(quality[key])
    return None


class WindowedLM:
    """``prefill`` / ``step`` of a batched GPT-2 where every query re-runs the stream's context trimmed to its last
    ``window`` ids from scratch (positions 0..W-1): ``_ModelAdapter.next_token_probs`` with ``max_context``
    (``src/neuralstego/lm/arithmetic.py:45-74``), which ``encode_with_lm`` also trims to (``codec/arithmetic.py:
    337-347``).  One batched causal forward of ``[B, W]`` tokens per step (``BatchedGPT2.window_logits``)."""

    takes_full_context = True  # the whole context reaches prefill (trimmed here, as the reference trims it)

    def __init__(self, lm, window: int):
        import torch

        if window <= 0:  # the provider maps 0 to "no trimming" (ids[-0:] is the whole list) before it gets here
            raise ConfigurationError("max_context must be positive")
        if not hasattr(lm, "window_logits"):
            raise ConfigurationError("max_context needs a GPT-2 provider (BatchedGPT2.window_logits)")
        # a window above n_positions is fine while the context is shorter (the reference's slice keeps it whole);
        # only a forward over more ids than the model has positions fails (_logits), as the reference's model does
        self.lm, self.window, self.shape = lm, int(window), lm.shape
        self.device = lm.device
        self.ids = torch.zeros((0, 0), dtype=torch.long)

    def _logits(self):
        ids = self.ids[:, -self.window:]
        if ids.shape[1] > self.shape.n_positions:
            raise ConfigurationError(f"a context of {ids.shape[1]} ids (max_context {self.window}) exceeds the model's "
                                     f"{self.shape.n_positions} positions")
        return self.lm.window_logits(ids.contiguous())

    def prefill(self, context, B: int, max_new: int):
        import torch

        del max_new
        ctx = [int(t) for t in context]
        if not ctx:
            raise ConfigurationError("context must contain at least one token")  # lm/arithmetic.py:46-48
        if min(ctx) < 0 or max(ctx) >= self.shape.vocab:
            raise ConfigurationError(f"context token ids must lie in [0, {self.shape.vocab})")
        self.ids = torch.tensor(ctx[-self.window:], device=self.device, dtype=torch.long)[None].repeat(int(B), 1)
        return self._logits()

    def step(self, tokens):
        import torch

        tok = tokens.to(device=self.device, dtype=torch.long).view(-1, 1)
        self.ids = torch.cat([self.ids[:, -(self.window - 1):] if self.window > 1 else self.ids[:, :0], tok], 1)
        return self._logits()


class HipRankLM:
    """Rank-coder provider: batched GPT-2 (or any ``prefill``/``step`` batched LM) + the HIP rank kernel."""

    def __init__(self, model=None, tokenizer=None, *, batched_lm=None, device: Optional[str] = None,
                 logits_dtype: str = "f32", compute_dtype=None, max_batch: int = 4096):
        import torch

        if not torch.cuda.is_available():
            from .._lib import NativeLibraryError

            raise NativeLibraryError("HipRankLM needs a ROCm GPU (the rank coder has no CPU path)")
        if batched_lm is None:
            from .gpt2 import BatchedGPT2

            dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
            ldt = torch.float16 if logits_dtype == "f16" else torch.float32
            batched_lm = BatchedGPT2(model, device=dev, compute_dtype=compute_dtype, logits_dtype=ldt)
        if getattr(batched_lm, "prob_rows", False):
            logits_dtype = "f64"  # a generic provider's own float64 ProbDists (ProviderBatchedLM)
        self.lm = batched_lm
        self.vocab = self.lm.shape.vocab
        # the byte stand-in only where it can spell bytes (a small provider vocabulary has no tokenizer: its
        # callers pass token ids, and encode_seed then raises)
        if tokenizer is None and self.vocab >= 257:
            tokenizer = ByteTokenizer(self.vocab)
        self.tokenizer = tokenizer
        self.logits_dtype = logits_dtype
        self.max_batch = int(max_batch)
        self.device_index = torch.cuda.current_device()
        self._ctx: Dict[int, CoderContext] = {}
        self._encode_states: List[CodecState] = []
        self._decode_states: Deque[CodecState] = deque()

    def _coder(self, B: int, vocab: Optional[int] = None) -> CoderContext:
        """One coder context (the parameters never change here) sized for the largest batch -- and, for a
        generic provider's rows, the longest row -- seen so far: a smaller one reuses it, a larger one replaces it
        (the kernels take B per call; a provider row's entry count is registered per step)."""
        V = max(int(vocab or 0), self.vocab)
        ctx = self._ctx.get(0)
        if ctx is not None and (ctx.max_batch < B or ctx.params.vocab < V):
            ctx.close()
            ctx = None
        if ctx is None:
            params = CoderParams(vocab=V, precision=16, temp=1.0, topk=V, dtype=self.logits_dtype, banned=[])
            ctx = CoderContext(params, max_batch=max(B, 1), device=self.device_index)
            self._ctx[0] = ctx
        self.vocab = V
        return ctx

    def _fit(self, sess, rows):
        """A provider step whose rows outgrow the context (a longer dict, a larger ndarray) moves the session to a
        wider context: its stream state lives in the session's tensors, the context holds scratch only."""
        if getattr(rows, "prob_rows", False) and rows.ncols > sess.ctx.params.vocab:
            sess.ctx = self._coder(sess.B, rows.ncols)

    # ------------------------------------------------------------------ protocol (api.py:42-56)
    def encode_seed(self, text: str) -> List[int]:
        tok = self.tokenizer
        if tok is None:
            raise ConfigurationError(f"no tokenizer for a {self.vocab}-id vocabulary: pass token ids as context")
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
        return self.encode_batch([bits], context, quality=quality)[0]

    def decode_arithmetic(self, tokens: List[int], context: List[int], *, quality: Mapping[str, object]) -> List[int]:
        if not tokens:
            if self._decode_states:
                self._decode_states.popleft()
            return []
        if not self._decode_states:
            raise ConfigurationError("decode state unavailable for the rank coder")
        st = self._decode_states.popleft()
        return self.decode_batch([tokens], context, quality=quality, states=[st])[0]

    def drain_states(self) -> List[CodecState]:
        out = [dict(s) for s in self._encode_states]
        self._encode_states.clear()
        return out

    def load_states(self, states: Iterable[CodecState]) -> None:
        self._decode_states = deque(dict(s) for s in states)

    # ------------------------------------------------------------------ batched
    def _context(self, context: Sequence[int], lm=None) -> List[int]:
        """The prefill context: GPT-2 keeps the reference's last 1022 ids (and needs one); a host provider
        (``ProviderBatchedLM``) or a ``max_context`` window gets it untrimmed, as ``next_token_probs`` would."""
        if getattr(lm if lm is not None else self.lm, "takes_full_context", False):
            return [int(t) for t in context]
        return list(context)[-1022:] or [0]

    def _lm_for(self, quality):
        """The batched LM of a call: the provider's own, or a :class:`WindowedLM` over it when the quality asks for
        ``max_context`` (a generic provider's context window is applied by ``codec.rank`` instead)."""
        mc = _max_context(quality)
        if mc is None or getattr(self.lm, "prob_rows", False):
            return self.lm
        if mc < 0:  # the reference's ids[-max_context:] would then DROP the first |max_context| ids: not supported
            raise ConfigurationError("max_context must not be negative")
        if mc == 0:  # `len(ids) > 0` holds and ids[-0:] is the whole context: no trimming (lm/arithmetic.py:49-50)
            return self.lm
        return WindowedLM(self.lm, mc)

    def encode_batch(self, bit_lists: Sequence[Sequence[int]], context: Sequence[int], *,
                     quality: Mapping[str, object], max_steps: int = 1 << 16) -> List[List[int]]:
        toks, states = self.encode_batch_states(bit_lists, context, quality=quality, max_steps=max_steps)
        for st in states:
            self._encode_states.append(dict(st))
            self._decode_states.append(dict(st))
        return toks

    def encode_batch_states(self, bit_lists: Sequence[Sequence[int]], context: Sequence[int], *,
                            quality: Mapping[str, object], max_steps: int = 1 << 16):
        """:meth:`encode_batch` returning ``(tokens, states)`` -- each stream's ``{"history", "residual_bits"}``
        side channel -- without queueing the states on the provider (``codec.rank.encode_with_lm`` hands them
        to the caller's ``state`` dict instead)."""
        B = len(bit_lists)
        if B == 0:
            return [], []
        payloads = [_bits_to_bytes(list(b)) for b in bit_lists]
        empty = [len(p) == 0 for p in payloads]
        ctx = self._coder(B)
        sess = RankEncodeSession(ctx, [p if p else b"\x00" for p in payloads], temp=_temperature(quality),
                                 quality=quality)
        if any(empty):  # encode_with_lm returns no token for an empty payload (:150-154)
            sess.nbits[[i for i, e in enumerate(empty) if e]] = 0
        import torch

        lm = self._lm_for(quality)
        logits = lm.prefill(self._context(context, lm), B, 8 * max(len(p) for p in payloads) + 2)
        self._fit(sess, logits)
        # host providers (ProviderBatchedLM): check after every step, so the provider is never queried past the
        # last token (the reference's loop ends before another next_token_probs call, codec/arithmetic.py:146)
        host = getattr(lm, "prob_rows", False)
        every = 1 if host else 8
        for t in range(max_steps):
            if t % every == 0:
                sess.raise_errors()
                if sess.all_done():
                    break
            self._fit(sess, logits)
            tok = sess.step(logits)
            if host:
                sess.raise_errors()
                if sess.all_done():
                    break
            logits = lm.step(tok.to(torch.long))
        toks, cons = sess.tokens(), sess.consumed()
        states = []
        for i in range(B):
            if empty[i]:
                toks[i], cons[i] = [], []
            states.append({"history": tuple(cons[i]), "residual_bits": (8 * len(payloads[i])).to_bytes(8, "big")})
        return toks, states

    def decode_batch(self, token_lists: Sequence[Sequence[int]], context: Sequence[int], *,
                     quality: Mapping[str, object], states: Optional[Sequence[CodecState]] = None) -> List[List[int]]:
        import torch

        B = len(token_lists)
        if B == 0:
            return []
        if states is None:
            states = [self._decode_states.popleft() if self._decode_states else {} for _ in range(B)]
        hist = [list(s.get("history") or ()) for s in states]
        if not getattr(self.lm, "prob_rows", False):  # GPT-2 ids feed the embedding gather: check on the host
            for tl in token_lists:
                if any(not 0 <= int(t) < self.vocab for t in tl):
                    from ..codec.errors import DecodeDivergenceError

                    raise DecodeDivergenceError(f"token id outside [0, {self.vocab})")
        ctx = self._coder(B)
        sess = RankDecodeSession(ctx, token_lists, hist, temp=_temperature(quality), quality=quality)
        lm = self._lm_for(quality)
        logits = lm.prefill(self._context(context, lm), B, max(sess.T, 1) + 1)
        for t in range(sess.T):
            self._fit(sess, logits)
            sess.step(logits)
            if t + 1 < sess.T:
                logits = lm.step(sess.tok[t].to(torch.long))
        out = []
        for i, pl in enumerate(sess.payloads()):
            nb = states[i].get("residual_bits")
            if nb:
                pl = pl[: int.from_bytes(bytes(nb), "big") // 8]
            out.append(_bytes_to_bits(pl))
        return out


__all__ = ["HipRankLM"]
