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

from ..coder import CoderContext, CoderParams, DecodeSession, EncodeSession, SampleSession, StreamingDecodeSession
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
    # top-k aliases: the LAST one in the mapping wins, as the reference's key loop does
    # (src/neuralstego/lm/arithmetic.py:77-95) -- api.stego_encode merges {**_DEFAULT_QUALITY, **user}, so a
    # caller's (or a regeneration attempt's) "top_k" follows the default "topk" and must override it
    topk = 50000
    for key, value in q.items():
        if value is not None and key.replace("-", "_").lower() in ("topk", "top_k"):
            topk = int(value)
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


CTX_CACHE_SIZE = 4  # live coder contexts per provider (distinct quality settings)


class _StepGraph:
    """One lockstep encode step -- the HIP coder step on the current logits, then the GPT-2 decode step that
    turns its tokens into the next logits -- captured once as a hipGraph (``torch.cuda.CUDAGraph``) and replayed
    per token.  Everything that changes per step lives on the device (coder state, token buffer, the cache
    length ``d_L``), so a replay issues no host work besides the launch.  Construction runs one real step (on a
    side stream, which also warms up every kernel and GEMM plan) before capturing the next."""

    def __init__(self, lm, coder_step, logits):
        import torch

        self.lm, self.coder_step = lm, coder_step  # coder_step(logits) -> the step's token buffer [B] (device)
        self.logits = logits.clone()
        lm.begin_static(self.logits)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self._body()
        torch.cuda.current_stream().wait_stream(side)
        lm.L += 1
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._body()

    def _body(self) -> None:
        self.lm.step_static(self.coder_step(self.logits))

    def replay(self) -> None:
        self.graph.replay()
        self.lm.L += 1


class _StopCheck:
    """The reference's per-token stop test ``stop_text in enc.decode(output)`` (``code_base/arithmetic.py:
    207-210``) without a host round trip per token.  A new occurrence of ``stop_text`` must end inside the newest
    token, so that token's text contains the last character of ``stop_text``; a per-id device table of such
    tokens is gathered by the emitted tokens inside the step (graph-capturable), and the host reads one flag
    per step and decodes 16-token tails only for the flagged streams."""

    def __init__(self, provider, sess, stop_text: str):
        import torch

        self.sess, self.stop_text, self.tok = sess, stop_text, provider.tokenizer
        self.table = provider.stop_table(stop_text)
        self.hit = torch.zeros(sess.B, dtype=torch.bool, device=sess.state.device)
        self.any = torch.zeros(1, dtype=torch.bool, device=sess.state.device)
        self.any_host = torch.zeros(1, dtype=torch.bool).pin_memory()

    def flag(self, tok) -> None:
        import torch

        live = (self.sess.state.view(torch.int32)[:, 7] & 1) == 0
        torch.logical_and(self.table.index_select(0, tok.long()), live, out=self.hit)
        torch.any(self.hit, dim=0, keepdim=True, out=self.any)

    def check(self) -> None:
        import torch

        self.any_host.copy_(self.any, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        if not bool(self.any_host[0]):
            return
        cand = torch.nonzero(self.hit).flatten().cpu().tolist()
        n = self.sess.fields()["ntokens"]
        stop = []
        for i in cand:
            k = int(n[i])
            tail = self.sess.hist[i, max(0, k - 16):k].cpu().tolist()
            if self.stop_text in self.tok.decode(tail):
                stop.append(i)
        if stop:
            self.sess.mark_done(stop)


class HipArithmeticLM:
    """Arithmetic-coding provider: batched GPT-2 on PyTorch-ROCm + the HIP coder step."""

    decodes_without_state = True  # the interval coder needs no per-token history (unlike the rank coder)
    skip_done = True  # finished streams skip their attention (encode: done flag, decode: stop position; A/B, tests)
    slot_compaction = True  # native slot loops: compact the live slots once the queue is drained (off: tests that
                            # read per-step logits by row)

    def __init__(self, model, tokenizer=None, *, device: Optional[str] = None, logits_dtype: str = "f32",
                 compute_dtype=None, banned: Optional[Sequence[int]] = None, max_batch: int = 4096,
                 kv_dtype: str = "fp16", attention_window: int = 0, logit_scale: float = 1.0):
        import torch

        from .gpt2 import BatchedGPT2

        if not torch.cuda.is_available():
            from .._lib import NativeLibraryError

            raise NativeLibraryError("HipArithmeticLM needs a ROCm GPU (the coder has no CPU path)")
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        ldt = torch.float16 if logits_dtype == "f16" else torch.float32
        lm = BatchedGPT2(model, device=dev, compute_dtype=compute_dtype, logits_dtype=ldt, kv_dtype=kv_dtype,
                         logit_scale=logit_scale)
        if attention_window:
            if not lm.native:
                raise ConfigurationError("an attention window needs the native fp16 decode step on the GPU")
            if int(attention_window) < 1:
                raise ConfigurationError("attention_window must be positive (0 = unbounded)")
            lm.window = int(attention_window)
        self._init(lm, tokenizer, dev, logits_dtype, banned, max_batch)

    @classmethod
    def from_batched(cls, batched_lm, tokenizer=None, *, logits_dtype: str = "f32",
                     banned: Optional[Sequence[int]] = None, max_batch: int = 4096) -> "HipArithmeticLM":
        """Provider over any batched-logits LM with the ``prefill(context, B, max_new)`` / ``step(tokens)``
        protocol (e.g. :class:`~neuralsteganography_amd.synthetic.SyntheticBatchedLM`)."""
        import torch

        if not torch.cuda.is_available():
            from .._lib import NativeLibraryError

            raise NativeLibraryError("HipArithmeticLM needs a ROCm GPU (the coder has no CPU path)")
        self = cls.__new__(cls)
        self._init(batched_lm, tokenizer, torch.device("cuda", torch.cuda.current_device()), logits_dtype, banned,
                   max_batch)
        return self

    def _init(self, lm, tokenizer, dev, logits_dtype, banned, max_batch) -> None:
        self.lm = lm
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
        """Coder context for ``params`` serving batches up to ``B``.  Keyed on the parameters only (the kernels
        take B per call): a context built for a larger batch serves every smaller one, a larger B replaces it,
        and at most ``CTX_CACHE_SIZE`` parameter sets stay alive (least recently used closed first) -- each
        wide-path context holds 2*B*V*8 bytes of sort keys."""
        key = (params.vocab, params.precision, params.temp, params.topk, params.dtype,
               tuple(params.banned_ids()))
        ctx = self._ctx_cache.pop(key, None)
        if ctx is not None and ctx.max_batch < B:
            ctx.close()
            ctx = None
        if ctx is None:
            ctx = CoderContext(params, max_batch=max(B, 1), device=self.device.index)
        self._ctx_cache[key] = ctx  # re-inserted last: dict order is the LRU order
        while len(self._ctx_cache) > CTX_CACHE_SIZE:
            old = next(iter(self._ctx_cache))
            self._ctx_cache.pop(old).close()
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

    def stop_table(self, stop_text: str):
        """Device bool table [vocab]: the id's decoded text contains the last character of ``stop_text``
        (only such a token can complete a new occurrence).  Cached per stop text."""
        import torch

        cache = self.__dict__.setdefault("_stop_tables", {})
        tab = cache.get(stop_text)
        if tab is None:
            host = torch.from_numpy(stop_candidates(self.tokenizer, self.vocab, stop_text))
            tab = cache[stop_text] = host.to(self.device)
        return tab

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
                     stall_steps: int = 4096, return_stats: bool = False, stop_text: Optional[str] = None,
                     graphs: Optional[bool] = None, slots: Optional[int] = None):
        """Encode independent bit lists (one GPT-2 forward + one coder launch per token for every live stream).

        On the native GPU model (the product path) the messages run through ``slots`` slots (default
        ``min(len(bit_lists), max_batch)``, :class:`~neuralsteganography_amd.lm.slots.SlotEncoder`): a finished
        message's slot takes the next queued one, KV pages follow the live tokens (``lm/kvpages.py``), the youngest
        messages are re-queued when the device is full, and the live slots are compacted once the queue is drained.
        A message's tokens do not depend on its slot or neighbours (batch-invariant decode step).  Other LMs (the
        PyTorch fp32 forward, synthetic rows) run the lockstep loop below.

        With ``graphs`` (default; needs the native fp16 step) the per-token step is captured once as a hipGraph
        and replayed, which removes the per-launch host cost (it dominates at small batch, and at B = 4096 it
        keeps the GPU busy across the host checks); the cache budget bounds the replays and the loop continues
        eagerly (growing the cache) if it runs out.  The token history starts at the KV budget: when a stream
        would outgrow it, the graph is dropped, the history grown and the step captured again.

        The reference coder has no underflow handling: when the interval straddles the midpoint and one
        token takes the whole range, no bit is ever fixed and ``code_base/arithmetic.py:114`` loops
        forever.  Here a stream that fixes no payload bit for ``stall_steps`` tokens raises
        :class:`ArithmeticRangeError` instead of hanging."""
        B = len(bit_lists)
        if B == 0:
            return []
        params = coder_params_from_quality(quality, self.vocab, self.logits_dtype, self.banned)
        finish = bool(dict(quality or {}).get("finish_sent", False))
        max_bits = max(len(b) for b in bit_lists)
        budget = 2 * max_bits + 64            # initial KV/history capacity (grows on demand)
        hard_cap = 64 * max_bits + 4096       # a stream fixing < 1/64 bit per token is reported, not looped
        if graphs is None:
            graphs = True
        if getattr(self.lm, "native", False):
            from .slots import SlotEncoder

            S = max(1, min(B, int(slots) if slots else self.max_batch))
            ctx = self._coder(params, S)
            if finish:
                ctx.set_sentence_end(self.sentence_end_table())
            enc = SlotEncoder(self, ctx, bit_lists, context, slots=S, finish=finish, stop_text=stop_text,
                              stats=return_stats, check_every=check_every, stall_steps=stall_steps, hard_cap=hard_cap,
                              use_graph=bool(graphs), compact=self.slot_compaction)
            toks, st = enc.run()
            self.last_schedule = {"slots": S, "evictions": enc.evictions, "compactions": enc.compactions,
                                  "max_live": enc.max_live, "kv_pages_peak": enc.kv_peak}
            for b in bit_lists:
                sc = _bits_count_state(len(b))
                self._encode_states.append(sc)
                self._decode_states.append(dict(sc))
            return (toks, st) if return_stats else toks
        ctx = self._coder(params, B)
        if finish:
            ctx.set_sentence_end(self.sentence_end_table())
        logits = self.lm.prefill(context, B, budget)
        use_graph = graphs and getattr(self.lm, "hip_attention", False) and hasattr(self.lm, "begin_static")
        # token history: starts at the KV budget and grows at the host checks (a captured graph holds the
        # buffer's address, so it is re-captured after a growth; the 64x hard cap up front would be 8.6 GB at
        # B = 4096)
        sess = EncodeSession(ctx, bit_lists, max_tokens=budget, stats=return_stats)
        stop = _StopCheck(self, sess, stop_text) if stop_text is not None else None

        def coder_step(lg):
            tok = sess.step(lg, finish_sent=finish)
            if stop is not None:
                stop.flag(tok)  # device-side: did any live stream emit a token that can complete stop_text?
            return tok

        native = getattr(self.lm, "native", False) and self.skip_done
        if native:  # finished streams skip their attention reads (the coder state's flags word, NS_ST_DONE)
            import torch

            self.lm.done_flags = sess.state.view(torch.int32)[:, 7]
        try:
            toks = self._encode_loop(sess, coder_step, logits, stop, bit_lists, check_every, stall_steps, hard_cap,
                                     use_graph)
        finally:
            if native:
                self.lm.done_flags = None
        for b in bit_lists:
            st = _bits_count_state(len(b))
            self._encode_states.append(st)
            self._decode_states.append(dict(st))
        if return_stats:
            return toks, sess.stats()
        return toks

    def _encode_loop(self, sess, coder_step, logits, stop, bit_lists, check_every, stall_steps, hard_cap, use_graph):
        B = sess.B
        t = 0
        last_pos = None
        last_move = 0
        graph = None
        while True:
            if stop is not None and t > 0:
                stop.check()  # code_base/arithmetic.py:207-210 ('<eos>' in run_single.py's message->bits mode)
            if t % check_every == 0:
                f = sess.fields()
                if bool((f["flags"] & 1).all()):
                    break
                if graph is not None and int(f["ntokens"].max(initial=0)) + check_every + 1 > sess.hist.shape[1]:
                    logits, graph = graph.logits, None  # the history must grow: re-capture with the new buffer
                if graph is None:
                    sess.ensure_history(check_every + 1)
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
            if use_graph and self.lm.static_capacity_left() >= 1:
                if graph is None:
                    graph = _StepGraph(self.lm, coder_step, logits)
                else:
                    graph.replay()
                t += 1
                continue
            if graph is not None:  # the preallocated cache is used up: continue eagerly (the cache grows)
                logits, graph, use_graph = graph.logits, None, False
            tok = coder_step(logits)
            logits = self.lm.step(tok)
            t += 1
        del graph
        return sess.tokens()

    def decode_batch(self, token_lists: Sequence[Sequence[int]], context: Sequence[int], *,
                     quality: Mapping[str, object], graphs: Optional[bool] = None,
                     slots: Optional[int] = None) -> List[List[int]]:
        """Decode token lists (ragged); returns every emitted bit (callers truncate).  On the native GPU model the
        lists run through ``slots`` slots (:class:`~neuralsteganography_amd.lm.slots.SlotDecoder`, longest first,
        a message's pages mapped when it is admitted); with ``graphs`` the per-token step (coder + GPT-2 decode) is a
        replayed hipGraph, as in :meth:`encode_batch`."""
        import torch

        from ..codec.errors import DecodeDivergenceError

        B = len(token_lists)
        if B == 0:
            return []
        for tl in token_lists:  # received ids feed the embedding gather: validate on the host first
            if any((int(t) < 0 or int(t) >= self.vocab) for t in tl):
                raise DecodeDivergenceError(f"received token id outside [0, {self.vocab})")
        params = coder_params_from_quality(quality, self.vocab, self.logits_dtype, self.banned)
        if graphs is None:
            graphs = True
        if getattr(self.lm, "native", False):  # the product path: slots, pages mapped at admission (lm/slots.py)
            from .slots import SlotDecoder

            S = max(1, min(B, int(slots) if slots else self.max_batch))
            dec = SlotDecoder(self, self._coder(params, S), token_lists, context, slots=S, use_graph=bool(graphs),
                              compact=self.slot_compaction)
            out = dec.run()
            self.last_decode_schedule = {"slots": S, "evictions": dec.evictions, "compactions": dec.compactions}
            return out
        ctx = self._coder(params, B)
        sess = DecodeSession(ctx, token_lists)
        logits = self.lm.prefill(context, B, max(sess.T, 1) + 1)
        native = getattr(self.lm, "native", False) and self.skip_done
        if native:
            # the forward after token t feeds token t + 1's logits: a stream of n tokens needs none once the cache
            # length reaches prefill + n - 1, so its attention is skipped from there (ragged, uneven covers)
            import torch

            lens = torch.tensor([len(t) for t in token_lists], dtype=torch.int32)
            self.lm.stop_len = (lens + (self.lm.L - 1)).to(self.lm.device)
        try:
            if (graphs and sess.T > 2 and getattr(self.lm, "hip_attention", False) and hasattr(self.lm, "begin_static")
                    and self.lm.static_capacity_left() >= sess.T):  # replays cannot grow the cache
                graph = _StepGraph(self.lm, sess.step_static, logits)  # runs token 0, captures the next step
                for _ in range(1, sess.T):  # the last replay's forward feeds nothing (the cache holds T + 1)
                    graph.replay()
                del graph
                return sess.bits()
            for t in range(sess.T):
                sess.step(logits)
                if t + 1 < sess.T:
                    logits = self.lm.step(sess.tok[t])
            return sess.bits()
        finally:
            if native:
                self.lm.stop_len = None

    def decode_counted(self, token_lists: Sequence[Sequence[int]], context: Sequence[int], *,
                       quality: Mapping[str, object], done=None, check_every: int = 64):
        """``decode_batch`` that also records, per stream, the cumulative number of bits emitted after each
        token (the span splitter of ``text_to_spans`` needs the token at which a packet completes).  A stream
        whose token falls outside the kept top-k stops emitting (its later counts stay flat) instead of
        raising.  ``done(bits_lists, counts_lists) -> bool`` is polled every ``check_every`` tokens and ends
        the loop early once it holds.  Returns ``(bits per stream, counts per stream)``."""
        import numpy as np
        import torch

        from ..coder import _state_fields

        B = len(token_lists)
        if B == 0:
            return [], []
        for tl in token_lists:
            if any((int(t) < 0 or int(t) >= self.vocab) for t in tl):
                from ..codec.errors import DecodeDivergenceError

                raise DecodeDivergenceError(f"received token id outside [0, {self.vocab})")
        params = coder_params_from_quality(quality, self.vocab, self.logits_dtype, self.banned)
        ctx = self._coder(params, B)
        sess = DecodeSession(ctx, token_lists)
        counts = torch.zeros((max(sess.T, 1), B), dtype=torch.int64, device=sess.state.device)
        logits = self.lm.prefill(context, B, max(sess.T, 1) + 1)

        def snapshot(n):
            f = _state_fields(sess.state)
            ob = sess.out_bits.cpu().numpy()
            cn = counts[:n].cpu().numpy()
            bits = [np.unpackbits(ob[i], bitorder="little")[: int(f["bit_pos"][i])].tolist() for i in range(B)]
            return bits, [cn[: min(n, len(token_lists[i])), i].tolist() for i in range(B)]

        t = 0
        lens = np.asarray([len(tl) for tl in token_lists])
        while t < sess.T:
            sess.step(logits)
            counts[t].copy_(sess.state[:, 2])  # bit_pos after token t
            t += 1
            if t < sess.T:
                logits = self._lm_step(sess.tok[t - 1], lens > t)  # streams with a token t left to decode
            if done is not None and t % check_every == 0 and t < sess.T and done(*snapshot(t)):
                break
        return snapshot(t)


    def _lm_step(self, tokens, live):
        """``lm.step`` for the lockstep decodes, telling a native model which streams still need logits."""
        if getattr(self.lm, "native", False):
            return self.lm.step(tokens, live=live)
        return self.lm.step(tokens)

    def decode_tokens_repair(self, token_lists: Sequence[Sequence[int]], context: Sequence[int], *,
                             quality: Mapping[str, object], enc=None) -> List[List[int]]:
        """Batched ``decode_arithmetic`` token loop with the reference's BPE repair (code_base/arithmetic.py
        :254-371): a received token outside the kept top-k' is repaired on the host from the kernel's
        ranked ids (:300-342, :func:`bpe_repair`), the token list is edited as the reference edits it, and
        the step is re-issued; an unrepairable token decodes as rank 0 while the LM is still fed the
        received token, exactly as the reference does.  Returns every emitted bit per stream."""
        return self.decode_counted_repair(token_lists, context, quality=quality, enc=enc, strict=True)[0]

    def decode_counted_repair(self, token_lists: Sequence[Sequence[int]], context: Sequence[int], *,
                              quality: Mapping[str, object], enc=None, done=None, check_every: int = 64,
                              strict: bool = False):
        """:meth:`decode_tokens_repair` that also returns, per stream, the cumulative number of bits emitted
        after each token of the (repaired) list and the repaired token list itself -- the span splitter of
        ``texts_to_spans`` needs both when a cover text re-tokenises differently from the emitted ids.
        ``done(bits_lists, counts_lists, token_lists) -> bool`` is polled every ``check_every`` tokens and ends
        the loop early once it holds.  With ``strict`` a repaired token that still falls outside the top-k
        raises :class:`DecodeDivergenceError`; otherwise that stream stops emitting (its counts stay flat).
        Returns ``(bits per stream, counts per stream, token lists, edits)``: ``edits[b]`` lists ``(p, list)``,
        the stream's token list after each repair at position ``p`` (a repair at ``p`` changes positions >= p
        only), so a caller that learns afterwards that the stream ended at token e takes the list of the last
        repair at p <= e -- tokens decoded past e (another span's, out of context) may have been "repaired"."""
        import torch

        from ..coder import _state_fields

        enc = enc if enc is not None else self.tokenizer
        lists = [[int(t) for t in tl] for tl in token_lists]
        B = len(lists)
        if B == 0:
            return [], [], [], []
        for tl in lists:  # received ids feed the embedding gather: validate on the host first
            if any(not 0 <= t < self.vocab for t in tl):
                raise ConfigurationError(f"received token id outside [0, {self.vocab})")
        params = coder_params_from_quality(quality, self.vocab, self.logits_dtype, self.banned)
        ctx = self._coder(params, B)
        sess = StreamingDecodeSession(ctx, B, max_tokens=max(len(x) for x in lists) + 8)
        logits = self.lm.prefill(context, B, max(len(x) for x in lists) + 8)
        pos = [0] * B
        counts: List[List[int]] = [[] for _ in range(B)]
        edits: List[list] = [[] for _ in range(B)]
        dead = [False] * B  # non-strict: a stream whose repaired token still diverged stops here
        steps = 0
        while True:
            active = [pos[b] < len(lists[b]) and not dead[b] for b in range(B)]
            if not any(active):
                break
            tok = [lists[b][pos[b]] if active[b] else 0 for b in range(B)]
            last = [active[b] and pos[b] == len(lists[b]) - 1 for b in range(B)]
            sess.step(logits, tok, last, active)
            feed = list(tok)
            bad = sess.diverged()
            if bad:
                redo = [0] * B
                for b in bad:
                    coder_tok = repair_or_restore(enc, lists[b], pos[b], sess.ranked_ids(b), strict=strict)
                    if any(not 0 <= t < self.vocab for t in lists[b]):
                        raise ConfigurationError(f"repair produced a token id outside [0, {self.vocab})")
                    redo[b] = coder_tok
                    feed[b] = lists[b][pos[b]]  # repaired token, or the received one when unrepairable
                    edits[b].append((pos[b], list(lists[b])))
                sess.clear(bad)
                act2 = [b in bad for b in range(B)]
                last2 = [act2[b] and pos[b] == len(lists[b]) - 1 for b in range(B)]
                sess.step(logits, redo, last2, act2)
                still = sess.diverged()
                if still:
                    if strict:
                        from ..codec.errors import DecodeDivergenceError

                        raise DecodeDivergenceError(f"streams {still[:8]}: repaired token still outside the top-k")
                    sess.clear(still)
                    for b in still:
                        dead[b] = True
            bit_pos = _state_fields(sess.state)["bit_pos"]
            for b in range(B):
                if active[b] and not dead[b]:
                    counts[b].append(int(bit_pos[b]))
                    pos[b] += 1
            steps += 1
            if not any(pos[b] < len(lists[b]) and not dead[b] for b in range(B)):
                break
            if done is not None and steps % check_every == 0 and done(sess.bits(), counts, lists):
                break
            nxt = [pos[b] < len(lists[b]) and not dead[b] for b in range(B)]  # streams that decode a next token
            logits = self._lm_step(torch.tensor(feed, device=self.device, dtype=torch.long), nxt)
        return sess.bits(), counts, lists, edits

    def sample_batch(self, B: int, length: int, context: Sequence[int], *, temperature: float = 1.0,
                     topk: int = -1, seed: int = 0, stream_offset: int = 0, stats: bool = True):
        """B independent non-stego samples of ``length`` tokens from one context (code_base/sample.py, batched):
        returns ``(token lists, per-stream {avg_NLL, avg_KL, avg_Hq})``."""
        import torch

        params = CoderParams(vocab=self.vocab, precision=16, temp=float(temperature),
                             topk=int(topk) if int(topk) > 0 else self.vocab, dtype=self.logits_dtype,
                             banned=self.banned)
        ctx = self._coder(params, B)
        sess = SampleSession(ctx, B, seed=seed, topk=topk, temp=temperature, stream_offset=stream_offset,
                             max_tokens=max(1, length), stats=stats)
        logits = self.lm.prefill(context, B, length + 1)
        for t in range(length):
            tok = sess.step(logits)
            if t + 1 < length:
                logits = self.lm.step(tok.to(torch.long))
        return sess.tokens(), (sess.stats() if stats else None)


def stop_candidates(tokenizer, vocab: int, stop_text: str):
    """Per-id bool table of the tokens that can complete a new occurrence of ``stop_text`` (the newest token of
    ``stop_text in enc.decode(output)``, ``code_base/arithmetic.py:207-210``): the id's lone text contains the
    last character of ``stop_text``.  When that character is more than one UTF-8 byte, a byte-level BPE can
    split it across tokens and the completing token's lone text is U+FFFD (``errors='replace'``) or empty
    (``errors='ignore'``): such ids -- lone text with U+FFFD, empty, or not re-encoding to the id -- are
    candidates too, and so is an id whose lone decode raises."""
    import numpy as np

    if not stop_text:
        raise ConfigurationError("stop_text must be non-empty")
    last = stop_text[-1]
    multibyte = len(last.encode("utf-8")) > 1
    tab = np.zeros(vocab, dtype=np.bool_)
    for i in range(vocab):
        try:
            txt = tokenizer.decode([i])
        except Exception:
            tab[i] = True  # undecodable alone: always check it on the host
            continue
        if last in txt:
            tab[i] = True
        elif multibyte:
            if not txt or "\ufffd" in txt:
                tab[i] = True
                continue
            try:
                try:
                    back = list(tokenizer.encode(txt, add_special_tokens=False))
                except TypeError:
                    back = list(tokenizer.encode(txt))
            except Exception:
                back = None
            tab[i] = back != [i]
    return tab


def bpe_repair(enc, inp: List[int], i: int, ranked_ids: Sequence[int]):
    """The reference's BPE repair for a received token outside the kept top-k (code_base/arithmetic.py:300-342),
    restated line for line over ``ranked_ids`` (the kernel's ranked kept ids).  Edits ``inp`` in place as the
    reference does -- including its deletion loop, which removes every other following token when more than
    one is merged -- and returns ``(token to decode, repaired?)``; unrepairable tokens decode as rank 0."""
    true_token_text = enc.decode([inp[i]])
    for cand in ranked_ids:
        cand = int(cand)
        prop_token_text = enc.decode([cand])
        if inp[i] == 128 and cand == 198:  # common case that is not caught
            inp[i] = cand
            return cand, True
        if len(prop_token_text) <= len(true_token_text) and \
                prop_token_text == true_token_text[:len(prop_token_text)]:
            suffix = true_token_text[len(prop_token_text):]
            suffix_tokens = enc.encode(suffix)
            inp[i] = cand
            inp[i + 1:i + 1] = suffix_tokens
            return cand, True
        elif len(prop_token_text) > len(true_token_text) and \
                true_token_text == prop_token_text[:len(true_token_text)]:
            whole_text = true_token_text
            num_extra = 1
            while len(whole_text) < len(prop_token_text):
                whole_text += enc.decode([inp[i + num_extra]])
                num_extra += 1
            if prop_token_text == whole_text[:len(prop_token_text)]:
                inp[i] = cand
                for j in range(1, num_extra):
                    del inp[i + j]
                if len(whole_text) > len(prop_token_text):
                    suffix = whole_text[len(prop_token_text):]
                    inp[i + 1:i + 1] = enc.encode(suffix)
                return cand, True
    return int(ranked_ids[0]), False


def repair_or_restore(enc, inp: List[int], i: int, ranked_ids: Sequence[int], *, strict: bool) -> int:
    """:func:`bpe_repair` for the batched decoder: the token the coder decodes at position ``i``.

    The reference's longer-token branch reads ``inp[i + num_extra]`` and deletes ``inp[i + j]`` as it goes; when
    the merge reaches past the end of the text that raises ``IndexError`` out of ``decode_arithmetic``
    (``code_base/arithmetic.py:321-333``) -- possibly after ``inp`` was already edited.  Here the list is restored
    to its state before the attempt (so the LM is fed the received token and later spans are cut from an unedited
    list); strict decoding raises :class:`DecodeDivergenceError` as the reference raises, the lenient span
    splitter decodes the rank-0 token as an unrepairable one."""
    snapshot = list(inp)
    try:
        return bpe_repair(enc, inp, i, ranked_ids)[0]
    except IndexError:
        inp[:] = snapshot
        if strict:
            from ..codec.errors import DecodeDivergenceError

            raise DecodeDivergenceError(f"BPE repair at token {i} runs past the end of the text") from None
        return int(ranked_ids[0])


__all__ = ["HipArithmeticLM", "ByteTokenizer", "coder_params_from_quality", "bpe_repair", "repair_or_restore",
           "stop_candidates"]
