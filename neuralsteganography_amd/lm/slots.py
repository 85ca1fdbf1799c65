"""Slot schedulers of the native encode / decode loops (round 6): slot refill, page mapping, eviction, compaction.

The reference encodes every message in its own loop with its own KV cache (``code_base/arithmetic.py:96-122``; the
api splits a secret into independent chunks, ``src/neuralstego/api.py:736-747``).  Batched on the GPU, B messages
share one decode step; covers differ in length (a peaked, trained-LM-like row gives far longer covers than the
mean), so a lockstep batch spends its steps on finished streams.  Here messages queue for S SLOTS:

* every slot runs one message from the shared context (cache length ``T0``, the prefill's logits as its first
  coder step's row) to its end, with its own cache length and position ids (``lens[b] % n_positions``,
  ``code_base/arithmetic.py:44-48``) and its own KV pages (``lm/kvpages.py``);
* every ``check_every`` steps the host reads the coder states once: finished slots hand their tokens (or bits) over
  and take the next queued message; pages are mapped ahead for the live slots;
* when the device runs out of pages, the youngest live messages are EVICTED (pages returned, message re-queued and
  later re-run from its start -- the same tokens, since a stream's result does not depend on its neighbours) rather
  than failing; a message that cannot fit alone raises :class:`KVCapacityError`;
* when the queue is empty and at most half the slots are live, the live slots are COMPACTED into a smaller batch
  (page tables move with their rows, no KV is copied): the GEMMs stop computing finished rows.

A stream's logits are bit-identical whatever the batch it runs in (the decode step is batch-invariant, including the
paged attention), so a message's tokens are the same alone, in lockstep, or refilled into any slot.  Between host
checks the step (coder + GPT-2 decode) is one captured hipGraph replay; a graph is re-captured when a buffer it
holds is replaced (a wider page table, a longer history, a compaction).
"""

from __future__ import annotations

from collections import deque
from typing import List, Optional, Sequence

import numpy as np

from .. import _lib
from ..coder import EncodeSession, _state_fields, _stats_rows
from ..exceptions import KVCapacityError


class _SlotGraph:
    """``body()`` (one whole step into fixed buffers) run once eagerly on a side stream -- a real step, which also
    warms every kernel up -- then captured as a hipGraph and replayed per later step."""

    def __init__(self, body):
        import torch

        self.body = body
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            body()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            body()

    def replay(self) -> None:
        self.graph.replay()


def _layout_key(*tensors) -> tuple:
    return tuple(t.data_ptr() if t is not None else 0 for t in tensors)


class _Pinned:
    """Double-buffered pinned host copies of a device tensor, taken asynchronously on the current stream with an
    event (the check pipeline of the slot loops: a check reads the PREVIOUS check's copy, whose event the GPU has
    passed, while the steps enqueued since keep it busy)."""

    def __init__(self):
        self.bufs = [None, None]
        self.k = 0

    def take(self, dev_tensor):
        import torch

        b = self.bufs[self.k]
        if b is None or b.shape != dev_tensor.shape or b.dtype != dev_tensor.dtype:
            b = self.bufs[self.k] = torch.empty(dev_tensor.shape, dtype=dev_tensor.dtype, pin_memory=True)
        b.copy_(dev_tensor, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.k ^= 1
        return b, ev


def _rows_after(event, side, tensor, rows, ncols=None):
    """``tensor[rows, :ncols]`` on the host, gathered on the ``side`` stream once ``event`` has passed (rows that no
    later step writes: finished streams), without waiting for the steps enqueued on the main stream since."""
    import torch

    with torch.cuda.stream(side):
        side.wait_event(event)
        idx = torch.as_tensor(np.asarray(rows, dtype=np.int64), device=tensor.device)
        out = tensor.index_select(0, idx)
        if ncols is not None:
            out = out[:, :ncols]
        host = out.cpu()
    return host


class SlotEncoder:
    """Encode ``bit_lists`` through ``slots`` slots of ``provider.lm`` (a native :class:`BatchedGPT2`)."""

    def __init__(self, provider, ctx, bit_lists: Sequence[Sequence[int]], context: Sequence[int], *, slots: int,
                 finish: bool, stop_text: Optional[str], stats: bool, check_every: int, stall_steps: int,
                 hard_cap: int, use_graph: bool, compact: bool = True):
        self.p, self.lm, self.ctx = provider, provider.lm, ctx
        self.bits = bit_lists
        self.N = len(bit_lists)
        self.S = max(1, min(int(slots), self.N))
        self.context = context
        self.finish, self.stop_text, self.stats = finish, stop_text, stats
        self.check_every, self.stall_steps, self.hard_cap = int(check_every), int(stall_steps), int(hard_cap)
        self.use_graph, self.allow_compact = use_graph, compact
        self.evictions = 0
        self.compactions = 0
        self.max_live = 0
        self.kv_peak = 0

    # ------------------------------------------------------------------
    def run(self):
        import torch

        from ..codec.errors import ArithmeticRangeError
        from .arithmetic import _StopCheck

        lm, S, N = self.lm, self.S, self.N
        max_bits = max(len(b) for b in self.bits)
        # initial token-history / page-table width (both grow on demand; a provider may set a small one in tests)
        budget = getattr(self.p, "slot_budget_tokens", None) or 2 * max_bits + 64
        logits = lm.prefill(self.context, S, budget)  # [S, ld]: every slot starts on the context's logits
        first = lm.first_logits
        T0 = lm.kv.T0
        stride = max(1, (max_bits + 7) // 8)
        sess = EncodeSession(self.ctx, self.bits[:S], max_tokens=budget, stats=self.stats, payload_stride=stride)
        stop = _StopCheck(self.p, sess, self.stop_text) if self.stop_text is not None else None
        slot_msg = np.arange(S, dtype=np.int64)  # message per slot, -1 = empty
        queue = deque(range(S, N))
        tokens: List[Optional[List[int]]] = [None] * N
        stats_out: List[Optional[dict]] = [None] * N
        last_pos = np.zeros(S, dtype=np.int64)
        last_move = np.zeros(S, dtype=np.int64)
        t = 0
        graph, gkey = None, None
        admit_blocked = False

        def body():
            tok = sess.step(logits, finish_sent=self.finish)
            if stop is not None:
                stop.flag(tok)
            lm.step_static(tok)

        skip = getattr(self.p, "skip_done", True)  # finished streams skip their attention (A/B switch)

        def done_view():
            return sess.state.view(torch.int32)[:, 7] if skip else None

        # check pipeline (graph replays, no per-step stop test): a check processes the coder states copied at the
        # PREVIOUS check while the steps enqueued since run -- the GPU never waits for the host; a finished slot is
        # seen one period later (it idles through it, skipping its attention) and its tokens are gathered on a side
        # stream.  Eager or stop-text loops read the states synchronously.
        pipelined = self.use_graph and stop is None
        pin, pending = _Pinned(), None
        side = torch.cuda.Stream() if pipelined else None
        lm.begin_static(logits)
        lm.done_flags = done_view()
        try:
            while True:
                if stop is not None and t > 0:
                    stop.check()
                if t % self.check_every == 0:
                    if pipelined:
                        f, ev = (None, None) if pending is None else (pending[0], pending[1])
                        if ev is not None:
                            ev.synchronize()
                            f = _state_fields(f)
                    else:
                        f, ev = sess.fields(), None
                    live = slot_msg >= 0
                    flags = f["flags"] if f is not None else np.zeros(sess.B, dtype=np.uint32)
                    # ---- harvest finished slots
                    fin = np.nonzero(live & ((flags & _lib.NS_ST_DONE) != 0))[0]
                    if fin.size:
                        bad = fin[(flags[fin] & _lib.NS_ST_ERR_RANGE) != 0]
                        if bad.size:
                            raise ArithmeticRangeError(
                                f"streams {slot_msg[bad].tolist()[:8]} found no CDF bucket for the payload index")
                        nt = f["ntokens"][fin]
                        if int(nt.max(initial=0)) > sess.hist.shape[1]:
                            raise RuntimeError("token history overflow")
                        ncol = max(1, int(nt.max()))
                        if ev is not None:
                            host = _rows_after(ev, side, sess.hist, fin, ncol).numpy()
                            acc = _rows_after(ev, side, sess.stats_acc, fin).numpy() if self.stats else None
                        else:
                            host = sess.hist[torch.as_tensor(fin, device=sess.hist.device), :ncol].cpu().numpy()
                            acc = sess.stats_acc[torch.as_tensor(fin, device=sess.hist.device)].cpu().numpy() \
                                if self.stats else None
                        for j, s in enumerate(fin.tolist()):
                            m = int(slot_msg[s])
                            tokens[m] = host[j, : int(nt[j])].tolist()
                            if self.stats:
                                stats_out[m] = _stats_rows(acc[j:j + 1], f["bit_pos"][s:s + 1])[0]
                        lm.kv.release(fin)
                        slot_msg[fin] = -1
                        admit_blocked = False
                        live = slot_msg >= 0
                    # ---- stalls (the reference loops forever on a stream that fixes no bit)
                    pos = f["bit_pos"] if f is not None else last_pos
                    ntok = f["ntokens"] if f is not None else np.zeros(sess.B, dtype=np.int64)
                    moved = live & (pos != last_pos)
                    last_pos[moved], last_move[moved] = pos[moved], t
                    stuck = np.nonzero(live & (((t - last_move) >= self.stall_steps) |
                                               (ntok >= self.hard_cap)))[0]
                    if stuck.size:
                        ids = slot_msg[stuck].tolist()[:8]
                        if all(pos[s] >= len(self.bits[slot_msg[s]]) for s in stuck):
                            raise ArithmeticRangeError(
                                f"finish_sent: streams {ids} produced no sentence-ending token in "
                                f"{self.stall_steps} tokens (the reference would keep generating forever)")
                        raise ArithmeticRangeError(
                            f"streams {ids} fixed no payload bit for {self.stall_steps} tokens: the interval "
                            "straddles the midpoint and one token takes the whole range (the reference coder "
                            "has no underflow handling and would loop forever)")
                    # ---- refill empty slots from the queue
                    empty = np.nonzero(~live)[0]
                    if queue and empty.size and not admit_blocked:
                        room = lm.pool.free_pages + lm.pool.growable_pages() - int(live.sum()) - 1
                        n_adm = int(min(empty.size, len(queue), max(0, room)))
                        if n_adm:
                            sl = empty[:n_adm]
                            ms = [queue.popleft() for _ in range(n_adm)]
                            self._admit(sess, logits, first, sl, ms, slot_msg, last_pos, last_move, t)
                            live = slot_msg >= 0
                    nlive = int(live.sum())
                    self.max_live = max(self.max_live, nlive)
                    if nlive == 0:
                        if not queue:
                            break
                        raise KVCapacityError("no device memory for even one stream's first KV page")
                    # ---- compaction: the queue is drained and at most half the slots are live
                    compacted = False
                    if self.allow_compact and not queue and nlive <= sess.B // 2 and sess.B > 1:
                        compacted = True
                        if f is not None:
                            ntok = ntok[np.nonzero(live)[0]]
                        keep = np.nonzero(live)[0]
                        sess, logits, slot_msg, last_pos, last_move = self._compact(
                            sess, logits, keep, slot_msg, last_pos, last_move, stop)
                        if stop is not None:
                            stop.sess = sess
                            stop.hit = torch.zeros(sess.B, dtype=torch.bool, device=sess.state.device)
                        live = slot_msg >= 0
                        self.compactions += 1
                    # ---- pages for the next check_every + 1 steps; evict the youngest when the device is full
                    self._map_pages(sess, slot_msg, queue, live, T0)
                    if (slot_msg >= 0).sum() < nlive:
                        admit_blocked = True
                    # ---- token history for the next steps (two periods ahead of a pipelined state copy)
                    ahead = (2 if pipelined else 1) * self.check_every + 1
                    if int(ntok.max(initial=0)) + ahead > sess.hist.shape[1]:
                        sess.ensure_history(ahead)
                    if stop is not None:
                        stop.sess = sess
                    if pipelined:
                        pending = pin.take(sess.state)
                key = _layout_key(logits, sess.state, sess.hist, sess.payload, lm.kv.table, lm.kv.lens,
                                  sess.stats_acc) + (lm.kv.version,)
                if self.use_graph:
                    if graph is None or key != gkey:
                        graph = None
                        lm.done_flags = done_view()
                        lm.begin_static(logits)
                        graph, gkey = _SlotGraph(body), key
                    else:
                        graph.replay()
                else:
                    lm.done_flags = done_view()
                    lm.begin_static(logits)
                    body()
                lm.advance(1)
                t += 1
        finally:
            if graph is not None:  # a pipelined loop ends with steps still queued on its graph
                torch.cuda.current_stream().synchronize()
            lm.done_flags = None
            del graph
        self.sess = sess
        self.kv_peak = lm.kv.peak
        return tokens, (stats_out if self.stats else None)

    # ------------------------------------------------------------------
    def _admit(self, sess, logits, first, slots, msgs, slot_msg, last_pos, last_move, t):
        import torch

        lm = self.lm
        sess.load_slots(slots, [self.bits[m] for m in msgs])
        lm.kv.reset(slots)
        idx = torch.as_tensor(np.asarray(slots, dtype=np.int64), device=logits.device)
        logits.index_copy_(0, idx, first.expand(len(slots), -1).to(logits.dtype))
        slot_msg[slots] = msgs
        last_pos[slots] = 0
        last_move[slots] = t

    def _map_pages(self, sess, slot_msg, queue, live, T0):
        """Pages for every live slot's next ``check_every + 1`` positions; on a full device evict the youngest live
        messages (fewest positions fed) back to the queue's front until the others are served."""
        lm = self.lm
        while True:
            sl = np.nonzero(slot_msg >= 0)[0]
            if sl.size == 0:
                return
            failed = lm.kv.ensure(sl, lm.kv.lens_host[sl] + self.check_every + 1)
            if failed.size == 0:
                return
            if sl.size == 1:
                raise KVCapacityError(
                    f"message {int(slot_msg[sl[0]])} needs more KV pages than the device holds "
                    f"({lm.pool.total} pages of {lm.pool.page_bytes} B)")
            victim = np.asarray([sl[np.argmin(lm.kv.lens_host[sl])]])  # the youngest: fewest positions fed
            queue.appendleft(int(slot_msg[victim[0]]))
            lm.kv.release(victim)
            sess.park_slots(victim)
            slot_msg[victim] = -1
            self.evictions += 1

    def _compact(self, sess, logits, keep, slot_msg, last_pos, last_move, stop):
        import torch

        lm = self.lm
        empty = np.setdiff1d(np.arange(sess.B), keep)
        lm.kv.release(empty)
        lm.kv.compact(keep)
        lm.B = lm.kv.B
        sess.compact(keep)
        idx = torch.as_tensor(keep, device=logits.device)
        logits = logits.index_select(0, idx).contiguous()
        return sess, logits, slot_msg[keep].copy(), last_pos[keep].copy(), last_move[keep].copy()


class SlotDecoder:
    """Decode ``token_lists`` through ``slots`` slots, longest first: pages are mapped as the streams grow (as the
    encoder maps them, with the same eviction), and a slot's end is known on the host from its token count."""

    def __init__(self, provider, ctx, token_lists: Sequence[Sequence[int]], context: Sequence[int], *, slots: int,
                 use_graph: bool, check_every: int = 16, compact: bool = True):
        self.p, self.lm, self.ctx = provider, provider.lm, ctx
        self.lists = token_lists
        self.N = len(token_lists)
        self.S = max(1, min(int(slots), self.N))
        self.context = context
        self.use_graph, self.check_every, self.allow_compact = use_graph, int(check_every), compact
        self.compactions = 0
        self.evictions = 0

    def run(self) -> List[List[int]]:
        import torch

        from .. import _lib as L
        from ..codec.errors import DecodeDivergenceError
        from ..coder import _bit_rows_to_lists, _ptr, _state_tensor, _stream_handle

        lm, S, N = self.lm, self.S, self.N
        lens_all = np.asarray([len(t) for t in self.lists], dtype=np.int64)
        Tcap = max(1, int(lens_all.max(initial=0)))
        order = np.argsort(-lens_all, kind="stable")  # longest first: the tail is short messages
        logits = lm.prefill(self.context, S, Tcap + 1)
        first = lm.first_logits
        T0 = lm.kv.T0
        dev = logits.device
        P = self.ctx.params.precision
        out_stride = int((Tcap * P + P + 7) // 8 + 8)
        st = {"tokmat": torch.zeros((S, Tcap), dtype=torch.int32, device=dev),
              "nlen": torch.zeros(S, dtype=torch.int32, device=dev),
              "stop": torch.zeros(S, dtype=torch.int32, device=dev),
              "state": _state_tensor(S, dev),
              "out_bits": torch.zeros((S, out_stride), dtype=torch.uint8, device=dev)}
        self.ctx.check(L.lib().ns_init_state(self.ctx._h, _ptr(st["state"]), S, _stream_handle()), "ns_init_state")
        st["state"].view(torch.int32)[:, 7] = L.NS_ST_DONE
        slot_msg = np.full(S, -1, dtype=np.int64)
        nlen_host = np.zeros(S, dtype=np.int64)
        queue = deque(order.tolist())
        out: List[Optional[List[int]]] = [None] * N
        init_row = torch.tensor([[0, 1 << P, 0, 0]], dtype=torch.int64, device=dev)
        p = self.ctx.params
        graph, gkey = None, None
        bufs = {}
        admit_blocked = False

        def body():
            tix = lm.kv.lens - T0
            idx = tix.clamp(0, Tcap - 1).long().unsqueeze(1)
            tok = torch.gather(st["tokmat"], 1, idx).squeeze(1).contiguous()
            act = (tix < st["nlen"]).to(torch.uint8)
            last = (tix == st["nlen"] - 1).to(torch.uint8)
            bufs["tok"], bufs["act"], bufs["last"] = tok, act, last
            rc = L.lib().ns_decode_step(self.ctx._h, _ptr(logits), logits.stride(0), st["state"].shape[0], _ptr(tok),
                                        _ptr(last), _ptr(act), _ptr(st["state"]), _ptr(st["out_bits"]), out_stride,
                                        float(p.temp), int(p.topk), self.ctx._banned, self.ctx._nbanned, None, 0,
                                        _stream_handle())
            self.ctx.check(rc, "ns_decode_step")
            lm.step_static(tok)

        t = 0
        # check pipeline as in the encoder: a slot counts as finished once the event recorded at the previous check
        # has passed with its last token fed (its message and positions as of that check); its bits are gathered on a
        # side stream while the steps enqueued since run
        pipelined = self.use_graph
        side = torch.cuda.Stream() if pipelined else None
        pending = None
        try:
            while True:
                if t % self.check_every == 0:
                    live = slot_msg >= 0
                    if pipelined:
                        if pending is not None:
                            ev, msg_then, fed_then = pending
                            ev.synchronize()
                            done = live & (slot_msg == msg_then) & (fed_then >= nlen_host)
                        else:
                            ev, done = None, np.zeros(slot_msg.shape, dtype=bool)
                    else:
                        ev, done = None, live & ((lm.kv.lens_host - T0) >= nlen_host)
                    fin = np.nonzero(done)[0]
                    if fin.size:
                        if ev is not None:
                            srows = _rows_after(ev, side, st["state"], fin).numpy()
                            f = _state_fields(torch.from_numpy(srows))
                            rows = _rows_after(ev, side, st["out_bits"], fin)
                        else:
                            f = _state_fields(st["state"][torch.as_tensor(fin, device=dev)])
                            rows = st["out_bits"][torch.as_tensor(fin, device=dev)]
                        bad = fin[(f["flags"] & L.NS_ST_ERR_DIVERGE) != 0]
                        if bad.size:
                            raise DecodeDivergenceError(
                                f"streams {slot_msg[bad].tolist()[:8]}: received token outside the kept top-k")
                        got = _bit_rows_to_lists(rows, f["bit_pos"])
                        for j, s in enumerate(fin.tolist()):
                            out[int(slot_msg[s])] = got[j]
                        lm.kv.release(fin)
                        slot_msg[fin] = -1
                        nlen_host[fin] = 0
                        admit_blocked = False
                        fi = torch.as_tensor(fin, device=dev)
                        st["nlen"][fi] = 0
                        st["stop"][fi] = 0
                        live = slot_msg >= 0
                    empty = np.nonzero(~live)[0]
                    if queue and empty.size and not admit_blocked:
                        room = lm.pool.free_pages + lm.pool.growable_pages() - int(live.sum()) - 1
                        n_adm = int(min(empty.size, len(queue), max(0, room)))
                        if n_adm:
                            adm_s = empty[:n_adm]
                            adm_m = [queue.popleft() for _ in range(n_adm)]
                            lm.kv.reset(adm_s)
                            self._admit(st, logits, first, init_row, adm_s, adm_m, slot_msg, nlen_host, T0, Tcap)
                            live = slot_msg >= 0
                    # pages for the next check_every + 1 positions (never past a message's last fed token); on a full
                    # device the youngest messages go back to the queue's front (re-decoded later: the same bits)
                    while live.any():
                        sl = np.nonzero(live)[0]
                        upto = np.minimum(lm.kv.lens_host[sl] + self.check_every + 1, T0 + nlen_host[sl])
                        if lm.kv.ensure(sl, upto).size == 0:
                            break
                        if sl.size == 1:
                            raise KVCapacityError(f"message {int(slot_msg[sl[0]])} ({int(nlen_host[sl[0]])} tokens) "
                                                  "needs more KV pages than the device holds")
                        v = sl[np.argmin(lm.kv.lens_host[sl])]
                        queue.appendleft(int(slot_msg[v]))
                        lm.kv.release([v])
                        vi = torch.as_tensor([int(v)], device=dev)
                        st["nlen"][vi] = 0
                        st["stop"][vi] = 0
                        slot_msg[v], nlen_host[v] = -1, 0
                        live = slot_msg >= 0
                        admit_blocked = True
                        self.evictions += 1
                    if not live.any():
                        break
                    if self.allow_compact and not queue and int(live.sum()) <= st["state"].shape[0] // 2 and \
                            st["state"].shape[0] > 1:
                        keep = np.nonzero(live)[0]
                        lm.kv.release(np.setdiff1d(np.arange(st["state"].shape[0]), keep))
                        lm.kv.compact(keep)
                        lm.B = lm.kv.B
                        ki = torch.as_tensor(keep, device=dev)
                        for k in st:
                            st[k] = st[k].index_select(0, ki).contiguous()
                        logits = logits.index_select(0, ki).contiguous()
                        slot_msg, nlen_host = slot_msg[keep].copy(), nlen_host[keep].copy()
                        self.compactions += 1
                    lm.stop_len = st["stop"] if getattr(self.p, "skip_done", True) else None
                    if pipelined:
                        ev_now = torch.cuda.Event()
                        ev_now.record()
                        pending = (ev_now, slot_msg.copy(), lm.kv.lens_host - T0)
                key = _layout_key(logits, st["state"], st["tokmat"], lm.kv.table, lm.kv.lens) + (lm.kv.version,)
                if self.use_graph:
                    if graph is None or key != gkey:
                        graph = None
                        lm.begin_static(logits)
                        graph, gkey = _SlotGraph(body), key
                    else:
                        graph.replay()
                else:
                    lm.begin_static(logits)
                    body()
                lm.advance(1)
                t += 1
        finally:
            if graph is not None:
                torch.cuda.current_stream().synchronize()
            lm.stop_len = None
            del graph
        return out

    def _admit(self, st, logits, first, init_row, slots, msgs, slot_msg, nlen_host, T0, Tcap):
        import torch

        dev = logits.device
        n = len(slots)
        mat = np.zeros((n, Tcap), dtype=np.int32)
        nl = np.zeros(n, dtype=np.int64)
        for i, m in enumerate(msgs):
            tl = self.lists[m]
            nl[i] = len(tl)
            if len(tl):
                mat[i, : len(tl)] = np.asarray(tl, dtype=np.int32)
        idx = torch.as_tensor(np.asarray(slots, dtype=np.int64), device=dev)
        st["tokmat"][idx] = torch.from_numpy(mat).to(dev)
        nlt = torch.from_numpy(nl.astype(np.int32)).to(dev)
        st["nlen"][idx] = nlt
        st["stop"][idx] = nlt + (T0 - 1)
        st["state"][idx] = init_row.expand(n, 4)
        st["out_bits"][idx] = 0
        logits.index_copy_(0, idx, first.expand(n, -1).to(logits.dtype))
        slot_msg[slots] = msgs
        nlen_host[slots] = nl
