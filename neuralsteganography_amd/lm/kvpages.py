"""Paged KV cache of the native decode step (round 6): 32-position pages owned per stream.

The reference keeps one unbounded KV cache per message and runs every message in its own loop
(``code_base/arithmetic.py:96-122``; ``limit_past`` is a no-op, ``code_base/utils.py:19-30``).  Batched, that is B
caches of different, unknown lengths.  A dense ``[B, longest]`` allocation wastes the memory of every short
stream and must be copied to grow; here a stream's rows live in pages it owns:

* a PAGE holds 32 positions of one stream for every layer, ``[K|V][H][32][D]`` per layer in the cache's element
  type (1.18 MB for GPT-2-small fp16 over its 12 layers), so the attention of one (stream, head) reads 4 KiB
  contiguous per page and layer; pages live in SEGMENTS of ``seg_pages`` pages stored layer-major,
  ``[layer][page][K|V][H][32][D]``, so one layer's pages are contiguous (a decode step's attention walks one layer
  at a time: as few address-translation regions per launch as the dense cache had -- pages that interleave the
  layers measured 3-22 % slower, ``tools/paged_attn_probe.py``); a page's table entry is its layer-0 block's
  address and layer ``i`` is ``i * seg_pages * block`` elements further;
* the page TABLE ``[B, width]`` (uint64 device addresses, 0 = none) maps a stream's row ``r`` (position ``T0 + r``)
  to page ``table[b, r // 32]`` -- ``ns_decode_attention_paged`` reads it; per-stream cache lengths ``lens[B]``
  (int32, device) feed the position embedding and the attention and are advanced by the step's final layer norm;
* the POOL hands out pages from segments allocated on demand and kept across calls (warm pages); growth maps new
  segments and never copies a filled page, and a stream's pages return to the pool when it ends, so the memory in
  use follows the live tokens, not B x the longest stream.  When the device has no room for another segment the
  pool reports it (:class:`KVCapacityError` upstream), never PyTorch's out-of-memory.

The host keeps a mirror of the table and of the lengths (every slot advances one position per step), so page
bookkeeping needs no device read.  Pure host logic over torch tensors: the CPU tests drive it with CPU tensors.
"""

from __future__ import annotations

from typing import Callable, List, Optional

import numpy as np
import torch

PAGE_ROWS = 32


class KVPagePool:
    """Pages in layer-major segments of ``seg_pages`` pages each; a free list of page (layer-0 block) addresses.

    ``budget_bytes()`` says how much more device memory the pool may take (free memory minus what the caller must
    keep free); growth asks for ``max(needed, total / 4)`` pages, in whole segments, within that budget."""

    def __init__(self, n_layer: int, n_head: int, head_dim: int, dtype: torch.dtype, device,
                 budget_bytes: Optional[Callable[[], int]] = None, seg_pages: int = 1024):
        self.n_layer = int(n_layer)
        self.block_elems = 2 * n_head * PAGE_ROWS * head_dim  # one layer's [K|V][H][32][D]
        self.page_elems = self.n_layer * self.block_elems
        self.esize = torch.tensor([], dtype=dtype).element_size()
        self.block_bytes = self.block_elems * self.esize
        self.page_bytes = self.page_elems * self.esize
        self.dtype, self.device = dtype, torch.device(device)
        self.budget_bytes = budget_bytes
        self.seg_pages = max(1, int(seg_pages))
        self.segments: List[torch.Tensor] = []
        self._free = np.empty(0, dtype=np.int64)
        self._nfree = 0
        self.total = 0

    # ------------------------------------------------------------------
    def layer_offset(self, layer: int) -> int:
        """Elements from a page's address to its block of ``layer`` (``ns_decode_attention_paged``)."""
        return int(layer) * self.seg_pages * self.block_elems

    @property
    def free_pages(self) -> int:
        return self._nfree

    def growable_pages(self) -> int:
        if self.budget_bytes is None:
            return 1 << 40
        return max(0, int(self.budget_bytes()) // self.page_bytes)

    def _addresses(self, seg: torch.Tensor) -> np.ndarray:
        return seg.data_ptr() + self.block_bytes * np.arange(self.seg_pages, dtype=np.int64)

    def add_segment(self, npages: int) -> bool:
        """Map at least ``npages`` more pages (whole segments, one allocation each); False (nothing mapped) if the
        device cannot hold them."""
        nseg = -(-int(npages) // self.seg_pages)
        if nseg <= 0:
            return False
        new = []
        for _ in range(nseg):
            try:
                new.append(torch.empty((self.n_layer, self.seg_pages, self.block_elems), dtype=self.dtype,
                                       device=self.device))
            except torch.OutOfMemoryError:
                return False
        for seg in new:
            self.segments.append(seg)
            self._push(self._addresses(seg)[::-1])  # pages are taken from the top: lowest addresses first
            self.total += self.seg_pages
        return True

    def _push(self, addrs: np.ndarray) -> None:
        n = addrs.size
        if self._nfree + n > self._free.size:
            grown = np.empty(max(self._nfree + n, 2 * self._free.size), dtype=np.int64)
            grown[: self._nfree] = self._free[: self._nfree]
            self._free = grown
        self._free[self._nfree: self._nfree + n] = addrs
        self._nfree += n

    def take(self, n: int) -> Optional[np.ndarray]:
        """``n`` page addresses, growing the pool within its budget; None (nothing taken) if it cannot."""
        n = int(n)
        if n <= 0:
            return np.empty(0, dtype=np.int64)
        if self._nfree < n:
            short = n - self._nfree
            room = self.growable_pages() // self.seg_pages * self.seg_pages
            if room < short:
                return None
            want = min(room, max(short, self.total // 4))
            if not self.add_segment(want) and not (want > short and self.add_segment(short)):
                return None
        out = self._free[self._nfree - n: self._nfree][::-1].copy()
        self._nfree -= n
        return out

    def give(self, addrs: np.ndarray) -> None:
        addrs = np.asarray(addrs, dtype=np.int64)
        if addrs.size:
            self._push(addrs[::-1])

    def reset(self) -> None:
        """Every page free again (a new call: the previous call's tables are dropped)."""
        self._free = np.empty(0, dtype=np.int64)
        self._nfree = 0
        for seg in self.segments:
            self._push(self._addresses(seg)[::-1])

    def release_memory(self) -> None:
        self.segments = []
        self._free = np.empty(0, dtype=np.int64)
        self._nfree = 0
        self.total = 0


class PagedKV:
    """One call's page table, per-stream lengths and their host mirrors over a :class:`KVPagePool`.

    Slots are rows ``0..B-1``.  ``lens`` (device int32) is advanced by the decode step itself; the host mirror
    ``lens_host`` is advanced by :meth:`advance` (every slot moves one position per step, finished ones too: their
    attention is skipped, their length only feeds the position embedding of rows nobody reads).  ``version`` changes
    whenever a device tensor is replaced (a wider table, a compaction): a captured graph must then be re-captured."""

    def __init__(self, pool: KVPagePool, B: int, T0: int, width: int):
        self.pool, self.B, self.T0 = pool, int(B), int(T0)
        dev = pool.device
        self.width = max(1, int(width))
        self.table = torch.zeros((self.B, self.width), dtype=torch.int64, device=dev)
        self.host = np.zeros((self.B, self.width), dtype=np.int64)
        self.nch = np.zeros(self.B, dtype=np.int64)
        self.lens = torch.full((self.B,), self.T0, dtype=torch.int32, device=dev)
        self.lens_host = np.full(self.B, self.T0, dtype=np.int64)
        self.version = 0
        self.in_use = 0  # pages mapped now, and the most ever mapped at once in this call
        self.peak = 0

    # ------------------------------------------------------------------
    def pages_in_use(self) -> int:
        return int(self.nch.sum())

    def _grow_width(self, need: int) -> None:
        w = max(int(need), 2 * self.width)
        t = torch.zeros((self.B, w), dtype=torch.int64, device=self.table.device)
        t[:, : self.width] = self.table
        h = np.zeros((self.B, w), dtype=np.int64)
        h[:, : self.width] = self.host
        self.table, self.host, self.width = t, h, w
        self.version += 1

    def ensure(self, slots, upto) -> np.ndarray:
        """Give every slot in ``slots`` the pages for positions below ``upto`` (scalar or per slot).  All or nothing
        per slot; returns the slots that could not be served (the pool is out of memory)."""
        slots = np.asarray(slots, dtype=np.int64).reshape(-1)
        if slots.size == 0:
            return slots
        upto = np.broadcast_to(np.asarray(upto, dtype=np.int64), slots.shape)
        need = np.maximum(0, (upto - self.T0 + PAGE_ROWS - 1) // PAGE_ROWS)
        deficit = np.maximum(0, need - self.nch[slots])
        if not deficit.any():
            return np.empty(0, dtype=np.int64)
        if int(need.max()) > self.width:
            self._grow_width(int(need.max()))
        pages = self.pool.take(int(deficit.sum()))
        if pages is not None:
            self._assign(slots, deficit, pages)
            return np.empty(0, dtype=np.int64)
        failed = []
        for s, d in zip(slots.tolist(), deficit.tolist()):  # the pool is short: serve slots in order while it lasts
            if d == 0:
                continue
            p = self.pool.take(d)
            if p is None:
                failed.append(s)
            else:
                self._assign(np.array([s]), np.array([d]), p)
        return np.asarray(failed, dtype=np.int64)

    def _assign(self, slots: np.ndarray, deficit: np.ndarray, pages: np.ndarray) -> None:
        keep = deficit > 0
        slots, deficit = slots[keep], deficit[keep]
        rows = np.repeat(slots, deficit)
        starts = np.repeat(np.cumsum(deficit) - deficit, deficit)
        cols = self.nch[rows] + (np.arange(rows.size) - starts)
        self.host[rows, cols] = pages
        self.nch[slots] += deficit
        self.in_use += int(pages.size)
        self.peak = max(self.peak, self.in_use)
        dev = self.table.device
        self.table[torch.from_numpy(rows).to(dev), torch.from_numpy(cols).to(dev)] = torch.from_numpy(pages).to(dev)

    def release(self, slots) -> None:
        """Return the pages of ``slots`` to the pool and clear their table rows (the streams have ended)."""
        slots = np.asarray(slots, dtype=np.int64).reshape(-1)
        if slots.size == 0:
            return
        n = int(self.nch[slots].max(initial=0))
        if n:
            pages = self.host[slots, :n]
            pages = pages[pages != 0]
            self.pool.give(pages)
            self.in_use -= int(pages.size)
            self.host[slots, :n] = 0
            self.table[torch.from_numpy(slots).to(self.table.device), :n] = 0
        self.nch[slots] = 0

    def reset(self, slots) -> None:
        """``release`` + the slots' cache lengths back to the shared context (a new message starts there)."""
        slots = np.asarray(slots, dtype=np.int64).reshape(-1)
        self.release(slots)
        if slots.size:
            self.lens[torch.from_numpy(slots).to(self.lens.device)] = self.T0
            self.lens_host[slots] = self.T0

    def advance(self, n: int = 1) -> None:
        self.lens_host += int(n)

    def steps_reserved(self, slots) -> int:
        """Decode steps every slot in ``slots`` can still take within its pages."""
        slots = np.asarray(slots, dtype=np.int64).reshape(-1)
        if slots.size == 0:
            return 1 << 30
        return int((self.T0 + PAGE_ROWS * self.nch[slots] - self.lens_host[slots]).min())

    def compact(self, keep) -> None:
        """Keep only the slots ``keep`` (in that order) as rows 0..len(keep)-1; the other slots must have been
        released.  Page tables move with their rows: no page is copied."""
        keep = np.asarray(keep, dtype=np.int64).reshape(-1)
        gone = np.setdiff1d(np.arange(self.B), keep)
        if gone.size and self.nch[gone].any():
            raise RuntimeError("compact: a dropped slot still holds pages")
        kt = torch.from_numpy(keep).to(self.table.device)
        self.table = self.table.index_select(0, kt).contiguous()
        self.lens = self.lens.index_select(0, kt).contiguous()
        self.host, self.nch, self.lens_host = self.host[keep], self.nch[keep], self.lens_host[keep]
        self.B = int(keep.size)
        self.version += 1
