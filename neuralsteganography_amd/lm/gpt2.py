"""Batched GPT-2 forward with a preallocated KV cache, writing logits straight into the coder's layout.

This is the L1 "LM runtime" of SURVEY.md §1 rebuilt for batch B (PyTorch-ROCm holds the weights and the KV cache;
in the fp16 GPU configuration every GEMM and attention of the forward runs on the library's own MFMA kernels, see
below).  It reproduces the reference's forward semantics (``code_base/arithmetic.py:12-48,115-122``):

* the first call runs the whole context with default positions ``0..T-1``;
* every later call feeds ONE token per stream with ``position_ids = cache_len % n_positions``
  (``_position_ids_for_cache``, ``:44-48``) and attends to the whole cache: the reference never truncates
  it (``limit_past`` slices head_dim, a no-op, ``code_base/utils.py:19-30``).

In fp16 on the GPU (the product configuration) every forward runs on hand-written HIP kernels whose per-stream
results do not depend on the batch size (``include/nsg_lm.h``: MFMA GEMMs with the bias / gelu / residual
epilogues fused, layer norms, embedding; ``include/nsg_attn.h``: the decode step's KV append fused with a
fixed-split online-softmax attention, HBM-bound on the cache, and a causal MFMA flash attention for whole
sequences): the decode steps, the shared-context prefill, the guard's scoring forward and the ``max_context``
window forward.  A cover encoded in a batch of B streams decodes to the same logits alone, and a text scores the
same alone or in a batch.  fp32 compute and the CPU keep PyTorch (``addmm`` + ``scaled_dot_product_attention``) as
the forward's reference configuration (tests pin the two against each other and against Hugging Face).

Logits are produced as ``h @ wte^T`` into a ``[B, ld]`` buffer with ``ld = row_stride(V)`` (zero weight
columns beyond V), so the coder reads 16-byte-aligned rows without a copy.  Weights are taken from a
Hugging Face ``GPT2LMHeadModel`` (pretrained when available offline, random-init otherwise).
"""

from __future__ import annotations

import math
import weakref
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ..coder import row_stride


@dataclass
class GPT2Shape:
    n_layer: int
    n_head: int
    n_embd: int
    vocab: int
    n_positions: int
    eps: float


class BatchedGPT2:
    """GPT-2 decoder for B streams in lockstep.

    ``compute_dtype`` is the weight/activation dtype (fp16 on the GPU by default); ``logits_dtype`` is what
    the coder reads (``torch.float32`` or ``torch.float16``)."""

    def __init__(self, hf_model, *, device=None, compute_dtype=None, logits_dtype=torch.float32, kv_dtype="fp16",
                 logit_scale: float = 1.0):
        cfg = hf_model.config
        self.shape = GPT2Shape(cfg.n_layer, cfg.n_head, cfg.n_embd, cfg.vocab_size, cfg.n_positions,
                               cfg.layer_norm_epsilon)
        self.device = _normalise_device(torch.device(device) if device is not None else next(hf_model.parameters()).device)
        if compute_dtype is None:
            compute_dtype = torch.float16 if self.device.type == "cuda" else torch.float32
        self.dtype = compute_dtype
        self.logits_dtype = logits_dtype
        self.ld = row_stride(self.shape.vocab, "f16" if logits_dtype == torch.float16 else "f32")
        sd = {k: v.detach() for k, v in hf_model.state_dict().items()}
        dev, dt = self.device, self.dtype

        def w(name):
            return sd[name].to(device=dev, dtype=dt).contiguous()

        pre = "transformer."
        self.wte = w(pre + "wte.weight")
        self.wpe = w(pre + "wpe.weight")
        self.layers = []
        for i in range(self.shape.n_layer):
            p = f"{pre}h.{i}."
            self.layers.append({
                "ln1_w": w(p + "ln_1.weight"), "ln1_b": w(p + "ln_1.bias"),
                "qkv_w": w(p + "attn.c_attn.weight"), "qkv_b": w(p + "attn.c_attn.bias"),
                "o_w": w(p + "attn.c_proj.weight"), "o_b": w(p + "attn.c_proj.bias"),
                "ln2_w": w(p + "ln_2.weight"), "ln2_b": w(p + "ln_2.bias"),
                "fc_w": w(p + "mlp.c_fc.weight"), "fc_b": w(p + "mlp.c_fc.bias"),
                "pr_w": w(p + "mlp.c_proj.weight"), "pr_b": w(p + "mlp.c_proj.bias"),
            })
        self.lnf_w = w(pre + "ln_f.weight")
        self.lnf_b = w(pre + "ln_f.bias")
        # lm_head = wte^T padded to ld columns (zeros beyond V): logits land in the coder's row layout
        # logit_scale != 1 (synthetic "trained-entropy" rows, bench / tests only): the head alone is scaled, so a
        # random-init model's near-uniform rows (~15 bits of entropy) peak like a trained LM's (a few bits)
        head = torch.zeros((self.shape.n_embd, self.ld), device=dev, dtype=dt)
        head[:, : self.shape.vocab] = self.wte.t() if logit_scale == 1.0 else (self.wte.float().t() * float(logit_scale)).to(dt)
        self.head = head
        self.B = 0
        self.L = 0
        self.T0 = 0  # positions held once in the shared prefix cache (kp, vp) instead of per stream
        self.position_cap = None  # optional cap on the initial per-stream cache length (the cache still grows)
        self.chunked_cache = True  # native decode: chunk-plane KV layout (False: plain per-pair rows; A/B only)
        # attention window (opt-in, 0 = the reference's unbounded cache): decode steps attend to the last `window`
        # positions only -- a sliding-window approximation bounding the per-step KV traffic (native path only)
        self.window = 0
        self.kp = self.vp = None
        self.k_cache = self.v_cache = None
        # Decode steps in fp16 on the GPU run entirely on the batch-invariant HIP kernels (include/nsg_lm.h and
        # the fixed-split attention of include/nsg_attn.h; fail loudly if the library is missing): a stream's
        # logits are bit-identical whatever the batch it runs in, so a cover encoded among B streams decodes
        # alone.  Weights are kept transposed ([N, K], K contiguous).  fp32 compute and the CPU keep the PyTorch
        # path (SDPA), the forward's reference configuration in the tests.
        self.native = self.device.type == "cuda" and self.dtype == torch.float16
        self.hip_attention = self.native  # graph capture needs the native step (kept name: callers probe it)
        # KV cache element type: "fp16" (the reference configuration) or "fp8" (OCP e4m3fn, opt-in: half the
        # bytes the HBM-bound decode attention reads; logits differ at the fp8 quantisation level, the same for
        # encoder and decoder, batch-invariant)
        if kv_dtype not in ("fp16", "fp8"):
            raise ValueError("kv_dtype must be 'fp16' or 'fp8'")
        if kv_dtype == "fp8" and not self.native:
            raise ValueError("an fp8 KV cache needs the native fp16 decode step on the GPU")
        self.kv_dtype = kv_dtype
        self.kv_torch_dtype = torch.uint8 if kv_dtype == "fp8" else self.dtype
        self._static_logits = None
        # native path: the paged KV cache (lm/kvpages.py) -- a pool of 32-position pages kept across calls, and the
        # current call's page table + per-stream lengths
        self.pool = None
        self.kv = None
        self.kv_segment_pages = None  # pages per pool segment (None: from the first call's batch)
        self.first_logits = None  # [1, ld] logits of the shared context (a refilled slot's first coder step)
        # optional per-stream done flags read by the decode attention (int32 tensor view [B], bit 0 = finished, e.g.
        # the coder state's flags word): finished streams skip their cache reads; their logits are never used again
        self.done_flags = None
        # optional per-stream stop positions (int32 [B]): a stream whose cache length reached its stop skips its
        # attention (decode: the position after which its logits are no longer read)
        self.stop_len = None
        # decode-step lanes (native path): 2 = the batch's two row halves on two streams with alternating attention
        # launches (one half's GEMMs overlap the other's attention); 1 = one launch chain
        self.decode_lanes = 1
        self.decode_lanes_min_batch = 1024
        self.decode_lanes_order = "alternate"  # or "free": no ordering between the lanes; "split": attention stream +
        # GEMM stream
        self.decode_lane_cu_split = None  # "split": fraction of each XCD's CUs masked to the attention stream
        self._side = None
        self._split = None
        if self.native:
            from .. import _lib

            self._attn = _lib.lib().ns_decode_attention_ex
            self._kv_format = _lib.NS_KV_FP8 if kv_dtype == "fp8" else _lib.NS_KV_FP16
            if self.shape.n_embd // self.shape.n_head != 64:
                raise ValueError("the HIP decode attention needs head_dim 64 (GPT-2 small/medium/large)")
            for lw in self.layers:
                for name in ("qkv", "o", "fc", "pr"):
                    lw[name + "_wt"] = lw[name + "_w"].t().contiguous()
            self.head_t = self.head.t().contiguous()  # [ld, C]: wte rows, zero rows beyond V
            self._nb = None

    # ------------------------------------------------------------------
    def kv_bytes_per_position(self, B: int) -> int:
        s = self.shape
        return 2 * s.n_layer * B * s.n_embd * torch.tensor([], dtype=self.kv_torch_dtype).element_size()

    def headroom_bytes(self, B: int) -> int:
        """Device memory kept free beside the KV cache for what is allocated after it: the logit
        rows of the step (fixed graph buffer, a coder-side copy, the decoder's), the wide coder path's scratch
        (two 8-byte key arrays per id), the activation buffers of the native step and the guard's scoring chunk,
        plus 2 GiB for the runtime and the allocator's rounding."""
        s = self.shape
        per_stream = self.ld * 4 * 3 + s.vocab * 16 + 16 * s.n_embd * 2
        return (2 << 30) + int(B) * per_stream

    def fit_positions(self, B: int, want: int, reserve: float = 0.05, count_cached: bool = True) -> int:
        """Largest cache length <= ``want`` that fits the device's free memory, minus :meth:`headroom_bytes` and
        a ``reserve`` fraction.  The reference's cache is unbounded; at B = 4096 a 1 KiB payload needs ~1.1k
        positions (170 GB for GPT-2-small fp16), so the budget is sized from what is free, not guessed."""
        if self.position_cap is not None:
            want = min(int(want), int(self.position_cap))
        if self.device.type != "cuda":
            return int(want)
        # the previous cache is dropped first; memory PyTorch's caching allocator holds but no tensor uses (e.g.
        # that cache, or the pre-touched one bench.py hands back) counts as free: reusing those segments keeps
        # the pages warm (releasing them and allocating afresh measured a much slower first pass over the new
        # cache).  When a small tensor carved out of a freed block makes the request not fit the hole (seen as a
        # 120 GiB OOM between two encodes of different batch sizes), _allocate_fitted releases the idle segments
        # and sizes the cache again from what the device then reports free (count_cached=False).
        self.k_cache = self.v_cache = None
        free, _ = torch.cuda.mem_get_info(self.device)
        if count_cached:
            free += torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
        budget = int(free * (1.0 - reserve)) - self.headroom_bytes(B)
        return max(1, min(int(want), budget // self.kv_bytes_per_position(B)))

    def _native_buffers(self, B: int):
        """Activation buffers of the native decode step (fixed addresses: a captured graph replays them)."""
        if self._nb is None or self._nb["B"] != B:
            C, dev, dt = self.shape.n_embd, self.device, self.dtype
            self._nb = {"B": B, "h": torch.empty((B, C), device=dev, dtype=dt),
                        "a": torch.empty((B, C), device=dev, dtype=dt),
                        "qkv": torch.empty((B, 3 * C), device=dev, dtype=dt),
                        "o": torch.empty((B, C), device=dev, dtype=dt),
                        "f": torch.empty((B, 4 * C), device=dev, dtype=dt)}
        return self._nb

    def _cache_shape(self, B: int, rows: int, plain: bool):
        s = self.shape
        hd = s.n_embd // s.n_head
        if plain:
            return (s.n_layer, B, s.n_head, rows, hd)
        # chunk planes: [layer][rows/32][B][H][32][D] -- the rows a decode step reads stay dense in memory
        # whatever the capacity (fewer pages touched than per-pair row ranges padded to the capacity)
        return (s.n_layer, (rows + 31) // 32, B, s.n_head, 32, hd)

    def _cache_strides(self, layer: int):
        """(b, h, chunk) element strides of one layer's stream cache for the attention kernels."""
        kc = self.k_cache[layer]
        if kc.dim() == 5:  # chunk planes [nch, B, H, 32, D]
            return kc.stride(1), kc.stride(2), kc.stride(0)
        return kc.stride(0), kc.stride(1), 0  # plain [B, H, rows, D]

    def _allocate_fitted(self, B: int, base: int, want: int, T0: int = 0) -> None:
        """allocate(B, base + fit_positions(B, want)), falling back to a fresh budget after releasing PyTorch's
        idle segments when the cached ones are too fragmented for the request."""
        try:
            self.allocate(B, base + self.fit_positions(B, want), T0=T0)
        except torch.OutOfMemoryError:
            self.k_cache = self.v_cache = None
            torch.cuda.empty_cache()
            self.allocate(B, base + self.fit_positions(B, want, count_cached=False), T0=T0)

    def allocate(self, B: int, max_len: int, T0: int = 0, dtype=None, plain=None) -> None:
        """Per-stream KV cache for absolute positions [T0, max_len): positions below T0 (the shared context,
        native path only) live once in ``kp``/``vp`` instead of B times.  The native decode step keeps the cache
        in chunk planes (``plain`` False); the PyTorch path (and the prefill) in plain [B, H, rows, D] rows."""
        self.k_cache = self.v_cache = None
        if plain is None:
            plain = not self.native or not self.chunked_cache
        shp = self._cache_shape(B, max_len - T0, plain)
        # uninitialised: attention only ever reads positions < L + 1, all written before they are read
        kdt = self.kv_torch_dtype if dtype is None else dtype
        self.k_cache = torch.empty(shp, device=self.device, dtype=kdt)
        self.v_cache = torch.empty(shp, device=self.device, dtype=kdt)
        self.B, self.L, self.max_len, self.T0 = B, 0, max_len, T0
        if T0 == 0:
            self.kp = self.vp = None

    def grow(self, extra: int) -> None:
        """Enlarge the dense KV cache of the PyTorch path (fp32 / CPU, the forward's reference configuration) by
        ``extra`` positions, copying the filled part.  The copy holds the old and the new cache at once, so the
        WHOLE new cache must fit beside the old one (the native path pages instead: no copy)."""
        from ..exceptions import KVCapacityError

        new_len = self.max_len + int(extra)
        if self.device.type == "cuda":
            free, _ = torch.cuda.mem_get_info(self.device)
            free += torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
            fit = (int(free * 0.9) - self.headroom_bytes(self.B)) // self.kv_bytes_per_position(self.B) + self.T0
            new_len = min(new_len, fit)
            if new_len <= self.L:
                raise KVCapacityError(f"KV cache full at {self.L} positions for B={self.B}: no device memory to grow")
        T0, n = self.T0, self.L - self.T0  # stream rows filled so far
        plain = self.k_cache.dim() == 5
        shp = self._cache_shape(self.B, new_len - T0, plain)
        k = torch.empty(shp, device=self.device, dtype=self.k_cache.dtype)
        v = torch.empty(shp, device=self.device, dtype=self.v_cache.dtype)
        if plain:
            k[:, :, :, :n] = self.k_cache[:, :, :, :n]
            v[:, :, :, :n] = self.v_cache[:, :, :, :n]
        else:
            nch = (n + 31) // 32  # whole chunk planes: the rows beyond n are never read before written
            k[:, :nch] = self.k_cache[:, :nch]
            v[:, :nch] = self.v_cache[:, :nch]
        self.k_cache, self.v_cache, self.max_len = k, v, new_len

    def _ln(self, x, wgt, b):
        return F.layer_norm(x, (self.shape.n_embd,), wgt, b, self.shape.eps)

    def _block(self, i, h, positions_new: int, causal: bool):
        s = self.shape
        lw = self.layers[i]
        B, T, C = h.shape
        H, D = s.n_head, C // s.n_head
        a = self._ln(h, lw["ln1_w"], lw["ln1_b"])
        qkv = torch.addmm(lw["qkv_b"], a.reshape(B * T, C), lw["qkv_w"]).view(B, T, 3, H, D)
        q = qkv[:, :, 0].transpose(1, 2)
        k = qkv[:, :, 1].transpose(1, 2)
        v = qkv[:, :, 2].transpose(1, 2)
        L0 = self.L
        self.k_cache[i, :B, :, L0:L0 + T] = k
        self.v_cache[i, :B, :, L0:L0 + T] = v
        kk = self.k_cache[i, :B, :, : L0 + T]
        vv = self.v_cache[i, :B, :, : L0 + T]
        if causal:
            o = F.scaled_dot_product_attention(q, kk, vv, is_causal=True)
        else:
            o = F.scaled_dot_product_attention(q, kk, vv)
        o = o.transpose(1, 2).reshape(B * T, C)
        h = h + torch.addmm(lw["o_b"], o, lw["o_w"]).view(B, T, C)
        m = self._ln(h, lw["ln2_w"], lw["ln2_b"])
        f = F.gelu(torch.addmm(lw["fc_b"], m.reshape(B * T, C), lw["fc_w"]), approximate="tanh")
        h = h + torch.addmm(lw["pr_b"], f, lw["pr_w"]).view(B, T, C)
        return h

    def _logits(self, h_last):
        hf = self._ln(h_last, self.lnf_w, self.lnf_b)
        out = hf @ self.head
        return out if out.dtype == self.logits_dtype else out.to(self.logits_dtype)

    def _quantize_fp8(self, t: torch.Tensor) -> torch.Tensor:
        from .. import _lib
        from ..coder import _stream_handle

        src = t.contiguous()
        out = torch.empty(src.shape, device=src.device, dtype=torch.uint8)
        if src.numel() % 4:
            raise ValueError("fp8 quantisation needs a multiple of 4 elements")
        rc = _lib.lib().ns_quantize_fp8(src.data_ptr(), out.data_ptr(), src.numel(), _stream_handle())
        if rc != 0:
            raise RuntimeError(f"ns_quantize_fp8 failed ({rc})")
        return out

    @torch.no_grad()
    def prefill(self, context: Sequence[int], B: int, max_new: int) -> torch.Tensor:
        """Run the shared context once (reference: first call, default positions) and broadcast its cache
        to B streams.  Returns the ``[B, ld]`` logits for the next token."""
        ctx = [int(t) for t in list(context)[-1022:]]  # code_base/arithmetic.py:90
        T = len(ctx)
        if T < 1:
            raise ValueError("context must contain at least one token")
        if min(ctx) < 0 or max(ctx) >= self.shape.vocab:  # host check: never gather out of the table
            raise ValueError(f"context token ids must lie in [0, {self.shape.vocab})")
        ids = torch.tensor([ctx], device=self.device, dtype=torch.long)
        if self.native:
            # the context runs once on the native sequence kernels (MFMA GEMMs + causal MFMA attention, no PyTorch
            # attention or BLAS), and its K/V -- the same for every stream -- are kept ONCE (kp/vp), read by every
            # stream's attention (ns_decode_attention_prefix): B-fold less prefix traffic and memory, identical bits
            s = self.shape
            H, D, C = s.n_head, s.n_embd // s.n_head, s.n_embd
            kp = torch.empty((s.n_layer, 1, H, T, D), device=self.device, dtype=self.dtype)
            vp = torch.empty_like(kp)

            def keep_kv(i, qkv):
                kp[i, 0] = qkv[:, C:2 * C].view(T, H, D).transpose(0, 1)
                vp[i, 0] = qkv[:, 2 * C:].view(T, H, D).transpose(0, 1)

            self.kv = None
            hs = self._seq_native(ids, kv_hook=keep_kv)
            lg = self._head_native(hs[T - 1:T])
            if self.kv_dtype == "fp8":  # the context rows get the same conversion as the decode-time appends
                kp, vp = self._quantize_fp8(kp), self._quantize_fp8(vp)
            self.kp, self.vp = kp, vp
            self.first_logits = lg
            self.begin_slots(B, T, max_new)
            return lg.repeat(B, 1)  # always a copy: slot refills write first_logits into these rows
        else:
            pos = torch.arange(T, device=self.device) % self.shape.n_positions
            h = self.wte[ids] + self.wpe[pos][None]
            self._allocate_fitted(B, 0, T + max_new)
            if self.max_len < T + 1:
                raise RuntimeError(f"no device memory for a {T + 1}-position KV cache at B={B}")
            # run the context for one stream, then copy its cache to every stream
            saveB = self.B
            self.B = 1
            for i in range(self.shape.n_layer):
                h = self._block(i, h, T, causal=True)
            self.B = saveB
            for i in range(self.shape.n_layer):
                self.k_cache[i, 1:B, :, :T] = self.k_cache[i, 0:1, :, :T]
                self.v_cache[i, 1:B, :, :T] = self.v_cache[i, 0:1, :, :T]
        self.L = T
        lg = self._logits(h[:, -1])
        return lg.expand(B, -1).contiguous()

    def _seq_native(self, ids: torch.Tensor, kv_hook=None) -> torch.Tensor:
        """Causal forward of B whole sequences ``[B, T]`` (positions 0..T-1, no cache) on the native kernels:
        embedding + ln_1, then per layer the c_attn GEMM, the causal MFMA attention (``ns_seq_attention``), c_proj
        with the residual in its epilogue, ln_2, c_fc with gelu_new, c_proj + residual.  Returns the residual
        stream ``[B*T, C]`` before ln_f.  Every row's result depends on its own sequence only (the GEMMs' and the
        attention's batch invariance), so a text scores the same alone or in a batch.  ``kv_hook(layer, qkv)``
        sees each layer's ``[B*T, 3C]`` c_attn output (the prefill keeps the context's K/V)."""
        from .. import _lib
        from ..coder import _stream_handle

        s = self.shape
        B, T = ids.shape
        C, H = s.n_embd, s.n_head
        D = C // H
        M = B * T
        L = _lib.lib()
        st = _stream_handle()
        dev, dt = self.device, self.dtype
        tok = ids.to(device=dev, dtype=torch.int32).reshape(M).contiguous()
        h = torch.empty((M, C), device=dev, dtype=dt)
        a = torch.empty_like(h)
        o = torch.empty_like(h)
        qkv = torch.empty((M, 3 * C), device=dev, dtype=dt)
        f = torch.empty((M, 4 * C), device=dev, dtype=dt)
        eps = float(s.eps)

        def ok(rc, what):
            if rc != 0:
                raise RuntimeError(f"{what} failed ({rc})")

        def gemm(x, wt, bias, y, epi, N, K):
            ok(L.ns_lm_gemm(x.data_ptr(), x.stride(0), wt.data_ptr(), wt.stride(0),
                            bias.data_ptr() if bias is not None else None, y.data_ptr(), y.stride(0), M, N, K, epi,
                            st), "ns_lm_gemm")

        def ln(x, w, b, y):
            ok(L.ns_lm_layernorm(x.data_ptr(), C, w.data_ptr(), b.data_ptr(), y.data_ptr(), C, M, C, eps, st),
               "ns_lm_layernorm")

        lw0 = self.layers[0]
        ok(L.ns_lm_embed_seq_ln(tok.data_ptr(), self.wte.data_ptr(), self.wpe.data_ptr(), s.vocab, s.n_positions, T,
                                h.data_ptr(), C, lw0["ln1_w"].data_ptr(), lw0["ln1_b"].data_ptr(), a.data_ptr(), C, M,
                                C, eps, st), "ns_lm_embed_seq_ln")
        for i, lw in enumerate(self.layers):
            if i > 0:
                ln(h, lw["ln1_w"], lw["ln1_b"], a)
            gemm(a, lw["qkv_wt"], lw["qkv_b"], qkv, _lib.NS_LM_EPI_STORE, 3 * C, C)
            if kv_hook is not None:
                kv_hook(i, qkv)
            ok(L.ns_seq_attention(qkv.data_ptr(), qkv.stride(0), o.data_ptr(), o.stride(0), B, T, H, D,
                                  1.0 / math.sqrt(D), st), "ns_seq_attention")
            gemm(o, lw["o_wt"], lw["o_b"], h, _lib.NS_LM_EPI_RESIDUAL, C, C)
            ln(h, lw["ln2_w"], lw["ln2_b"], a)
            gemm(a, lw["fc_wt"], lw["fc_b"], f, _lib.NS_LM_EPI_GELU, 4 * C, C)
            gemm(f, lw["pr_wt"], lw["pr_b"], h, _lib.NS_LM_EPI_RESIDUAL, C, 4 * C)
        return h

    def _head_native(self, hrows: torch.Tensor) -> torch.Tensor:
        """ln_f + the head GEMM of ``[R, C]`` residual rows on the native kernels: ``[R, ld]`` logits."""
        from .. import _lib
        from ..coder import _stream_handle

        L = _lib.lib()
        st = _stream_handle()
        C = self.shape.n_embd
        hrows = hrows.contiguous()
        R = hrows.shape[0]
        a = torch.empty_like(hrows)
        rc = L.ns_lm_layernorm(hrows.data_ptr(), C, self.lnf_w.data_ptr(), self.lnf_b.data_ptr(), a.data_ptr(), C, R,
                               C, float(self.shape.eps), st)
        if rc != 0:
            raise RuntimeError(f"ns_lm_layernorm failed ({rc})")
        out = torch.empty((R, self.ld), device=self.device, dtype=self.logits_dtype)
        epi = _lib.NS_LM_EPI_STORE_F32 if out.dtype == torch.float32 else _lib.NS_LM_EPI_STORE
        rc = L.ns_lm_gemm(a.data_ptr(), C, self.head_t.data_ptr(), self.head_t.stride(0), None, out.data_ptr(),
                          out.stride(0), R, self.ld, C, epi, st)
        if rc != 0:
            raise RuntimeError(f"ns_lm_gemm failed ({rc})")
        return out

    @torch.no_grad()
    def window_logits(self, ids: torch.Tensor) -> torch.Tensor:
        """Next-token logits ``[B, ld]`` of B token windows ``[B, W]`` each run from scratch with positions
        0..W-1 -- the src provider's ``_ModelAdapter`` forward over a context trimmed to ``max_context``
        (``src/neuralstego/lm/arithmetic.py:45-74``)."""
        B, W = ids.shape
        if W > self.shape.n_positions:
            raise ValueError(f"window longer than n_positions ({self.shape.n_positions})")
        if self.native:
            hs = self._seq_native(ids)
            return self._head_native(hs.view(B, W, -1)[:, -1])
        return self.forward_sequences(ids)[:, -1].contiguous()

    @torch.no_grad()
    def forward_sequences(self, ids: torch.Tensor) -> torch.Tensor:
        """Causal forward of B right-padded sequences ``[B, T]`` with positions ``0..T-1`` and no cache (the
        guard's scoring pass, ``metrics/lm_scorer.py:121-131``); returns ``[B, T, ld]`` logits in
        ``logits_dtype``.  Padding only follows the real tokens, so causality keeps it out of their rows.  fp16 on
        the GPU runs the native sequence kernels (a text's scores do not depend on the batch it is scored in)."""
        s = self.shape
        B, T = ids.shape
        if T > s.n_positions:
            raise ValueError(f"sequence longer than n_positions ({s.n_positions})")
        if self.native:
            return self._head_native(self._seq_native(ids)).view(B, T, self.ld)
        H, C = s.n_head, s.n_embd
        D = C // H
        pos = torch.arange(T, device=self.device)
        h = self.wte[ids.to(self.device).long()] + self.wpe[pos][None]
        for lw in self.layers:
            a = self._ln(h, lw["ln1_w"], lw["ln1_b"])
            qkv = torch.addmm(lw["qkv_b"], a.reshape(B * T, C), lw["qkv_w"]).view(B, T, 3, H, D)
            q, k, v = (qkv[:, :, j].transpose(1, 2) for j in range(3))
            o = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B * T, C)
            h = h + torch.addmm(lw["o_b"], o, lw["o_w"]).view(B, T, C)
            m = self._ln(h, lw["ln2_w"], lw["ln2_b"])
            f = F.gelu(torch.addmm(lw["fc_b"], m.reshape(B * T, C), lw["fc_w"]), approximate="tanh")
            h = h + torch.addmm(lw["pr_b"], f, lw["pr_w"]).view(B, T, C)
        out = self._ln(h, self.lnf_w, self.lnf_b).reshape(B * T, C) @ self.head
        out = out if out.dtype == self.logits_dtype else out.to(self.logits_dtype)
        return out.view(B, T, self.ld)

    # ------------------------------------------------------------------ paged KV (native path)
    def _pool_budget(self) -> int:
        """Device bytes the page pool may still take: free memory (with what PyTorch's allocator holds unused) less
        a 5 % reserve and :meth:`headroom_bytes` for what is allocated beside the cache."""
        free, total = torch.cuda.mem_get_info(self.device)
        free += torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
        return int(free - 0.05 * total) - self.headroom_bytes(max(self.B, 1))

    def page_pool(self, B: int = 0):
        """The page pool (created on first use; ``kv_segment_pages`` pages per segment, default from the first
        call's batch: 2B rounded up to a power of two within [64, 1024])."""
        from .kvpages import KVPagePool

        if self.pool is None:
            s = self.shape
            seg = self.kv_segment_pages
            if seg is None:
                seg = min(1024, max(64, 1 << max(0, 2 * int(B or self.B or 1) - 1).bit_length()))
            me = weakref.ref(self)  # no reference cycle: a dropped model frees its pool at once (no gc pass needed)

            def budget():
                lm = me()
                return lm._pool_budget() if lm is not None else 0

            self.pool = KVPagePool(s.n_layer, s.n_head, s.n_embd // s.n_head, self.kv_torch_dtype, self.device,
                                   budget_bytes=budget, seg_pages=seg)
        return self.pool

    def begin_slots(self, B: int, T0: int, max_new: int = 32) -> None:
        """A new call over ``B`` stream slots, every one at the shared context (cache length ``T0``): a fresh page
        table (every page of the pool free again), no page assigned yet."""
        from .kvpages import PAGE_ROWS, PagedKV

        pool = self.page_pool(B)
        self.kv = None
        pool.reset()
        self.kv = PagedKV(pool, B, T0, (max(1, int(max_new)) + PAGE_ROWS - 1) // PAGE_ROWS + 1)
        self.B, self.L, self.T0 = int(B), int(T0), int(T0)
        self._nb = None

    def warm_pool(self, pages: int = None, B: int = 1) -> int:
        """Grow the page pool to ``pages`` pages (default: as many as the device budget allows at batch ``B``) and
        write every new page once, so a timed call finds its pages mapped and warm (a first pass over freshly
        allocated device memory measured up to 12 % slower per step).  Returns the pool's size in pages."""
        pool = self.page_pool(B)
        saveB, self.B = self.B, max(self.B, int(B))
        try:
            want = pool.total + pool.growable_pages() if pages is None else int(pages)
            while pool.total < want and pool.growable_pages() >= pool.seg_pages:  # a segment at a time, in budget
                if not pool.add_segment(pool.seg_pages):
                    break
            for seg in pool.segments:
                seg.zero_()
        finally:
            self.B = saveB
        return pool.total

    def release_cache(self) -> None:
        """Drop the paged cache, its pool and the shared context's K/V (device memory back to PyTorch)."""
        self.kv = None
        if self.pool is not None:
            self.pool.release_memory()
        self.pool = None
        self.kp = self.vp = None
        self.k_cache = self.v_cache = None
        self._nb = None

    def _decode_native(self, tokens: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """One decode step of every slot on the batch-invariant HIP kernels: embed + ln_1 at each stream's own
        position (``lens[b] % n_positions``), then per layer c_attn GEMM, the paged KV-append attention
        (``ns_decode_attention_paged``: each stream over its own pages and length), c_proj GEMM with the residual add
        in its epilogue, ln_2, c_fc GEMM with gelu_new in its epilogue, c_proj GEMM + residual; ln_f (advancing every
        ``lens[b]`` by one) and the head GEMM straight into ``out`` ([B, ld] logits).  Every per-step quantity lives
        on the device, so the same launches are captured once as a hipGraph and replayed."""
        from .. import _lib
        from ..coder import _stream_handle

        kv = self.kv
        B = kv.B
        L = _lib.lib()
        st = _stream_handle()
        tok = tokens if tokens.dtype == torch.int32 else tokens.to(torch.int32)
        if not tok.is_contiguous() or tok.shape != (B,):
            tok = tok.reshape(B).contiguous()
        df = self.done_flags
        if df is not None and (df.dtype != torch.int32 or df.shape != (B,) or not _same_device(df.device, self.device)):
            raise ValueError(f"done_flags must be an int32 [{B}] view on {self.device}")
        done_ptr, done_stride = (df.data_ptr(), df.stride(0)) if df is not None else (None, 0)
        sl = self.stop_len
        if sl is not None and (sl.dtype != torch.int32 or sl.shape != (B,) or not sl.is_contiguous()
                               or not _same_device(sl.device, self.device)):
            raise ValueError(f"stop_len must be a contiguous int32 [{B}] tensor on {self.device}")
        stop_ptr = sl.data_ptr() if sl is not None else None
        if out.shape != (B, self.ld) or out.stride(1) != 1:
            raise ValueError(f"logits buffer must be [{B}, {self.ld}]")
        lanes = self._lanes(B)
        if len(lanes) == 1:
            self._decode_rows(L, st, tok, out, 0, B, done_ptr, done_stride, stop_ptr)
            return out
        main = torch.cuda.current_stream(self.device)
        if self.decode_lanes_order == "split":
            return self._decode_split(L, main, tok, out, lanes, done_ptr, done_stride, stop_ptr)
        # two lanes (row halves) on two streams, their attention launches alternating (lane 0 layer i, lane 1 layer
        # i, lane 0 layer i + 1, ...): one lane's GEMMs / layer norms run beside the other lane's HBM-bound attention
        # instead of after it.  Rows are independent (batch invariance), so the bits are those of one launch chain.
        side = self._side_stream()
        fork = torch.cuda.Event()
        fork.record(main)
        side.wait_event(fork)
        (r0, n0), (r1, n1) = lanes
        steps = [self._decode_rows(L, st, tok, out, r0, n0, done_ptr, done_stride, stop_ptr, gen=True),
                 self._decode_rows(L, side.cuda_stream, tok, out, r1, n1, done_ptr, done_stride, stop_ptr, gen=True)]
        streams = (main, side)
        alternate = self.decode_lanes_order == "alternate"
        prev = None  # (lane, event after its latest attention launch)
        for _ in range(self.shape.n_layer):
            for k in (0, 1):
                next(steps[k])  # up to the attention launch
                if alternate and prev is not None:
                    streams[k].wait_event(prev[1])
                next(steps[k])  # the attention launch
                if alternate:
                    ev = torch.cuda.Event()
                    ev.record(streams[k])
                    prev = (k, ev)
        for k in (0, 1):
            for _ in steps[k]:  # ln_f and the head
                pass
        join = torch.cuda.Event()
        join.record(side)
        main.wait_event(join)
        return out

    def _decode_split(self, L, main, tok, out, lanes, done_ptr, done_stride, stop_ptr):
        """Two lanes, the attention launches on one stream (lane 0 layer i, lane 1 layer i, lane 0 layer i + 1, ...)
        and every other launch on a second one: lane k's GEMMs of layer i run while lane 1-k's attention of layer i
        streams.  With ``decode_lane_cu_split`` the two streams are CU-masked (that fraction of every XCD's CUs for the
        attention stream, the rest for the other), so the GEMMs get CUs while the attention holds the rest."""
        if torch.cuda.is_current_stream_capturing():  # measured: the runtime crashes ending such a capture, and a
            raise RuntimeError("split decode lanes run eagerly only (graphs=False)")  # graph drops the CU masks
        sa, sg = self._split_streams()
        fork = torch.cuda.Event()
        fork.record(main)
        sg.wait_event(fork)
        sa.wait_event(fork)
        gens = [self._decode_rows_gen(L, sg.cuda_stream, tok, out, r, n, done_ptr, done_stride, stop_ptr,
                                      st_attn=sa.cuda_stream) for r, n in lanes]
        att = [None, None]  # event after each lane's latest attention launch
        for _ in range(self.shape.n_layer):
            for k in (0, 1):
                if att[k] is not None:
                    sg.wait_event(att[k])
                next(gens[k])  # lane k: the launches before its attention (on sg)
                ev = torch.cuda.Event()
                ev.record(sg)
                sa.wait_event(ev)
                next(gens[k])  # its attention (on sa)
                att[k] = torch.cuda.Event()
                att[k].record(sa)
        for k in (0, 1):
            sg.wait_event(att[k])
            for _ in gens[k]:  # the last layer's GEMMs, ln_f and the head
                pass
        for stream in (sg, sa):  # both streams rejoin the caller's directly (a graph capture ends on it)
            join = torch.cuda.Event()
            join.record(stream)
            main.wait_event(join)
        return out

    def _split_streams(self):
        if self._split is None:
            frac = self.decode_lane_cu_split
            if frac is None:
                self._split = (torch.cuda.Stream(self.device), torch.cuda.Stream(self.device))
            else:
                self._split = (_cu_masked_stream(self.device, frac, True), _cu_masked_stream(self.device, frac, False))
        return self._split

    def _lanes(self, B: int):
        """Row ranges of the decode step's lanes: one, or two halves (``decode_lanes`` = 2) when B is large enough
        for both halves to fill the chip."""
        if self.decode_lanes <= 1 or B < max(2, self.decode_lanes_min_batch):
            return [(0, B)]
        h = (B // 2 + 15) // 16 * 16  # 16-row aligned split (whole MFMA row blocks in lane 0)
        if not 0 < h < B:
            h = B // 2
        return [(0, h), (h, B - h)]

    def _side_stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
        return self._side

    def _decode_rows(self, L, st, tok, out, r0, n, done_ptr, done_stride, stop_ptr, gen=False):
        """The decode step's launches for rows [r0, r0 + n) on stream ``st``.  ``gen``: a generator that yields
        before and after each layer's attention launch (the caller orders the lanes' attention launches)."""
        it = self._decode_rows_gen(L, st, tok, out, r0, n, done_ptr, done_stride, stop_ptr)
        if gen:
            return it
        for _ in it:
            pass

    def _decode_rows_gen(self, L, st, tok, out, r0, B, done_ptr, done_stride, stop_ptr, st_attn=None):
        from .. import _lib

        st_attn = st if st_attn is None else st_attn
        s = self.shape
        kv = self.kv
        C = s.n_embd
        H, D = s.n_head, C // s.n_head
        nb = self._native_buffers(kv.B)
        if not (B > 0 and r0 >= 0 and r0 + B <= kv.B):  # host check before any launch: rows inside every buffer
            raise ValueError(f"decode rows [{r0}, {r0 + B}) outside the batch of {kv.B}")

        def row(t, r=r0):  # address of row r of a [*, ...] tensor
            return t.data_ptr() + r * t.stride(0) * t.element_size()

        h, a, qkv, o, f = (row(nb[k]) for k in ("h", "a", "qkv", "o", "f"))
        ldq, ldf = nb["qkv"].stride(0), nb["f"].stride(0)
        T0 = kv.T0
        eps = float(s.eps)

        def ok(rc, what):
            if rc != 0:
                raise RuntimeError(f"{what} failed ({rc})")

        def gemm(x, ldx, wt, bias, y, ldy, epi, N, K):
            ok(L.ns_lm_gemm(x, ldx, wt.data_ptr(), wt.stride(0), bias.data_ptr() if bias is not None else None, y,
                            ldy, B, N, K, epi, st), "ns_lm_gemm")

        lens = row(kv.lens)
        lw0 = self.layers[0]
        ok(L.ns_lm_embed_ln_rows(row(tok), self.wte.data_ptr(), self.wpe.data_ptr(), s.vocab, s.n_positions,
                                 lens, h, C, lw0["ln1_w"].data_ptr(), lw0["ln1_b"].data_ptr(), a, C, B, C, eps, st),
           "ns_lm_embed_ln_rows")

        def ln_gemm(ln_w, ln_b, wt, bias, y, ldy, epi, N):  # ln(h) -> GEMM, one launch at small B (same bits)
            ok(L.ns_lm_ln_gemm(h, C, ln_w.data_ptr(), ln_b.data_ptr(), eps, wt.data_ptr(), wt.stride(0),
                               bias.data_ptr(), y, ldy, B, N, C, epi, a, C, st), "ns_lm_ln_gemm")

        table = row(kv.table)
        done = done_ptr + r0 * done_stride * 4 if done_ptr else None
        stop = stop_ptr + r0 * 4 if stop_ptr else None
        for i, lw in enumerate(self.layers):
            if i > 0:
                ln_gemm(lw["ln1_w"], lw["ln1_b"], lw["qkv_wt"], lw["qkv_b"], qkv, ldq, _lib.NS_LM_EPI_STORE, 3 * C)
            else:  # ln_1 of layer 0 comes with the embedding
                gemm(a, C, lw["qkv_wt"], lw["qkv_b"], qkv, ldq, _lib.NS_LM_EPI_STORE, 3 * C, C)
            kp = self.kp[i, 0] if T0 else None  # [H, T0, D]
            vp = self.vp[i, 0] if T0 else None
            yield  # before the attention launch
            rc = L.ns_decode_attention_paged(qkv, ldq, table, kv.table.stride(0), kv.width, kv.pool.layer_offset(i),
                                             kp.data_ptr() if T0 else None, vp.data_ptr() if T0 else None,
                                             kp.stride(0) if T0 else 0, T0, B, H, D, lens, self.window,
                                             self._kv_format, done, done_stride, stop, o, C, 1.0 / math.sqrt(D),
                                             st_attn)
            ok(rc, "ns_decode_attention_paged")
            yield  # after it
            gemm(o, C, lw["o_wt"], lw["o_b"], h, C, _lib.NS_LM_EPI_RESIDUAL, C, C)
            ln_gemm(lw["ln2_w"], lw["ln2_b"], lw["fc_wt"], lw["fc_b"], f, ldf, _lib.NS_LM_EPI_GELU, 4 * C)
            gemm(f, ldf, lw["pr_wt"], lw["pr_b"], h, C, _lib.NS_LM_EPI_RESIDUAL, C, 4 * C)
        # ln_f also advances every stream's cache length (no launch of its own)
        ok(L.ns_lm_layernorm_rows(h, C, self.lnf_w.data_ptr(), self.lnf_b.data_ptr(), a, C, B, C, eps, lens, st),
           "ns_lm_layernorm_rows")
        epi = _lib.NS_LM_EPI_STORE_F32 if out.dtype == torch.float32 else _lib.NS_LM_EPI_STORE
        gemm(a, C, self.head_t, None, row(out), out.stride(0), epi, self.ld, C)

    # ------------------------------------------------------------------ graph-capturable decode step
    def begin_static(self, logits_out: torch.Tensor) -> None:
        """Prepare :meth:`step_static`: the logits go to the fixed buffer ``logits_out`` ([B, ld]) -- positions
        and cache lengths already live on the device -- so the same captured hipGraph replays every decode step.
        Needs the native HIP step (fp16 on the GPU)."""
        if not self.native:
            raise RuntimeError("graph-captured decode steps need the native HIP step (fp16 on the GPU)")
        if logits_out.shape != (self.kv.B, self.ld) or logits_out.dtype != self.logits_dtype:
            raise ValueError(f"static logits must be [{self.kv.B}, {self.ld}] {self.logits_dtype}")
        self._static_logits = logits_out

    def static_capacity_left(self) -> int:
        """Decode steps every slot can take within the pages it holds (graph replays cannot map pages)."""
        return self.kv.steps_reserved(np.arange(self.kv.B))

    def reserve(self, steps: int) -> bool:
        """Lockstep callers: map the pages every slot needs for the next ``steps`` decode steps (False: the device
        has no memory for them)."""
        return self.kv.ensure(np.arange(self.kv.B), self.L + int(steps)).size == 0

    def advance(self, n: int = 1) -> None:
        """The host side of ``n`` executed decode steps (the device advanced ``lens`` itself)."""
        self.L += int(n)
        self.kv.advance(n)

    @torch.no_grad()
    def step_static(self, tokens: torch.Tensor) -> torch.Tensor:
        """:meth:`step` into the fixed logits buffer, without host-side page mapping or length bookkeeping: issues no
        host synchronisation and no allocation, so it can be captured once.  The caller maps pages ahead
        (:meth:`reserve`, or the slot scheduler) and calls :meth:`advance` per executed step."""
        self._decode_native(tokens, self._static_logits)
        return self._static_logits

    @torch.no_grad()
    def step(self, tokens: torch.Tensor, live=None) -> torch.Tensor:
        """Feed one token per stream (``[B]`` int); position = cache length mod n_positions.  ``live`` (host bool
        ``[B]``, native path): only these streams get pages and attention this step -- a lockstep caller whose
        streams end at different lengths (the span splitter's decodes) stops paying, in memory and reads, for the
        finished ones; their logits rows are not meaningful afterwards."""
        B = self.B
        if tokens.shape != (B,):
            raise ValueError(f"expected {B} tokens")
        if self.native:
            from ..exceptions import KVCapacityError

            if live is None:
                ok = self.reserve(1)
            else:
                live = np.asarray(live, dtype=bool).reshape(B)
                ok = self.kv.ensure(np.nonzero(live)[0], self.L + 1).size == 0
            if not ok:
                raise KVCapacityError(f"KV cache full at {self.L} positions for B={B}: no device memory for a page")
            out = torch.empty((B, self.ld), device=self.device, dtype=self.logits_dtype)
            saved = self.stop_len
            if live is not None and not live.all():  # the attention skips a stream whose length reached its stop
                stop = np.where(live, np.iinfo(np.int32).max, 0).astype(np.int32)
                self.stop_len = torch.from_numpy(stop).to(self.device)
            try:
                self._decode_native(tokens, out)
            finally:
                self.stop_len = saved
            self.advance(1)
            return out
        if self.L >= self.max_len:
            self.grow(max(64, self.max_len))
        pos = self.L % self.shape.n_positions
        h = (self.wte[tokens.long()] + self.wpe[pos])[:, None, :]
        for i in range(self.shape.n_layer):
            h = self._block(i, h, 1, causal=False)
        self.L += 1
        return self._logits(h[:, -1])


def _cu_masked_stream(device, frac: float, first: bool):
    """A HIP stream whose kernels may run on a subset of the CUs (``hipExtStreamCreateWithCUMask``): the first
    ``frac`` of every 8 consecutive CU ids (``first``) or the rest -- an even share of each XCD whatever way the ids
    interleave the XCDs.  Eager launches only (a captured graph does not keep a stream's mask)."""
    import ctypes

    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    k = max(1, min(7, int(round(8 * float(frac)))))
    bits = [((i % 8) < k) == first for i in range(ncu)]
    words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
    for i, on in enumerate(bits):
        if on:
            words[i // 32] |= 1 << (i % 32)
    hip = ctypes.CDLL("libamdhip64.so")
    handle = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(handle), ctypes.c_uint32(len(words)), words)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    return torch.cuda.ExternalStream(handle.value, device=device)


def _normalise_device(dev: torch.device) -> torch.device:
    """``cuda`` without an index is the current device (a tensor's device always carries its index: comparing
    ``torch.device('cuda')`` with ``cuda:0`` is False)."""
    if dev.type == "cuda" and dev.index is None:
        return torch.device("cuda", torch.cuda.current_device())
    return dev


def _same_device(a: torch.device, b: torch.device) -> bool:
    return a.type == b.type and (a.index or 0) == (b.index or 0)


def random_gpt2(name: str = "gpt2", *, seed: int = 1234, **overrides):
    """Random-init GPT-2 of a named size (no network: the architecture only).  SURVEY.md §8(c)."""
    from transformers import GPT2Config, GPT2LMHeadModel

    sizes = {"gpt2": dict(n_layer=12, n_head=12, n_embd=768),
             "gpt2-medium": dict(n_layer=24, n_head=16, n_embd=1024),
             # HooshvareLab/gpt2-fa (config C4): GPT-2-small geometry with its 42,001-id Persian vocabulary
             # (unverified offline -- architecture only, random weights)
             "gpt2-fa": dict(n_layer=12, n_head=12, n_embd=768, vocab_size=42001, bos_token_id=42000,
                             eos_token_id=42000),
             "tiny": dict(n_layer=2, n_head=2, n_embd=64)}
    kw = dict(sizes[name])
    kw.update(overrides)
    torch.manual_seed(seed)
    cfg = GPT2Config(**kw)
    model = GPT2LMHeadModel(cfg)
    model.eval()
    return model
