"""Decode attention at the C3 geometry: the lockstep chunk-plane kernel vs the paged kernel over pool layouts.

    python tools/paged_attn_probe.py [--L 544] [--kv fp16|fp8] [--window 0]

(a) dense chunk planes [nch][B][H][32][D] of one layer (ns_decode_attention_ex, round 5's product path);
(b) pages holding every layer back to back, [page][layer][K|V][H][32][D] (one layer's block every 1.18 MB);
(c) layer-major segments, [layer][page][K|V][H][32][D] (one layer's pages contiguous), pages in allocation order;
(d) (c) with the pages of a stream scattered at random over the segment.
Pages are allocated chunk by chunk over the streams, as the slot scheduler maps them.  Prints one JSON line per
layout with the kernel's average time (HIP events over K launches) and the algorithmic HBM rate.
"""

import argparse
import json
import math
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from neuralsteganography_amd import _lib  # noqa: E402
from neuralsteganography_amd.coder import _stream_handle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--L", type=int, default=544)
    ap.add_argument("--T0", type=int, default=32)
    ap.add_argument("--kv", default="fp16", choices=["fp16", "fp8"])
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--only", default="abcd")
    a = ap.parse_args()
    B, H, D, T0, L, NL = a.B, 12, 64, a.T0, a.L, a.layers
    C = H * D
    rows = L + 1 - T0
    nch = (rows + 31) // 32
    edt = torch.uint8 if a.kv == "fp8" else torch.float16
    fmt = _lib.NS_KV_FP8 if a.kv == "fp8" else _lib.NS_KV_FP16
    esz = 1 if a.kv == "fp8" else 2
    g = torch.Generator(device="cuda").manual_seed(7)
    qkv = torch.randn((B, 3 * C), generator=g, device="cuda", dtype=torch.float16)
    kp = torch.zeros((H, T0, D), device="cuda", dtype=edt)
    vp = torch.zeros((H, T0, D), device="cuda", dtype=edt)
    out = torch.empty((B, C), device="cuda", dtype=torch.float16)
    lens = torch.full((B,), L, dtype=torch.int32, device="cuda")
    lib = _lib.lib()
    st = _stream_handle()
    s0 = max(0, L + 1 - a.window) if a.window else 0
    keys = L + 1 - s0
    own = keys - max(0, T0 - s0)
    alg = B * H * own * 2 * D * esz + H * max(0, T0 - s0) * 2 * D * esz + B * 3 * C * 2 + B * C * 2

    def timeit(launch):
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            launch()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.steps

    def report(name, ms):
        print(json.dumps({"layout": name, "B": B, "L": L, "kv": a.kv, "window": a.window, "kernel_ms": ms,
                          "alg_bytes": alg, "GBps": alg / (ms / 1e3) / 1e9}), flush=True)

    if "a" in a.only:
        kc = torch.zeros((nch, B, H, 32, D), device="cuda", dtype=edt)
        vc = torch.zeros_like(kc)

        def dense():
            rc = lib.ns_decode_attention_ex(qkv.data_ptr(), qkv.stride(0), kc.data_ptr(), vc.data_ptr(), kc.stride(1),
                                            kc.stride(2), kc.stride(0), kp.data_ptr(), vp.data_ptr(), kp.stride(0), T0,
                                            B, H, D, L, None, T0 + nch * 32, a.window, fmt, None, 0, None,
                                            out.data_ptr(), out.stride(0), 1.0 / math.sqrt(D), st)
            assert rc == 0, rc
        report("dense chunk planes", timeit(dense))
        del kc, vc
        torch.cuda.empty_cache()
    npages = B * nch
    blk = 2 * H * 32 * D  # one layer's block of a page, elements
    order = np.arange(npages).reshape(nch, B).T  # page of (stream b, chunk c) = c * B + b

    def paged(pool_base, page_bytes, layer_off, perm=None):
        pg = order if perm is None else perm[order]
        table = torch.from_numpy(np.ascontiguousarray(pool_base + page_bytes * pg.astype(np.int64))).cuda()

        def run():
            rc = lib.ns_decode_attention_paged(qkv.data_ptr(), qkv.stride(0), table.data_ptr(), table.stride(0),
                                               table.shape[1], layer_off, kp.data_ptr(), vp.data_ptr(), kp.stride(0),
                                               T0, B, H, D, lens.data_ptr(), a.window, fmt, None, 0, None,
                                               out.data_ptr(), out.stride(0), 1.0 / math.sqrt(D), st)
            assert rc == 0, rc
        return run

    layer = NL // 2
    if "b" in a.only:
        pool = torch.zeros((npages, NL * blk), device="cuda", dtype=edt)
        report("pages [page][layer]", timeit(paged(pool.data_ptr(), NL * blk * esz, layer * blk)))
        del pool
        torch.cuda.empty_cache()
    if "c" in a.only or "d" in a.only:
        pool = torch.zeros((NL, npages, blk), device="cuda", dtype=edt)
        if "c" in a.only:
            report("segments [layer][page]", timeit(paged(pool.data_ptr(), blk * esz, layer * npages * blk)))
        if "d" in a.only:
            perm = np.random.default_rng(1).permutation(npages)
            report("segments [layer][page], pages shuffled",
                   timeit(paged(pool.data_ptr(), blk * esz, layer * npages * blk, perm)))
        del pool
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
