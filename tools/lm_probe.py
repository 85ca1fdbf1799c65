"""Decode-step probe of the batch-invariant GPT-2 kernels (include/nsg_lm.h) vs the PyTorch / hipBLASLt ops.

For one batch size B and cache length L: each GEMM of a decode step (c_attn, attn c_proj, c_fc, mlp c_proj,
lm head) timed on ns_lm_gemm and on torch.addmm/matmul (TFLOP/s), the attention at L (GB/s of K/V read), a
layer norm, and whole decode steps (native vs PyTorch path).  HIP events on the launch stream; prints JSON
lines.  usage: python tools/lm_probe.py [--batch 4096] [--lens 64,512] [--model gpt2] [--reps 20]
"""

from __future__ import annotations

import argparse
import json
import math
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--lens", default="64,512")
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-step", action="store_true")
    ap.add_argument("--configs", action="store_true", help="time every ns_lm_gemm_config tile configuration")
    ap.add_argument("--kv", default="fp16", choices=["fp16", "fp8"], help="KV cache element type")
    ap.add_argument("--attn-only", action="store_true")
    args = ap.parse_args()
    import torch

    from neuralsteganography_amd import _lib
    from neuralsteganography_amd.coder import _stream_handle
    from neuralsteganography_amd.lm.gpt2 import BatchedGPT2, random_gpt2

    dev = torch.device("cuda", 0)
    B = args.batch
    L = _lib.lib()

    def timed(fn, reps=args.reps):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    lm = BatchedGPT2(random_gpt2(args.model), device=dev, logits_dtype=torch.float16, kv_dtype=args.kv)
    s = lm.shape
    C = s.n_embd
    lw = lm.layers[0]
    x = torch.randn((B, 4 * C), device=dev).half()
    shapes = [("c_attn", lw["qkv_wt"], lw["qkv_b"], lw["qkv_w"], C, 0), ("attn_proj", lw["o_wt"], lw["o_b"], lw["o_w"], C, 2),
              ("c_fc", lw["fc_wt"], lw["fc_b"], lw["fc_w"], C, 1), ("mlp_proj", lw["pr_wt"], lw["pr_b"], lw["pr_w"], 4 * C, 2),
              ("lm_head", lm.head_t, None, lm.head, C, 0)]
    # the same shapes with a plain store (the epilogue's own cost) and the fp32-logits head the bench's coder reads
    shapes += [("c_fc_store", lw["fc_wt"], lw["fc_b"], lw["fc_w"], C, 0), ("lm_head_f32", lm.head_t, None, lm.head, C, 3)]
    for name, wt, bias, w, K, epi in ([] if args.attn_only else shapes):
        N = wt.shape[0]
        xa = x[:, :K].contiguous()
        y = torch.empty((B, N), device=dev, dtype=torch.float32 if epi == 3 else torch.float16)
        st = _stream_handle()
        bp = bias.data_ptr() if bias is not None else None

        def native():
            rc = L.ns_lm_gemm(xa.data_ptr(), K, wt.data_ptr(), K, bp, y.data_ptr(), N, B, N, K, epi, st)
            assert rc == 0

        def ref():
            if bias is not None:
                return torch.addmm(bias, xa, w)
            return xa @ w

        ms_n, ms_t = timed(native), timed(ref)
        fl = 2.0 * B * N * K
        rec = {"gemm": name, "M": B, "N": N, "K": K, "ms_native": ms_n, "ms_torch": ms_t,
               "tflops_native": fl / ms_n / 1e9, "tflops_torch": fl / ms_t / 1e9}
        if args.configs:
            per = {}
            for cfg in range(L.ns_lm_gemm_configs()):
                if cfg < 3 and B > 256:
                    continue  # direct (small-batch) kernels re-read the weights per 64 rows

                def one(cfg=cfg):
                    rc = L.ns_lm_gemm_config(xa.data_ptr(), K, wt.data_ptr(), K, bp, y.data_ptr(), N, B, N, K, epi,
                                             cfg, st)
                    assert rc == 0

                per[cfg] = round(fl / timed(one) / 1e9, 1)
            rec["tflops_by_config"] = per
        print(json.dumps(rec), flush=True)
    a = torch.randn((B, C), device=dev).half()
    ln_out = torch.empty_like(a)

    def ln():
        L.ns_lm_layernorm(a.data_ptr(), C, lw["ln1_w"].data_ptr(), lw["ln1_b"].data_ptr(), ln_out.data_ptr(), C, B, C,
                          1e-5, _stream_handle())

    ms_ln = timed(ln)
    ms_ln_t = timed(lambda: torch.nn.functional.layer_norm(a, (C,), lw["ln1_w"], lw["ln1_b"], 1e-5))
    print(json.dumps({"layernorm": C, "M": B, "ms_native": ms_ln, "ms_torch": ms_ln_t,
                      "GBs_native": 2 * B * C * 2 / ms_ln / 1e6}), flush=True)

    H, D = s.n_head, C // s.n_head
    lens = [int(v) for v in args.lens.split(",")]
    lm.allocate(B, max(lens) + 2)
    if args.kv == "fp8":
        lm.k_cache[0].random_(0, 120)  # finite e4m3fn bytes (NaN is 0x7f / 0xff)
        lm.v_cache[0].random_(0, 120)
    else:
        lm.k_cache[0].normal_()
        lm.v_cache[0].normal_()
    qkv = torch.randn((B, 3 * C), device=dev).half()
    o = torch.empty((B, C), device=dev).half()
    for Lc in lens:
        kc, vc = lm.k_cache[0], lm.v_cache[0]

        fn = L.ns_decode_attention_fp8 if args.kv == "fp8" else L.ns_decode_attention_prefix

        sb, sh, sz = lm._cache_strides(0)  # the chunk-plane layout the decode step uses

        def attn():
            rc = fn(qkv.data_ptr(), qkv.stride(0), kc.data_ptr(), vc.data_ptr(), sb, sh, sz, None, None,
                    0, 0, B, H, D, Lc, None, Lc + 2, 0, o.data_ptr(), o.stride(0), D ** -0.5, _stream_handle())
            assert rc == 0

        ms = timed(attn)
        kv = B * H * (Lc + 1) * D * 2 * (1 if args.kv == "fp8" else 2)
        rec = {"attention_L": Lc, "B": B, "ms": ms, "GBs": kv / ms / 1e6}
        if not args.no_step:
            tok = torch.randint(0, s.vocab, (B,), device=dev)

            def step_native():
                lm.L = Lc
                lm.step(tok)

            lm.native = True
            rec["ms_step_native"] = timed(step_native, max(3, args.reps // 4))
            lm.native = False
            rec["ms_step_torch"] = timed(step_native, max(3, args.reps // 4))
            lm.native = True
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
