"""End-to-end probe: GPT-2 forward (random-init weights) + HIP coder step at batch B, per cache length.

For each cache length L it fills the KV cache with random values, sets the cache length to L and times
(a) one BatchedGPT2.step (the whole forward: GEMMs + attention over L positions + head into the coder's
[B, ld] layout), (b) the attention part alone, (c) one coder step on those logits.  Prints one JSON line per
L.  usage: python tools/e2e_probe.py [--batch 4096] [--lens 64,512,1024] [--model gpt2]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--lens", default="64,512,1024")
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--logits", default="f32")
    args = ap.parse_args()
    import torch
    import torch.nn.functional as F

    from neuralsteganography_amd import synthetic
    from neuralsteganography_amd.coder import CoderContext, CoderParams, EncodeSession
    from neuralsteganography_amd.lm.gpt2 import BatchedGPT2, random_gpt2

    dev = torch.device("cuda", 0)
    B = args.batch
    lens = [int(x) for x in args.lens.split(",")]
    ldt = torch.float16 if args.logits == "f16" else torch.float32
    lm = BatchedGPT2(random_gpt2(args.model), device=dev, logits_dtype=ldt)
    s = lm.shape
    lm.allocate(B, max(lens) + 1)
    lm.k_cache.normal_()
    lm.v_cache.normal_()
    params = CoderParams(vocab=s.vocab, precision=26, temp=0.9, topk=300, dtype=args.logits)
    ctx = CoderContext(params, max_batch=B, device=0)
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(i, 1024)) for i in range(B)]
    sess = EncodeSession(ctx, bits)
    tok = torch.randint(0, s.vocab, (B,), device=dev)
    H, D = s.n_head, s.n_embd // s.n_head

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            out = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3, out

    print(json.dumps({"model": args.model, "batch": B, "kv_bytes_per_token": 2 * s.n_layer * s.n_embd * 2,
                      "mem_gb": torch.cuda.memory_allocated() / 1e9}), flush=True)
    for L in lens:
        lm.L = L

        def fwd():
            lm.L = L
            return lm.step(tok)

        lm.hip_attention = True
        ms_fwd, logits = timed(fwd, args.reps)
        lm.hip_attention = False
        ms_fwd_sdpa, _ = timed(fwd, args.reps)
        lm.hip_attention = True
        q = torch.randn((B, H, 1, D), device=dev, dtype=lm.dtype)

        def attn():
            for i in range(s.n_layer):
                kk = lm.k_cache[i, :B, :, : L + 1]
                vv = lm.v_cache[i, :B, :, : L + 1]
                o = F.scaled_dot_product_attention(q, kk, vv)
            return o

        qkv = torch.randn((B, 3 * s.n_embd), device=dev, dtype=lm.dtype)
        out = torch.empty((B, s.n_embd), device=dev, dtype=lm.dtype)
        from neuralsteganography_amd import _lib
        from neuralsteganography_amd.coder import _stream_handle

        def attn_hip():
            for i in range(s.n_layer):
                kc, vc = lm.k_cache[i], lm.v_cache[i]
                rc = _lib.lib().ns_decode_attention(qkv.data_ptr(), qkv.stride(0), kc.data_ptr(), vc.data_ptr(),
                                                    kc.stride(0), kc.stride(1), B, H, D, L, out.data_ptr(),
                                                    out.stride(0), D ** -0.5, _stream_handle())
                assert rc == 0
            return out

        ms_attn, _ = timed(attn, args.reps)
        ms_attn_hip, _ = timed(attn_hip, args.reps)
        ms_coder, _ = timed(lambda: sess.step(logits), args.reps)
        kv = B * (L + 1) * 2 * s.n_layer * s.n_embd * 2
        print(json.dumps({"L": L, "ms_forward": ms_fwd, "ms_forward_sdpa": ms_fwd_sdpa, "ms_attention_sdpa": ms_attn,
                          "ms_attention_hip": ms_attn_hip, "ms_coder": ms_coder, "kv_bytes": kv,
                          "attn_sdpa_GBs": kv / (ms_attn / 1e3) / 1e9, "attn_hip_GBs": kv / (ms_attn_hip / 1e3) / 1e9,
                          "tok_per_s": B / ((ms_fwd + ms_coder) / 1e3)}), flush=True)


if __name__ == "__main__":
    main()
