"""Small-batch LM head: ln_f + head GEMM as two launches (today) vs the head alone under each direct / tiled
configuration (same bits by construction), HIP-event timed.  GPT-2-small shapes: N = 50,304 (padded vocab), K = 768.
usage: python tools/head_probe.py [--M 1 4 16] [--reps 200]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[1, 4, 16])
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    import torch

    from neuralsteganography_amd import _lib
    from neuralsteganography_amd.coder import _stream_handle

    L = _lib.lib()
    st = _stream_handle()
    dev = torch.device("cuda", 0)
    N, K = 50304, 768
    g = torch.Generator(device=dev).manual_seed(3)
    wt = (torch.randn((N, K), generator=g, device=dev) / 28.0).half()
    lw = (1.0 + 0.1 * torch.randn((K,), generator=g, device=dev)).half()
    lb = (0.1 * torch.randn((K,), generator=g, device=dev)).half()
    stream = torch.cuda.current_stream()

    def timed(fn):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps * 1e3

    for M in a.M:
        x = torch.randn((M, K), generator=g, device=dev).half()
        xa = torch.empty_like(x)
        y = torch.empty((M, N), device=dev).half()

        def two():
            assert L.ns_lm_layernorm(x.data_ptr(), K, lw.data_ptr(), lb.data_ptr(), xa.data_ptr(), K, M, K, 1e-5,
                                     st) == 0
            assert L.ns_lm_gemm(xa.data_ptr(), K, wt.data_ptr(), K, None, y.data_ptr(), N, M, N, K,
                                _lib.NS_LM_EPI_STORE, st) == 0

        rec = {"M": M, "ln_plus_head_us": timed(two)}
        ref = y.clone()
        for cfg, name in [(0, "direct16"), (3, "t64_2"), (4, "t64_3")]:
            def one():
                assert L.ns_lm_gemm_config(xa.data_ptr(), K, wt.data_ptr(), K, None, y.data_ptr(), N, M, N, K,
                                           _lib.NS_LM_EPI_STORE, cfg, st) == 0
            rec[f"head_{name}_us"] = timed(one)
            torch.cuda.synchronize()
            rec[f"head_{name}_same_bits"] = bool(torch.equal(y, ref))

        def fused():
            assert L.ns_lm_ln_gemm(x.data_ptr(), K, lw.data_ptr(), lb.data_ptr(), 1e-5, wt.data_ptr(), K, None,
                                   y.data_ptr(), N, M, N, K, _lib.NS_LM_EPI_STORE, xa.data_ptr(), K, st) == 0
        rec["ln_gemm_entry_us"] = timed(fused)
        torch.cuda.synchronize()
        rec["ln_gemm_entry_same_bits"] = bool(torch.equal(y, ref))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
