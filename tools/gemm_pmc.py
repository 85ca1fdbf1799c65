"""Run one ns_lm_gemm_config shape REPS times (for rocprofv3 --pmc passes and kernel traces).
usage: python tools/gemm_pmc.py M N K EPI CFG [REPS]   (EPI: store|gelu|residual|f32)"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch

    from neuralsteganography_amd import _lib
    from neuralsteganography_amd.coder import _stream_handle

    M, N, K = (int(v) for v in sys.argv[1:4])
    epi = {"store": 0, "gelu": 1, "residual": 2, "f32": 3}[sys.argv[4]]
    cfg = int(sys.argv[5])
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (0.1 * torch.randn((M, K), generator=g, device="cuda")).half()
    wt = (0.1 * torch.randn((N, K), generator=g, device="cuda")).half()
    bias = (0.1 * torch.randn((N,), generator=g, device="cuda")).half()
    y = torch.zeros((M, N), device="cuda", dtype=torch.float32 if epi == 3 else torch.float16)
    L = _lib.lib()
    st = _stream_handle()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(reps + 3):
        if i == 3:
            e0.record()
        assert L.ns_lm_gemm_config(x.data_ptr(), K, wt.data_ptr(), K, bias.data_ptr(), y.data_ptr(), N, M, N, K,
                                   epi, cfg, st) == 0
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"M={M} N={N} K={K} cfg={cfg}: {ms * 1e3:.1f} us, {2.0 * M * N * K / ms / 1e9:.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
