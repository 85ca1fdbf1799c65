"""Debug helper: compare every ns_lm_gemm_config with the automatic choice for one shape and epilogue.
usage: python tools/gemm_cfg_check.py M N K epi   (epi: store|gelu|residual|f32)"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch

    from neuralsteganography_amd import _lib
    from neuralsteganography_amd.coder import _stream_handle

    M, N, K = (int(v) for v in sys.argv[1:4])
    epi = {"store": 0, "gelu": 1, "residual": 2, "f32": 3}[sys.argv[4]]
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (0.1 * torch.randn((M, K), generator=g, device="cuda")).half()
    wt = (0.1 * torch.randn((N, K), generator=g, device="cuda")).half()
    bias = (0.1 * torch.randn((N,), generator=g, device="cuda")).half()
    ydt = torch.float32 if epi == 3 else torch.float16
    y0 = torch.randn((M, N), generator=g, device="cuda").to(ydt)
    L = _lib.lib()
    ref = y0.clone()
    assert L.ns_lm_gemm(x.data_ptr(), K, wt.data_ptr(), K, bias.data_ptr(), ref.data_ptr(), N, M, N, K, epi,
                        _stream_handle()) == 0
    for cfg in range(L.ns_lm_gemm_configs()):
        y = y0.clone()
        rc = L.ns_lm_gemm_config(x.data_ptr(), K, wt.data_ptr(), K, bias.data_ptr(), y.data_ptr(), N, M, N, K, epi,
                                 cfg, _stream_handle())
        torch.cuda.synchronize()
        bad = (y != ref).nonzero()
        print(cfg, rc, int(bad.shape[0]), bad[:4].tolist(), float((y.float() - ref.float()).abs().max()))


if __name__ == "__main__":
    main()
