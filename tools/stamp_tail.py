"""Phase timeline of the split wide step's tail kernel (diagnostic build: -DNSG_STAMPS=1 -DNSG_WIDE_SPLIT=1
-DNSG_NOSORT=1).  Stamps of the tail kernel (thread 0, s_memtime of one CU): 11 entry, 5 after the exps + mass +
first barrier, 6 after the histogram + prefix, 7 after the scatter, 8 after wave 0's resolve + finish.
python tools/stamp_tail.py --lib neuralsteganography_amd/_build/variants/tstamps.so"""
import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--dtype", default="f32")
    a = ap.parse_args()
    os.environ["NSG_CODER_LIB"] = a.lib
    import numpy as np
    import torch

    from neuralsteganography_amd import _lib, synthetic
    from neuralsteganography_amd.coder import CoderContext, CoderParams, EncodeSession, row_stride

    L = _lib.lib()
    L.ns_set_stamps.restype = ctypes.c_int
    L.ns_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    V, B = 50257, 4096
    params = CoderParams(vocab=V, precision=16, temp=1.0, topk=50000, dtype=a.dtype)
    ctx = CoderContext(params, max_batch=B)
    ld = row_stride(V, a.dtype)
    g = torch.Generator(device="cuda")
    pool = []
    for i in range(3):
        g.manual_seed(i)
        pool.append((3.0 * torch.randn((B, ld), generator=g, device="cuda")).to(params.torch_dtype))
    sess = EncodeSession(ctx, [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, 256)) for s in range(B)])
    stamps = torch.zeros((B, 16), dtype=torch.int64, device="cuda")
    rows = []
    for t in range(6):
        stamps.zero_()
        L.ns_set_stamps(ctx._h, ctypes.c_void_p(stamps.data_ptr() if t >= 2 else 0))
        sess.step(pool[t % 3])
        torch.cuda.synchronize()
        if t < 2:
            continue
        raw = stamps.cpu().numpy().astype(np.int64)
        seq = raw[:, [11, 5, 6, 7, 8]]
        ok = np.all(seq > 0, axis=1) & np.all(np.diff(seq, axis=1) >= 0, axis=1)
        rows.append(np.diff(seq[ok], axis=1) / 2100.0)  # ticks -> us at ~2.1 GHz (shader clock, approximate)
    d = np.concatenate(rows)
    names = ["exps_mass_barrier", "histogram_prefix", "scatter", "resolve_finish"]
    out = {"lib": Path(a.lib).name, "valid": int(len(d)), "phases_us_at_2p1GHz": {}}
    for i, n in enumerate(names):
        out["phases_us_at_2p1GHz"][n] = {"mean": round(float(d[:, i].mean()), 2), "p50": round(float(np.median(d[:, i])), 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
