"""TEST INFRASTRUCTURE: one worker of bench.py's ``cpu_baseline`` leg ("one process per host core").

Run as a child process (no GPU): ``python -m oracle.cpu_baseline SECONDS STREAMS SEED VOCAB TEMP PRECISION TOPK
PAYLOAD_BYTES``.  Encodes STREAMS synthetic streams (3·N(0,1) fp32 logit rows, the bench workload's
distribution; payloads from ``synthetic.payload_bytes``) with the oracle's batched C encode step on ONE core for
about SECONDS and prints one JSON line: payload bits fixed, stream-steps, elapsed seconds.
"""

from __future__ import annotations

import ctypes
import json
import sys
import time

import numpy as np


def run(seconds: float, streams: int, seed: int, vocab: int, temp: float, precision: int, topk: int,
        payload_bytes: int) -> dict:
    from neuralsteganography_amd import synthetic
    from oracle import oracle

    L = oracle.lib()
    ld = ((vocab + 63) // 64) * 64
    rng = np.random.default_rng(seed)
    pool = [np.ascontiguousarray((3.0 * rng.standard_normal((streams, ld))).astype(np.float32)) for _ in range(2)]
    bits = [synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(seed * 100003 + s, payload_bytes))
            for s in range(streams)]
    nb = np.asarray([len(b) for b in bits], dtype=np.int64)
    pl = np.zeros((streams, (int(nb.max()) + 7) // 8), np.uint8)
    for i, b in enumerate(bits):
        pk = np.packbits(np.asarray(b, np.uint8), bitorder="little")
        pl[i, : pk.size] = pk
    banned = np.asarray([vocab - 1, 628], dtype=np.int32)
    st = (oracle.OrState * streams)()
    for i in range(streams):
        L.or_init_state(ctypes.byref(st[i]), precision)
    out = np.zeros(streams, np.int32)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        rows = pool[steps % 2]
        rc = L.or_encode_batch(rows.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ld, streams, vocab,
                               banned.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 2, 1.0 / temp, precision, topk,
                               pl.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), pl.shape[1],
                               nb.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), st,
                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        if rc != 0:
            raise RuntimeError(f"or_encode_batch failed ({rc})")
        steps += 1
    dt = time.perf_counter() - t0
    return {"bits": int(sum(st[i].bit_pos for i in range(streams))), "stream_steps": steps * streams,
            "seconds": dt}


if __name__ == "__main__":
    a = sys.argv[1:]
    print(json.dumps(run(float(a[0]), int(a[1]), int(a[2]), int(a[3]), float(a[4]), int(a[5]), int(a[6]),
                         int(a[7]))), flush=True)
