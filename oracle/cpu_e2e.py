"""TEST INFRASTRUCTURE: one worker of bench.py's end-to-end CPU baseline (BASELINE.md "CPU baseline plan",
item 2: a CPU GPT-2 forward plus the coder, on a subsample of streams, extrapolated per core).

Run as a child process (no GPU): ``python -m oracle.cpu_e2e SECONDS SEED VOCAB TEMP PRECISION TOPK PAYLOAD_BYTES``.
On ONE core it runs the reference's own token loop shape (``code_base/arithmetic.py:108-190``: batch 1, the
Hugging Face ``GPT2LMHeadModel`` forward over the 32-token context, then one token per call with the KV cache,
``code_base/arithmetic.py:115-122``) on random-init GPT-2-small weights in float32 (no checkpoint offline), and
feeds each step's logits to the oracle's C encode step (``oracle/nsg_oracle.c``, bit-exact to the reference).
Encodes one synthetic payload after another for about SECONDS and prints one JSON line: payload bits fixed,
cover tokens, elapsed seconds (model construction excluded).
"""

from __future__ import annotations

import ctypes
import json
import sys
import time

import numpy as np


def run(seconds: float, seed: int, vocab: int, temp: float, precision: int, topk: int, payload_bytes: int) -> dict:
    import torch
    from transformers import GPT2Config, GPT2LMHeadModel

    from neuralsteganography_amd import synthetic
    from oracle import oracle

    torch.set_num_threads(1)
    torch.manual_seed(seed)
    model = GPT2LMHeadModel(GPT2Config(vocab_size=vocab)).eval()
    L = oracle.lib()
    ld = ((vocab + 63) // 64) * 64
    row = np.zeros((1, ld), np.float32)
    banned = np.asarray([vocab - 1, 628], dtype=np.int32)
    context = [vocab - 1] + list(range(1000, 1031))  # SURVEY.md §8(d) context
    out = np.zeros(1, np.int32)
    bits_total = tokens = 0
    msg = 0
    t0 = time.perf_counter()
    with torch.inference_mode():
        while time.perf_counter() - t0 < seconds:
            bits = synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(seed * 100003 + msg, payload_bytes))
            msg += 1
            nb = np.asarray([len(bits)], dtype=np.int64)
            pl = np.zeros((1, (len(bits) + 7) // 8), np.uint8)
            pk = np.packbits(np.asarray(bits, np.uint8), bitorder="little")
            pl[0, : pk.size] = pk
            st = (oracle.OrState * 1)()
            L.or_init_state(ctypes.byref(st[0]), precision)
            res = model(torch.tensor([context]), use_cache=True)
            past = res.past_key_values
            n_ctx = len(context)
            while st[0].bit_pos < len(bits) and time.perf_counter() - t0 < seconds:
                row[0, :vocab] = res.logits[0, -1].numpy()
                rc = L.or_encode_batch(row.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ld, 1, vocab,
                                       banned.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 2, 1.0 / temp,
                                       precision, topk, pl.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                       pl.shape[1], nb.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), st,
                                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
                if rc != 0:
                    raise RuntimeError(f"or_encode_batch failed ({rc})")
                tokens += 1
                pos = torch.tensor([[(n_ctx + tokens - 1) % model.config.n_positions]])
                res = model(torch.tensor([[int(out[0])]]), past_key_values=past, position_ids=pos, use_cache=True)
                past = res.past_key_values
            bits_total += int(st[0].bit_pos)
    dt = time.perf_counter() - t0
    return {"bits": bits_total, "tokens": tokens, "seconds": dt, "messages": msg}


if __name__ == "__main__":
    a = sys.argv[1:]
    print(json.dumps(run(float(a[0]), int(a[1]), int(a[2]), float(a[3]), int(a[4]), int(a[5]), int(a[6]))),
          flush=True)
