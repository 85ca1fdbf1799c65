"""Diagnose a cover-text reveal with BPE repair on the GPU (tools only): encode covers with the char-merge test
tokenizer, then for each cover compare emitted ids, re-tokenised ids and the repaired decode."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from neuralsteganography_amd import synthetic  # noqa: E402
from neuralsteganography_amd.codec.textio import seed_to_ids, spans_to_text  # noqa: E402
from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM  # noqa: E402
from neuralsteganography_amd.lm.gpt2 import random_gpt2  # noqa: E402
from neuralsteganography_amd.stego import stego_decode_batch, stego_encode_batch  # noqa: E402
from tests.test_gpu_guard import CharMergeTokenizer  # noqa: E402

tok = CharMergeTokenizer()
m = random_gpt2("tiny", vocab_size=64, n_positions=2048, n_embd=128, n_head=2, seed=29)
lm = HipArithmeticLM(m, tok, banned=tok.banned())
q = {"temp": 1.0, "precision": 26, "topk": 300, "finish_sent": False}
secrets = [synthetic.payload_bytes(s, 5 + 7 * s) for s in range(12)]
seed = "Abc"
res = stego_encode_batch(secrets, chunk_bytes=24, ecc="none", quality=q, seed_text=seed, lm=lm)
print("json-spans decode ok:", stego_decode_batch([list(r) for r in res], ecc="none", quality=q, seed_text=seed,
                                                  lm=lm) == secrets, flush=True)
seed_ids = seed_to_ids(seed, tok)
for i, r in enumerate(res[:3]):
    spans = [list(s) for s in r]
    emitted = [t for s in spans for t in s]
    text = spans_to_text(spans, seed_ids, tok)
    retok = tok.encode(text)[len(seed_ids):]
    print(f"cover {i}: spans {[len(s) for s in spans]} emitted {len(emitted)} retok {len(retok)} "
          f"same={retok == emitted} text_tail={text[-20:]!r} emitted_tail={tok.decode(emitted[-5:])!r}", flush=True)
    ctx = list(lm.encode_seed(seed))
    bits, counts, lists, edits = lm.decode_counted_repair([retok], ctx, quality=dict(q, top_k=300))
    rep = lists[0]
    first_diff = next((j for j in range(min(len(rep), len(emitted))) if rep[j] != emitted[j]), None)
    print(f"  repaired len {len(rep)} == emitted: {rep == emitted}; first diff at {first_diff}; edits at "
          f"{[p for p, _ in edits[0]][:12]}", flush=True)
    if first_diff is not None:
        a = max(0, first_diff - 3)
        print("   emitted ", emitted[a:first_diff + 4], repr(tok.decode(emitted[a:first_diff + 4])))
        print("   repaired", rep[a:first_diff + 4], repr(tok.decode(rep[a:first_diff + 4])))
        print("   retok   ", retok[a:first_diff + 4])
