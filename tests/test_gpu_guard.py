"""GPU: the quality guard's LM metrics on the HIP row kernel and the batched cover generation loop.

* ns_score_rows (include/nsg_score.h) vs float64 torch log-softmax: NLL of the label and row entropy,
  fp32 and fp16 rows, ragged V, rows without a label; 2e-5 relative + 1e-9 absolute (fp32 partials).
* HipLMScorer (one causal forward + ns_score_rows) vs the reference formulas evaluated with Hugging Face's
  GPT2LMHeadModel on the CPU: ppl / avg_nll / token_count (metrics/lm_scorer.py:121-131, the shifted mean
  loss) and avg_entropy (metrics/entropy.py:36-46); fp32 compute 2e-4, fp16 compute 3e-2 absolute on avg_nll.
* cover_generate_batch over the HIP provider with a GPU-scored guard: every secret either passes (and its
  spans decode back) or raises QualityGateError after the whole schedule.
"""

import json

import numpy as np
import pytest
import torch

from neuralsteganography_amd import synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,V", [("f32", 50257), ("f16", 50257), ("f32", 700), ("f16", 61)])
def test_score_rows_matches_float64_reference(dtype, V):
    from neuralsteganography_amd import _lib
    from neuralsteganography_amd.coder import _stream_handle, row_stride

    n = 37
    ld = row_stride(V, dtype)
    g = torch.Generator(device="cuda").manual_seed(V)
    x = torch.randn((n, ld), generator=g, device="cuda") * 4.0
    x[3, :V] = 0.0  # flat row
    x[4, 5] = 60.0  # one dominant id
    t = x.half() if dtype == "f16" else x
    labels = torch.randint(0, V, (n,), device="cuda", dtype=torch.int32)
    labels[7] = -1
    nll = torch.full((n,), float("nan"), dtype=torch.float64, device="cuda")
    ent = torch.full_like(nll, float("nan"))
    rc = _lib.lib().ns_score_rows(t.data_ptr(), t.stride(0), n, V, _lib.NS_DTYPE_F16 if dtype == "f16" else 0,
                                  labels.data_ptr(), nll.data_ptr(), ent.data_ptr(), _stream_handle())
    assert rc == 0
    torch.cuda.synchronize()
    ref = t[:, :V].double()
    lp = torch.log_softmax(ref, -1)
    want_nll = -lp.gather(1, labels.clamp(min=0).long()[:, None])[:, 0]
    want_nll[7] = 0.0
    want_ent = -(lp.exp() * lp).sum(-1)
    for got, want in ((nll, want_nll), (ent, want_ent)):
        err = (got - want).abs() / (want.abs() + 1.0)
        assert err.max().item() < 2e-5, err.max().item()


def _hf_metrics(model, ids):
    with torch.no_grad():
        logits = model(torch.tensor([ids])).logits[0].double()
    lp = torch.log_softmax(logits[:-1], -1)
    nll = -lp.gather(1, torch.tensor(ids[1:])[:, None])[:, 0]
    p = torch.softmax(logits[:-1], -1)
    ent = -(p * torch.log(p + 1e-12)).sum(-1)
    return float(nll.mean()), float(ent.mean())


@pytest.mark.parametrize("compute_dtype,tol", [(torch.float32, 2e-4), (torch.float16, 3e-2)])
def test_hip_lm_scorer_matches_hf_formulas(compute_dtype, tol):
    from neuralsteganography_amd.lm.arithmetic import ByteTokenizer
    from neuralsteganography_amd.lm.gpt2 import BatchedGPT2, random_gpt2
    from neuralsteganography_amd.metrics import HipLMScorer

    m = random_gpt2("gpt2", seed=21)
    lm = BatchedGPT2(m, device="cuda", compute_dtype=compute_dtype,
                     logits_dtype=torch.float16 if compute_dtype == torch.float16 else torch.float32)
    tok = ByteTokenizer(50257)
    texts = ["hello world, a cover text to score.", "short one", "x", "", "   ", "longer text " * 9]
    sc = HipLMScorer(lm, tok, rows_per_batch=96)  # forces several padded batches
    got = sc.metrics_batch(texts)
    for text, g in zip(texts, got):
        if not text.split():
            assert g == {"ppl": 0.0, "avg_nll": 0.0, "token_count": 0, "avg_entropy": 0.0}
            continue
        ids = tok.encode(text)
        assert g["token_count"] == len(ids)
        if len(ids) < 2:
            assert np.isnan(g["avg_nll"]) and np.isnan(g["avg_entropy"])
            continue
        nll, ent = _hf_metrics(m, ids)
        assert abs(g["avg_nll"] - nll) < tol and abs(g["avg_entropy"] - ent) < tol
        assert abs(g["ppl"] - np.exp(nll)) < tol * np.exp(nll) * 2
    single = sc.score(texts[0])
    assert abs(single["avg_nll"] - got[0]["avg_nll"]) < 1e-3


def test_cover_generate_batch_with_gpu_guard_roundtrip():
    from neuralsteganography_amd.cover import cover_generate_batch
    from neuralsteganography_amd.detect import QualityGuard
    from neuralsteganography_amd.exceptions import QualityGateError
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2
    from neuralsteganography_amd.metrics import HipLMScorer, LMScorer
    from neuralsteganography_amd.stego import stego_decode, stego_encode

    m = random_gpt2("tiny", vocab_size=2000, n_positions=512, seed=17)
    lm = HipArithmeticLM(m, None, compute_dtype=torch.float32)
    guard = QualityGuard(lm_scorer=LMScorer(scorer=HipLMScorer.from_provider(lm)))
    secrets = [b"first secret", b"second, longer secret message", b"3"]
    # finish_sent off: the byte tokenizer's sentence ends (ids = 46, 33, 63 mod 256) are never a random LM's top-1
    q = {"temp": 0.9, "precision": 26, "topk": 300, "finish_sent": False}
    # a permissive gate passes everything at attempt 1
    out = cover_generate_batch(secrets, seed_text="seed", quality=q, ecc="none", lm=lm, quality_guard=guard,
                               gate_thresholds={"max_ppl": 1e9, "max_ngram_repeat": 1.0, "min_ttr": 0.0,
                                                "max_avg_entropy": 1e9})
    assert all(isinstance(t, str) for t in out)
    # an impossible gate rejects every attempt of every secret
    out = cover_generate_batch(secrets, seed_text="seed", quality=q, ecc="none", lm=lm, quality_guard=guard,
                               gate_thresholds={"max_ppl": 0.5}, regen_attempts=2, return_errors=True)
    assert all(isinstance(e, QualityGateError) and e.reasons[0].startswith("ppl ") for e in out)
    # the spans behind a cover decode back (cover_reveal's JSON-spans path)
    spans = stego_encode(secrets[1], ecc="none", seed_text="seed", quality=q, lm=lm)
    assert stego_decode(json.loads(json.dumps([list(s) for s in spans])), ecc="none", seed_text="seed", quality=q,
                        lm=lm) == secrets[1]


class IdTokenizer:
    """Test tokenizer whose decode/encode round-trip every id exactly: id i -> " w<i>", with a sentence-ending
    " w<i>." for every id but 3 -- a random LM's top-1 tail must reach a sentence end (the
    reference would loop forever otherwise); the last id is <|endoftext|>."""

    def __init__(self, vocab):
        self.vocab = vocab
        self.eos_id = vocab - 1

    def _piece(self, i):
        return "<|endoftext|>" if i == self.eos_id else f" w{i}" + ("." if i != 3 else "")

    def decode(self, ids, skip_special_tokens=False):
        return "".join("" if (skip_special_tokens and int(i) == self.eos_id) else self._piece(int(i)) for i in ids)

    def encode(self, text, add_special_tokens=False):
        import re

        out = []
        for m in re.finditer(r"<\|endoftext\|>|w(\d+)", text):
            out.append(self.eos_id if m.group(1) is None else int(m.group(1)))
        return out


@pytest.mark.parametrize("finish_sent", [True, False])
def test_cover_text_round_trip_gpu_provider(finish_sent):
    """cover_generate_batch (HIP provider, finish_sent tails) -> cover TEXT -> cover_reveal_batch: spans are
    recovered from the text by batched decoding (texts_to_spans) and every secret comes back."""
    from neuralsteganography_amd.cover import cover_generate_batch, cover_reveal_batch
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2

    m = random_gpt2("tiny", vocab_size=2000, n_positions=1024, seed=23)
    lm = HipArithmeticLM(m, IdTokenizer(2000), compute_dtype=torch.float32)
    q = {"temp": 0.9, "precision": 26, "topk": 300, "finish_sent": finish_sent}
    secrets = [b"first secret", bytes(range(60)), b"z"]
    seed = "w5. w6. w3"
    texts = cover_generate_batch(secrets, seed_text=seed, quality=q, ecc="none", lm=lm, quality_gate=False,
                                 chunk_bytes=24)
    assert all(t.startswith(seed) for t in texts)
    assert cover_reveal_batch(texts, seed_text=seed, quality=q, ecc="none", lm=lm) == secrets


class CharMergeTokenizer:
    """BPE-style test tokenizer over 64 ids: 'a'-'z', 'A'-'Z', '-', four digits, six two-letter merges ("th",
    "he", "in", "er", "an", "re": ids 57-62) and <|endoftext|> (63).  ``encode`` is greedy longest match, so a
    cover whose coder emitted 't', 'h' re-tokenises to the merge "th".  The provider bans the merges (and the
    end of text), so the coder only ever emits single characters and every merge in a re-tokenised text is a
    BPE artefact that the reference's repair (code_base/arithmetic.py:300-342) undoes: the only kept candidate
    whose text is a prefix of "th" is "t"."""

    MERGES = ["th", "he", "in", "er", "an", "re"]

    def __init__(self):
        import string

        # no whitespace piece: spans_to_text strips the cover (textio.py:37-55), which would drop a trailing one
        self.pieces = list(string.ascii_lowercase) + list(string.ascii_uppercase) + ["-"] + list("0123")
        self.pieces += self.MERGES + ["<|endoftext|>"]
        assert len(self.pieces) == 64
        self.lookup = {p: i for i, p in enumerate(self.pieces)}
        self.eos_id = 63

    def banned(self):
        return [63] + [self.lookup[m] for m in self.MERGES]

    def decode(self, ids):
        return "".join(self.pieces[int(i)] for i in ids)

    def encode(self, text, add_special_tokens=False):
        out, i = [], 0
        while i < len(text):
            if text.startswith("<|endoftext|>", i):
                out.append(63)
                i += len("<|endoftext|>")
                continue
            two = self.lookup.get(text[i:i + 2])
            if two is not None and i + 2 <= len(text):
                out.append(two)
                i += 2
            elif text[i] in self.lookup:
                out.append(self.lookup[text[i]])
                i += 1
            else:
                i += 1  # unknown character: dropped
        return out


def test_cover_text_reveal_with_bpe_repair():
    """Cover TEXT whose re-tokenisation differs from the emitted ids (greedy merges, within spans and across
    span boundaries): texts_to_spans repairs the received ids while decoding (code_base/arithmetic.py:233-242,
    300-342 via decode_counted_repair) and every secret comes back -- also those whose covers re-tokenise
    differently."""
    from neuralsteganography_amd.codec.textio import seed_to_ids, spans_to_text
    from neuralsteganography_amd.cover import cover_reveal_batch
    from neuralsteganography_amd.lm.arithmetic import HipArithmeticLM
    from neuralsteganography_amd.lm.gpt2 import random_gpt2
    from neuralsteganography_amd.stego import stego_encode_batch

    tok = CharMergeTokenizer()
    # fp16 compute: the batch-invariant native decode step, so a cover decodes at any batch size (fp32 compute
    # keeps PyTorch's GEMMs, whose results depend on the batch: decode would need the encoder's composition)
    m = random_gpt2("tiny", vocab_size=64, n_positions=2048, n_embd=128, n_head=2, seed=29)
    lm = HipArithmeticLM(m, tok, banned=tok.banned())
    q = {"temp": 1.0, "precision": 26, "topk": 300, "finish_sent": False}
    secrets = [synthetic.payload_bytes(s, 5 + 7 * s) for s in range(12)]
    seed = "Abc"
    res = stego_encode_batch(secrets, chunk_bytes=24, ecc="none", quality=q, seed_text=seed, lm=lm)
    seed_ids = seed_to_ids(seed, tok)
    texts, differs = [], []
    for r in res:
        assert all(t not in tok.banned() for s in r for t in s)
        text = spans_to_text([list(s) for s in r], seed_ids, tok)
        texts.append(text)
        differs.append(tok.encode(text) != seed_ids + [t for s in r for t in s])
    assert sum(differs) >= 3, "too few covers re-tokenise differently: pick another seed"
    got = cover_reveal_batch(texts, seed_text=seed, quality=q, ecc="none", lm=lm)
    assert got == secrets


def test_guard_metrics_are_batch_invariant_1024():
    """a cover's guard metrics (GPU perplexity / average entropy through the native scoring forward)
    are bit-identical scored alone and inside a batch of 1,024 texts of other lengths (the reference scores one
    cover at a time; a cover near the gate threshold must not pass or fail by batch composition)."""
    from neuralsteganography_amd.lm.arithmetic import ByteTokenizer
    from neuralsteganography_amd.lm.gpt2 import BatchedGPT2, random_gpt2
    from neuralsteganography_amd.metrics import HipLMScorer

    m = random_gpt2("gpt2", seed=22)
    lm = BatchedGPT2(m, device="cuda", compute_dtype=torch.float16, logits_dtype=torch.float16)
    sc = HipLMScorer(lm, ByteTokenizer(50257), rows_per_batch=40000)
    rng = np.random.default_rng(4)
    words = ["alpha", "beta", "gamma", "delta", "stego", "cover", "token", "text", "x"]
    texts = [" ".join(rng.choice(words, size=int(rng.integers(1, 40)))) for _ in range(1024)]
    batch = sc.metrics_batch(texts)
    for i in (0, 1, 511, 1023):
        alone = sc.metrics_batch([texts[i]])[0]
        assert alone == batch[i], i
