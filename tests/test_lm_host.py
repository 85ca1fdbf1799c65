"""CPU: batched GPT-2 forward vs Hugging Face (reference semantics incl. position wrap), provider registry,
codec slot and quality mapping."""

import copy

import pytest
import torch

from neuralsteganography_amd.codec import api as codec_api
from neuralsteganography_amd.exceptions import ConfigurationError
from neuralsteganography_amd.lm import load_lm
from neuralsteganography_amd.lm.arithmetic import ByteTokenizer, coder_params_from_quality
from neuralsteganography_amd.lm.gpt2 import BatchedGPT2, random_gpt2


def test_batched_gpt2_matches_hf_with_position_wrap():
    """code_base/arithmetic.py:44-48,115-122: one token per step, position = cache_len % n_positions, cache
    never truncated.  fp32 tolerance 1e-5 absolute."""
    m = random_gpt2("tiny", vocab_size=700, n_positions=16)
    g = BatchedGPT2(m, device="cpu", compute_dtype=torch.float32)
    ctx = [5, 7, 9, 11, 13]
    B = 3
    lg = g.prefill(ctx, B, 24)
    with torch.no_grad():
        out = m(torch.tensor([ctx]), use_cache=True)
    assert (lg[0, :700] - out.logits[0, -1]).abs().max().item() < 1e-5
    assert torch.all(lg[:, 700:] == 0)  # padded columns
    pasts = [copy.deepcopy(out.past_key_values) for _ in range(B)]
    gen = torch.Generator().manual_seed(0)
    for t in range(20):  # 5 + 20 > n_positions = 16: exercises the wrap
        tok = torch.randint(0, 700, (B,), generator=gen)
        lg = g.step(tok)
        for b in range(B):
            L = pasts[b].get_seq_length()
            with torch.no_grad():
                o = m(tok[b].view(1, 1), past_key_values=pasts[b], use_cache=True,
                      position_ids=torch.tensor([[L % 16]]))
            pasts[b] = o.past_key_values
            assert (lg[b, :700] - o.logits[0, -1]).abs().max().item() < 1e-5


def test_registry_and_codec_slot_with_mock():
    lm = load_lm("mock")
    toks = codec_api.encode_arithmetic(b"hello stego", lm, quality={})
    assert codec_api.decode_arithmetic(toks, lm, quality={}) == b"hello stego"
    assert codec_api.encode_arithmetic(b"", lm, quality={}) == []
    assert codec_api.decode_arithmetic([], lm, quality={}) == b""
    with pytest.raises(ConfigurationError):
        load_lm("no-such-model")


def test_quality_mapping_follows_reference_defaults_and_aliases():
    p = coder_params_from_quality({}, 50257, "f32")
    assert (p.temp, p.precision, p.topk) == (1.0, 16, 50000)  # code_base/arithmetic.py:85-87
    p = coder_params_from_quality({"temperature": 0.9, "top_k": 300, "precision": 26}, 50257, "f32")
    assert (p.temp, p.precision, p.topk) == (0.9, 26, 300)
    assert p.banned_ids() == [50256, 628]
    with pytest.raises(ConfigurationError):
        coder_params_from_quality({"temp": 0.0}, 50257, "f32")


def test_byte_tokenizer_seed():
    t = ByteTokenizer()
    assert t.encode("<|endoftext|>") == [50256]
    assert t.decode(t.encode("abc")) == "abc"
    assert ByteTokenizer(2000).encode("<|endoftext|>") == [1999]


def test_prefill_rejects_out_of_vocab_ids_on_host():
    g = BatchedGPT2(random_gpt2("tiny", vocab_size=700, n_positions=16), device="cpu",
                    compute_dtype=torch.float32)
    with pytest.raises(ValueError):
        g.prefill([1, 2, 700], 2, 4)
    with pytest.raises(ValueError):
        g.prefill([-1, 2], 2, 4)


def test_stop_candidates_multibyte_last_character_split_across_tokens():
    """a stop text whose last character is several UTF-8 bytes can be completed by a token
    that decodes alone to '' (ByteTokenizer, errors='ignore') or U+FFFD (HF GPT-2, errors='replace'); such ids
    must be in the per-id stop table, or the stop is never detected.  ASCII last characters keep the plain
    containment rule."""
    import numpy as np

    from neuralsteganography_amd.lm.arithmetic import stop_candidates

    tok = ByteTokenizer(300)
    e_bytes = list("é".encode("utf-8"))  # [0xc3, 0xa9]: the completing token 0xa9 decodes alone to ''
    tab = stop_candidates(tok, 300, "café")
    assert tab[e_bytes[1]] and tab[e_bytes[0]]
    assert not tab[ord("a")] and not tab[ord("x")]
    # the stop really is in the decoded output once the second byte arrives, and only then
    out = [ord(c) for c in "caf"] + e_bytes
    assert "café" not in tok.decode(out[:-1]) and "café" in tok.decode(out)

    class ReplaceTok:  # HF-style byte-level decode with errors='replace'
        def decode(self, ids):
            return bytes(int(i) % 256 for i in ids).decode("utf-8", errors="replace")

        def encode(self, text, add_special_tokens=False):
            return list(text.encode("utf-8"))

    tab2 = stop_candidates(ReplaceTok(), 256, "é")
    assert tab2[0xa9] and tab2[0xc3] and not tab2[ord("e")]
    ascii_tab = stop_candidates(tok, 300, "<eos>")
    assert ascii_tab[ord(">")] and not ascii_tab[0xa9]
    assert int(np.count_nonzero(ascii_tab)) == 1  # only '>' (ids 256..299 decode to bytes 0..43)
