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


def test_bpe_repair_merge_past_the_end_restores_the_list():
    """the reference's longer-token branch (code_base/arithmetic.py:321-333) deletes merged tokens one
    by one and raises IndexError when the merge reaches the end of the text -- after part of the list was edited.
    repair_or_restore puts the list back; strict decoding raises DecodeDivergenceError, lenient decoding takes
    the rank-0 token as unrepairable."""
    from neuralsteganography_amd.codec.errors import DecodeDivergenceError
    from neuralsteganography_amd.lm.arithmetic import bpe_repair, repair_or_restore

    class Pieces:
        pieces = ["a", "b", "c", "abc", "ab"]

        def decode(self, ids):
            return "".join(self.pieces[int(i)] for i in ids)

        def encode(self, text):
            out = []
            while text:  # greedy longest match
                best = max((i for i, p in enumerate(self.pieces) if text.startswith(p)), key=lambda i: len(self.pieces[i]))
                out.append(best)
                text = text[len(self.pieces[best]):]
            return out

    enc = Pieces()
    inp = [1, 0, 1, 2]  # "b" "a" "b" "c": candidate "abc" merges the last three tokens
    with pytest.raises(IndexError):
        bpe_repair(enc, list(inp), 1, [3, 4])
    part = list(inp)
    try:
        bpe_repair(enc, part, 1, [3, 4])
    except IndexError:
        pass
    assert part != inp  # the reference's loop had edited the list before raising
    lst = list(inp)
    assert repair_or_restore(enc, lst, 1, [3, 4], strict=False) == 3 and lst == inp
    lst = list(inp)
    with pytest.raises(DecodeDivergenceError):
        repair_or_restore(enc, lst, 1, [3, 4], strict=True)
    assert lst == inp
    lst = list(inp)
    assert repair_or_restore(enc, lst, 1, [4, 3], strict=True) == 4 and lst == [1, 4, 2]  # "a"+"b" -> "ab"


def test_kv_cache_budget_keeps_headroom_and_retries_fragmented_segments(monkeypatch):
    """VERDICT r3 #9 (CPU-mockable): the cache budget leaves headroom_bytes(B) + the reserve fraction free for
    what is allocated after the cache, and _allocate_fitted retries with a fresh budget (idle segments released,
    count_cached=False) when the first request fails on fragmented cached segments (the r03u OOM class)."""
    from types import SimpleNamespace

    m = random_gpt2("tiny", vocab_size=700, n_positions=64)
    g = BatchedGPT2(m, device="cpu", compute_dtype=torch.float32)
    B, GiB = 64, 1 << 30
    per_pos = g.kv_bytes_per_position(B)
    g.device = SimpleNamespace(type="cuda")  # the sizing arithmetic only
    mem = {"free": 40 * GiB, "reserved": 30 * GiB, "allocated": 10 * GiB}
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda dev=None: (mem["free"], 288 * GiB))
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda dev=None: mem["reserved"])
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda dev=None: mem["allocated"])
    want = 10 ** 9
    got = g.fit_positions(B, want)
    assert got == (int(60 * GiB * 0.95) - g.headroom_bytes(B)) // per_pos  # idle cached segments count as free
    assert g.fit_positions(B, want, count_cached=False) == (int(40 * GiB * 0.95) - g.headroom_bytes(B)) // per_pos
    assert g.fit_positions(B, 5) == 5
    assert g.headroom_bytes(4096) > g.headroom_bytes(1) > 2 * GiB

    calls, released = [], []

    def fake_allocate(B_, max_len, T0=0, dtype=None, plain=None):
        calls.append(max_len)
        if len(calls) == 1:
            raise torch.OutOfMemoryError("fragmented segments")

    def fake_empty_cache():
        released.append(True)
        mem["reserved"] = mem["allocated"]  # idle segments returned to the device
        mem["free"] += 20 * GiB

    monkeypatch.setattr(g, "allocate", fake_allocate)
    monkeypatch.setattr(torch.cuda, "empty_cache", fake_empty_cache)
    g._allocate_fitted(B, 32, want, T0=32)
    assert released == [True] and len(calls) == 2
    assert calls[0] == 32 + got
    assert calls[1] == 32 + (int(60 * GiB * 0.95) - g.headroom_bytes(B)) // per_pos
