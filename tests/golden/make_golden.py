"""Generate golden vectors by running the REFERENCE coder (``code_base/arithmetic.py``) in this container.

This script is the only place that executes reference code. It runs here (the build container, where
``/root/reference`` is mounted) and writes small ``.npz`` fixtures next to itself; the fixtures are data
(inputs + the reference's outputs) and travel with the repo. Nothing on the GPU box reads
``/root/reference``.

Shims:

* ``sys.modules["bitarray"]`` = stub (``code_base/utils.py:3`` imports it; the coder never uses it);
* ``code_base/`` first on ``sys.path`` (``arithmetic.py:9`` does ``from utils import ...``);
* ``arithmetic.max_positions = 1024`` (decode reads an undefined global, ``arithmetic.py:257``);
* the model is a synthetic-logit callable returning ``.logits [1, T, V]`` and ``.past_key_values=None``
  (so ``_prepare_past_for_model``/``_normalise_past`` see ``None`` and no transformers cache API runs);
* the tokenizer stub's ``decode`` never yields ``'<eos>'`` (``arithmetic.py:208-210``) and its ``encode``
  returns the preset token list (``arithmetic.py:233``);
* ``torch.Tensor.sort`` is forced ``stable=True`` through a ``TorchFunctionMode``: the reference's
  ``sort(descending=True)`` (``arithmetic.py:127,268``) has unspecified tie order; the stable order
  (value desc, token id asc) is the build's canonical tie-break (SURVEY.md §7 hard part 2).

Usage: ``python tests/golden/make_golden.py`` (about a minute on 8 cores).
"""

from __future__ import annotations

import json
import sys
import time
import types
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(REPO))

from neuralsteganography_amd import synthetic  # noqa: E402


def _import_reference():
    import torch
    from torch.overrides import TorchFunctionMode

    sys.modules.setdefault("bitarray", types.ModuleType("bitarray"))
    sys.path.insert(0, str(REF / "code_base"))
    import arithmetic as ref  # code_base/arithmetic.py

    assert Path(ref.__file__).resolve() == (REF / "code_base" / "arithmetic.py").resolve(), ref.__file__
    ref.max_positions = 1024

    class StableSort(TorchFunctionMode):
        def __torch_function__(self, func, types_, args=(), kwargs=None):
            kwargs = dict(kwargs or {})
            if func in (torch.Tensor.sort, torch.sort):
                kwargs["stable"] = True
            return func(*args, **kwargs)

    return ref, StableSort


class SyntheticModel:
    """Synthetic LM: call ``t`` returns row ``logits_row(seed, stream, t)`` (context is ignored)."""

    def __init__(self, seed, stream, vocab, scale, dtype, boost=None):
        import torch

        self.torch = torch
        self.seed, self.stream, self.vocab, self.scale, self.dtype = seed, stream, vocab, scale, dtype
        self.boost = dict(boost or {})  # call index -> token id whose logit gets +30
        self.calls = 0
        self.config = types.SimpleNamespace(n_positions=1024)

    def __call__(self, input_ids, past_key_values=None, use_cache=True, position_ids=None):
        row = synthetic.logits_row(self.seed, self.stream, self.calls, self.vocab, self.scale, self.dtype)
        if self.calls in self.boost:
            row = row.copy()
            row[self.boost[self.calls]] += 30.0
        self.calls += 1
        T = int(input_ids.shape[-1])
        logits = self.torch.zeros((1, T, self.vocab), dtype=self.torch.from_numpy(row).dtype)
        logits[0, -1] = self.torch.from_numpy(row.copy())
        return types.SimpleNamespace(logits=logits, past_key_values=None)


class StubTokenizer:
    """decode(): "." for sentence-ending ids (id % 97 == 5 when `finish` is set), else "a"; never '<eos>'."""

    def __init__(self, tokens=None, finish=False):
        self.tokens = list(tokens or [])
        self.finish = finish

    def decode(self, ids):
        if not self.finish:
            return ""
        return "".join("." if int(i) % 97 == 5 else "a" for i in ids)

    def encode(self, text):
        return list(self.tokens)


CONFIGS = {
    # name: vocab, dtype, logit scale, temp, precision, topk, payload bit lengths per stream
    # C2-C4 coder parameters (code_base/run_single.py:21-24) on V = 50,257.
    "g1_v50257_f32_p26_k300": dict(vocab=50257, dtype="f32", scale=3.0, temp=0.9, precision=26, topk=300,
                                   nbits=[384, 384, 256, 1, 7, 13, 200, 512]),
    # C5-like: fp16 logits (ties are common), topk 100.
    "g2_v50257_f16_p26_k100": dict(vocab=50257, dtype="f16", scale=3.0, temp=0.9, precision=26, topk=100,
                                   nbits=[256, 256, 128, 64]),
    # Peaked rows (scale 10): the 1/R threshold binds, so k < topk on many steps.
    "g3_v50257_f32_peaked_p26_k300": dict(vocab=50257, dtype="f32", scale=10.0, temp=1.0, precision=26,
                                          topk=300, nbits=[256, 256, 128, 64]),
    # api.py defaults (_DEFAULT_QUALITY, api.py:81-86): precision 16, topk 50000 (k in the thousands).
    "g4_v50257_f32_p16_k50000": dict(vocab=50257, dtype="f32", scale=3.0, temp=1.0, precision=16,
                                     topk=50000, nbits=[128, 96]),
    # message->bits mode (code_base/run_single.py:52-54): precision 40, topk 60000.
    "g5_v50257_f32_p40_k60000": dict(vocab=50257, dtype="f32", scale=3.0, temp=0.9, precision=40,
                                     topk=60000, nbits=[96, 64]),
    # Small vocabulary (still > 628, the reference bans id 628 unconditionally).
    "g6_v700_f32_p20_k500": dict(vocab=700, dtype="f32", scale=2.0, temp=0.8, precision=20, topk=500,
                                 nbits=[256, 100, 33, 8]),
    # topk above the non-banned count: every candidate kept.
    "g7_v640_f32_p12_k1000": dict(vocab=640, dtype="f32", scale=1.0, temp=1.3, precision=12, topk=1000,
                                  nbits=[200, 64]),
    # finish_sent=True (code_base/arithmetic.py:114,134-137): sentence-ending ids are id % 97 == 5.
    "g8_v50257_f32_p26_k300_finish": dict(vocab=50257, dtype="f32", scale=3.0, temp=0.9, precision=26, topk=300,
                                          nbits=[96, 64, 40, 8], finish_sent=True),
}

LOGIT_SEED = 7

# code_base/sample.py (the non-stego token loop): name -> vocab, dtype, logit scale, temp, topk, token counts
# per stream.  torch.multinomial draws from torch's seeded CPU generator (SAMPLE_TORCH_SEED).  The reference's
# default topk=-1 cannot run: sample.py:39 slices base_log_probs[:-1] (V-1 entries) against V probabilities.
SAMPLE_CONFIGS = {
    "s1_v50257_f32_k300_t09": dict(vocab=50257, dtype="f32", scale=3.0, temp=0.9, topk=300, lengths=[64, 32]),
    "s2_v50257_f32_k50000_t10": dict(vocab=50257, dtype="f32", scale=3.0, temp=1.0, topk=50000, lengths=[48]),
    "s3_v50257_f16_k100_t09": dict(vocab=50257, dtype="f16", scale=3.0, temp=0.9, topk=100, lengths=[48]),
    "s4_v700_f32_k690_t07": dict(vocab=700, dtype="f32", scale=2.0, temp=0.7, topk=690, lengths=[64]),
}
SAMPLE_TORCH_SEED = 1234

# code_base compat (neuralsteganography_amd/code_base.py): encode -> cover text -> decode through the toy
# tokenizer (tests/golden/toy_tokenizer.py), whose re-tokenisation triggers the decode repair
# (arithmetic.py:300-342); "eos" boosts token 650 ("<eos>") at one step so the '<eos>' stop (:207-210) fires.
COMPAT_CONFIGS = {
    "c1_toy_v700_repair": dict(vocab=700, dtype="f32", scale=2.0, temp=1.0, precision=16, topk=600,
                               nbits=[64, 40, 24, 96]),
    "c2_toy_v700_eos": dict(vocab=700, dtype="f32", scale=2.0, temp=1.0, precision=16, topk=600,
                            nbits=[200], boost={5: 650}),
}


class SampleModel(SyntheticModel):
    """sample.py:26 calls ``logits, past = model(prev.unsqueeze(0), past=past)`` (the pre-transformers-5 tuple
    API): return ``(logits, ())`` so ``limit_past`` (code_base/utils.py:19) sees an empty cache."""

    def __call__(self, input_ids, past=None):
        out = SyntheticModel.__call__(self, input_ids)
        return out.logits, ()


def run_config(name, cfg, ref, stable_sort_mode):
    dtype = np.float16 if cfg["dtype"] == "f16" else np.float32
    V = cfg["vocab"]
    banned = [V - 1, 628]
    context = synthetic.DEFAULT_CONTEXT
    out = {"tokens": [], "tok_off": [0], "bits": [], "bit_off": [0], "msg": [], "msg_off": [0],
           "stats": [], "tie_free": []}
    for s, nbits in enumerate(cfg["nbits"]):
        nbytes = (nbits + 7) // 8
        msg = synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, nbytes))[:nbits]
        model = SyntheticModel(LOGIT_SEED, s, V, cfg["scale"], dtype)
        finish = bool(cfg.get("finish_sent", False))
        with stable_sort_mode():
            toks, nll, kl_, wpb, hq = ref.encode_arithmetic(
                model, StubTokenizer(finish=finish), list(msg), context, finish_sent=finish, device="cpu",
                temp=cfg["temp"], precision=cfg["precision"], topk=cfg["topk"])
        nsteps = model.calls
        assert nsteps == len(toks)
        dmodel = SyntheticModel(LOGIT_SEED, s, V, cfg["scale"], dtype)
        with stable_sort_mode():
            bits = ref.decode_arithmetic(dmodel, StubTokenizer(toks, finish=finish), "", context, device="cpu",
                                         temp=cfg["temp"], precision=cfg["precision"], topk=cfg["topk"])
        assert bits[:nbits] == msg, f"{name} stream {s}: reference round trip failed"
        tie_free = all(synthetic.top_region_tie_free(
            synthetic.logits_row(LOGIT_SEED, s, t, V, cfg["scale"], dtype), min(cfg["topk"], V), banned)
            for t in range(nsteps))
        out["tokens"] += list(toks); out["tok_off"].append(len(out["tokens"]))
        out["bits"] += list(bits); out["bit_off"].append(len(out["bits"]))
        out["msg"] += list(msg); out["msg_off"].append(len(out["msg"]))
        out["stats"].append([nll, kl_, wpb, hq])
        out["tie_free"].append(tie_free)
        print(f"  {name} s={s} nbits={nbits} steps={nsteps} decoded={len(bits)} tie_free={tie_free}", flush=True)
    return out


def run_sample_config(name, cfg, stable_sort_mode):
    import torch

    sys.path.insert(0, str(REF / "code_base"))
    import sample as ref_sample  # code_base/sample.py

    assert Path(ref_sample.__file__).resolve() == (REF / "code_base" / "sample.py").resolve()
    dtype = np.float16 if cfg["dtype"] == "f16" else np.float32
    out = {"tokens": [], "tok_off": [0], "stats": []}
    torch.manual_seed(SAMPLE_TORCH_SEED)
    for s, length in enumerate(cfg["lengths"]):
        model = SampleModel(LOGIT_SEED, s, cfg["vocab"], cfg["scale"], dtype)
        with stable_sort_mode():
            toks, nll, kl_, hq = ref_sample.sample(model, StubTokenizer(), length, synthetic.DEFAULT_CONTEXT,
                                                   temperature=cfg["temp"], device="cpu", topk=cfg["topk"])
        assert len(toks) == length == model.calls
        out["tokens"] += list(toks); out["tok_off"].append(len(out["tokens"]))
        out["stats"].append([nll, kl_, hq])
        print(f"  {name} s={s} length={length} NLL={nll:.4f} KL={kl_:.4f} Hq={hq:.4f}", flush=True)
    return out


# src rank coder (src/neuralstego/codec/arithmetic.py encode_with_lm / decode_with_lm) behind the src
# ArithmeticLM's _ModelAdapter (lm/arithmetic.py:45-74: softmax of logits.double()/temp): name -> vocab,
# logit scale, temperature, codec quality, payload bytes per stream.
RANK_CONFIGS = {
    "r1_v50257_k50000": dict(vocab=50257, scale=3.0, temp=1.0, quality={"top_k": 50000}, nbytes=[32, 9]),
    "r2_v50257_k300": dict(vocab=50257, scale=3.0, temp=0.9, quality={"top_k": 300}, nbytes=[24, 5]),
    "r3_v50257_p09": dict(vocab=50257, scale=3.0, temp=1.0, quality={"top_p": 0.9}, nbytes=[24]),
    "r4_v50257_minp": dict(vocab=50257, scale=3.0, temp=1.0, quality={"min_prob": 1e-5}, nbytes=[24]),
    "r5_v50257_k1000_cap6": dict(vocab=50257, scale=3.0, temp=1.0, quality={"top_k": 1000, "cap_per_token_bits": 6},
                                 nbytes=[16]),
    "r6_v700_k600_t07": dict(vocab=700, scale=2.0, temp=0.7, quality={"top_k": 600, "top_p": 0.95}, nbytes=[20, 3]),
}


class RowProvider:
    """``next_token_probs`` of the src _ModelAdapter (lm/arithmetic.py:45-74) over synthetic rows: call t
    returns softmax(float64(logits_row(t)) / temp) computed by torch, whatever the context."""

    def __init__(self, seed, stream, vocab, scale, temp):
        import torch

        self.torch = torch
        self.seed, self.stream, self.vocab, self.scale, self.temp = seed, stream, vocab, scale, temp
        self.calls = 0

    def next_token_probs(self, context_ids):
        row = synthetic.logits_row(self.seed, self.stream, self.calls, self.vocab, self.scale, np.float32)
        self.calls += 1
        logits = self.torch.from_numpy(row.copy()).to(dtype=self.torch.float64) / self.temp
        return self.torch.nn.functional.softmax(logits, dim=-1).numpy()


def run_rank_config(name, cfg):
    sys.path.insert(0, str(REF / "src"))
    from neuralstego.codec import arithmetic as src_coder  # src/neuralstego/codec/arithmetic.py

    assert Path(src_coder.__file__).resolve() == (REF / "src/neuralstego/codec/arithmetic.py").resolve()
    out = {"tokens": [], "tok_off": [0], "cons": [], "payload": [], "pay_off": [0], "decoded": [], "dec_off": [0]}
    for s, nbytes in enumerate(cfg["nbytes"]):
        payload = synthetic.payload_bytes(s, nbytes)
        state = {}
        prov = RowProvider(LOGIT_SEED, s, cfg["vocab"], cfg["scale"], cfg["temp"])
        toks = src_coder.encode_with_lm(payload, prov, context=synthetic.DEFAULT_CONTEXT, quality=cfg["quality"],
                                        state=state)
        dstate = dict(state)
        dprov = RowProvider(LOGIT_SEED, s, cfg["vocab"], cfg["scale"], cfg["temp"])
        dec = src_coder.decode_with_lm(toks, dprov, context=synthetic.DEFAULT_CONTEXT, quality=cfg["quality"],
                                       state=dstate)
        assert dec == payload, f"{name} stream {s}: reference round trip failed"
        out["tokens"] += list(toks); out["tok_off"].append(len(out["tokens"]))
        out["cons"] += list(state["history"])
        out["payload"] += list(payload); out["pay_off"].append(len(out["payload"]))
        out["decoded"] += list(dec); out["dec_off"].append(len(out["decoded"]))
        print(f"  {name} s={s} bytes={nbytes} tokens={len(toks)} bits/token={8 * nbytes / max(1, len(toks)):.2f}",
              flush=True)
    return out


# src rank coder over GENERIC next_token_probs providers (codec/arithmetic.py:122-231 with the provider
# called directly, _next_distribution :337-347): the Zipf MockLM of codec/distribution.py:17-37 (imported from
# the reference itself) and a context-dependent dict provider (tests/golden/providers.py) with a context window.
PROVIDER_CONFIGS = {
    "z1_mock_v32_a12": dict(provider="mock", vocab=32, alpha=1.2, quality=None, nbytes=[16, 3]),
    "z2_mock_v1000_a11_k300_p09": dict(provider="mock", vocab=1000, alpha=1.1, quality={"top_k": 300, "top_p": 0.9},
                                       nbytes=[20]),
    "z3_ctxdict_v500_minp_w6": dict(provider="ctxdict", vocab=500, quality={"min_prob": 1e-3}, max_context=6,
                                    nbytes=[12, 5]),
    # round 4: float64 rows with near-tied neighbours (1e-9 .. 1e-8 relative), unnormalised,
    # over GPT-2's 50,257 ids: top_p (binding) + min_prob, min_prob (binding) + top_k; and a dict provider whose
    # ids exceed 2^17 with top_k + top_p
    "z4_neartie_v50257_p09_minp": dict(provider="neartie", vocab=50257, scale=0.79,
                                       quality={"top_p": 0.9, "min_prob": 2e-6}, nbytes=[24, 9]),
    "z5_neartiedict_v200000_k2000_p095": dict(provider="neartiedict", vocab=200000,
                                              quality={"top_k": 2000, "top_p": 0.95}, nbytes=[20, 7]),
    "z6_neartie_v50257_minp_k30000": dict(provider="neartie", vocab=50257, scale=0.79,
                                          quality={"min_prob": 1.3e-5, "top_k": 30000}, nbytes=[20]),
    # round 5: the z4 / z6 qualities over 100+ tokens per stream (more top_p / min_prob boundary
    # crossings on the near-tie rows)
    "z7_neartie_v50257_p09_minp_long": dict(provider="neartie", vocab=50257, scale=0.79,
                                            quality={"top_p": 0.9, "min_prob": 2e-6}, nbytes=[190, 170]),
    "z8_neartie_v50257_minp_k30000_long": dict(provider="neartie", vocab=50257, scale=0.79,
                                               quality={"min_prob": 1.3e-5, "top_k": 30000}, nbytes=[180]),
}

# crypto.encode_arithmetic / decode_arithmetic over GENERIC providers (the _QualityControlledLM normalises the
# provider's row with numpy's sum, then tempers / filters): T = 1 with top_p (exact), T = 0.8 with top_k
CRYPTO_PROVIDER_CONFIGS = {
    "x1_neartie_v50257_p09": dict(provider="neartie", vocab=50257, scale=0.79, quality={"top_p": 0.9},
                                  nbytes=[24, 6]),
    "x2_neartiedict_v200000_t08_k500": dict(provider="neartiedict", vocab=200000,
                                            quality={"temperature": 0.8, "top_k": 500}, nbytes=[18]),
    # round 5: x1's crypto quality over 100+ tokens per stream
    "x3_neartie_v50257_p09_long": dict(provider="neartie", vocab=50257, scale=0.79, quality={"top_p": 0.9},
                                       nbytes=[200, 160]),
}


def make_provider(cfg):
    if cfg["provider"] == "mock":
        sys.path.insert(0, str(REF / "src"))
        from neuralstego.codec.distribution import MockLM  # src/neuralstego/codec/distribution.py:17-37

        return MockLM(vocab_size=cfg["vocab"], alpha=cfg["alpha"])
    from tests.golden import providers

    if cfg["provider"] == "neartie":
        return providers.NearTieLM(cfg["vocab"], scale=cfg["scale"])
    if cfg["provider"] == "neartiedict":
        return providers.NearTieDictLM(cfg["vocab"])
    return providers.ContextDictLM(cfg["vocab"])


def run_provider_config(name, cfg):
    sys.path.insert(0, str(REF / "src"))
    from neuralstego.codec import arithmetic as src_coder  # src/neuralstego/codec/arithmetic.py

    assert Path(src_coder.__file__).resolve() == (REF / "src/neuralstego/codec/arithmetic.py").resolve()
    out = {"tokens": [], "tok_off": [0], "cons": [], "payload": [], "pay_off": [0], "decoded": [], "dec_off": [0]}
    for s, nbytes in enumerate(cfg["nbytes"]):
        payload = synthetic.payload_bytes(s, nbytes)
        state = {}
        toks = src_coder.encode_with_lm(payload, make_provider(cfg), context=synthetic.DEFAULT_CONTEXT,
                                        quality=cfg["quality"], state=state, max_context=cfg.get("max_context"))
        dstate = dict(state)
        dec = src_coder.decode_with_lm(toks, make_provider(cfg), context=synthetic.DEFAULT_CONTEXT,
                                       quality=cfg["quality"], state=dstate, max_context=cfg.get("max_context"))
        assert dec == payload, f"{name} stream {s}: reference round trip failed"
        out["tokens"] += list(toks); out["tok_off"].append(len(out["tokens"]))
        out["cons"] += list(state["history"])
        out["payload"] += list(payload); out["pay_off"].append(len(out["payload"]))
        out["decoded"] += list(dec); out["dec_off"].append(len(out["decoded"]))
        print(f"  {name} s={s} bytes={nbytes} tokens={len(toks)} bits/token={8 * nbytes / max(1, len(toks)):.2f}",
              flush=True)
    return out


# crypto quality LM (src/neuralstego/crypto/arithmetic.py encode_arithmetic / decode_arithmetic over
# _QualityControlledLM + crypto/quality.py apply_quality): name -> vocab, logit scale, crypto quality
# (temperature on probabilities, top_k, top_p), payload bytes per stream.  Base provider: the untempered
# _ModelAdapter softmax (RowProvider with temp 1.0).
CRYPTO_CONFIGS = {
    "k1_v50257_t08_k5000": dict(vocab=50257, scale=3.0, quality={"temperature": 0.8, "top_k": 5000}, nbytes=[64, 7]),
    "k2_v50257_t13_p09": dict(vocab=50257, scale=3.0, quality={"temperature": 1.3, "top_p": 0.9}, nbytes=[60, 5]),
    "k3_v50257_t07": dict(vocab=50257, scale=3.0, quality={"temperature": 0.7}, nbytes=[30, 2]),
    "k4_v700_t1_k300_p095": dict(vocab=700, scale=2.0, quality={"top_k": 300, "top_p": 0.95}, nbytes=[20]),
}


def crypto_rank_quality(q):
    """The crypto policy as the build's rank-kernel quality keys (prob_temp = temperature on probabilities)."""
    out = {"prob_temp": float(q.get("temperature", 1.0))}
    for k in ("top_k", "top_p"):
        if q.get(k) is not None:
            out[k] = q[k]
    return out


def run_crypto_config(name, cfg):
    sys.path.insert(0, str(REF / "src"))
    from neuralstego.crypto import arithmetic as crypto_coder  # src/neuralstego/crypto/arithmetic.py

    assert Path(crypto_coder.__file__).resolve() == (REF / "src/neuralstego/crypto/arithmetic.py").resolve()
    out = {"tokens": [], "tok_off": [0], "cons": [], "payload": [], "pay_off": [0], "decoded": [], "dec_off": [0]}
    for s, nbytes in enumerate(cfg["nbytes"]):
        payload = synthetic.payload_bytes(s, nbytes)
        prov = RowProvider(LOGIT_SEED, s, cfg["vocab"], cfg["scale"], 1.0)
        toks, state = crypto_coder.encode_arithmetic(payload, prov, quality=cfg["quality"],
                                                     seed_text=synthetic.DEFAULT_CONTEXT)
        dprov = RowProvider(LOGIT_SEED, s, cfg["vocab"], cfg["scale"], 1.0)
        dec = crypto_coder.decode_arithmetic(toks, dprov, quality=cfg["quality"], seed_text=synthetic.DEFAULT_CONTEXT,
                                             state=dict(state))
        assert dec == payload, f"{name} stream {s}: reference round trip failed"
        out["tokens"] += list(toks); out["tok_off"].append(len(out["tokens"]))
        out["cons"] += list(state["history"])
        out["payload"] += list(payload); out["pay_off"].append(len(out["payload"]))
        out["decoded"] += list(dec); out["dec_off"].append(len(out["decoded"]))
        print(f"  {name} s={s} bytes={nbytes} tokens={len(toks)} bits/token={8 * nbytes / max(1, len(toks)):.2f}",
              flush=True)
    return out


def run_crypto_provider_config(name, cfg):
    sys.path.insert(0, str(REF / "src"))
    from neuralstego.crypto import arithmetic as crypto_coder  # src/neuralstego/crypto/arithmetic.py

    assert Path(crypto_coder.__file__).resolve() == (REF / "src/neuralstego/crypto/arithmetic.py").resolve()
    out = {"tokens": [], "tok_off": [0], "cons": [], "payload": [], "pay_off": [0], "decoded": [], "dec_off": [0]}
    for s, nbytes in enumerate(cfg["nbytes"]):
        payload = synthetic.payload_bytes(s, nbytes)
        toks, state = crypto_coder.encode_arithmetic(payload, make_provider(cfg), quality=cfg["quality"],
                                                     seed_text=synthetic.DEFAULT_CONTEXT)
        dec = crypto_coder.decode_arithmetic(toks, make_provider(cfg), quality=cfg["quality"],
                                             seed_text=synthetic.DEFAULT_CONTEXT, state=dict(state))
        assert dec == payload, f"{name} stream {s}: reference round trip failed"
        out["tokens"] += list(toks); out["tok_off"].append(len(out["tokens"]))
        out["cons"] += list(state["history"])
        out["payload"] += list(payload); out["pay_off"].append(len(out["payload"]))
        out["decoded"] += list(dec); out["dec_off"].append(len(out["decoded"]))
        print(f"  {name} s={s} bytes={nbytes} tokens={len(toks)} bits/token={8 * nbytes / max(1, len(toks)):.2f}",
              flush=True)
    return out


def run_compat_config(name, cfg, ref, stable_sort_mode):
    from tests.golden.toy_tokenizer import ToyTokenizer

    enc = ToyTokenizer(cfg["vocab"])
    V = cfg["vocab"]
    context = synthetic.DEFAULT_CONTEXT
    out = {"tokens": [], "tok_off": [0], "bits": [], "bit_off": [0], "msg": [], "msg_off": [0], "stats": [],
           "text": [], "text_off": [0]}
    for s, nbits in enumerate(cfg["nbits"]):
        msg = synthetic.bytes_to_bits_lsb(synthetic.payload_bytes(s, (nbits + 7) // 8))[:nbits]
        boost = {int(k): v for k, v in cfg.get("boost", {}).items()}
        model = SyntheticModel(LOGIT_SEED, s, V, cfg["scale"], np.float32, boost=boost)
        with stable_sort_mode():
            toks, nll, kl_, wpb, hq = ref.encode_arithmetic(model, enc, list(msg), context, device="cpu",
                                                            temp=cfg["temp"], precision=cfg["precision"],
                                                            topk=cfg["topk"])
        text = enc.decode(toks)
        dmodel = SyntheticModel(LOGIT_SEED, s, V, cfg["scale"], np.float32, boost=boost)
        with stable_sort_mode():
            bits = ref.decode_arithmetic(dmodel, enc, text, context, device="cpu", temp=cfg["temp"],
                                         precision=cfg["precision"], topk=cfg["topk"])
        retok = enc.encode(text)
        out["tokens"] += list(toks); out["tok_off"].append(len(out["tokens"]))
        out["bits"] += list(bits); out["bit_off"].append(len(out["bits"]))
        out["msg"] += list(msg); out["msg_off"].append(len(out["msg"]))
        out["stats"].append([nll, kl_, wpb, hq])
        tb = list(text.encode("utf-8"))
        out["text"] += tb; out["text_off"].append(len(out["text"]))
        print(f"  {name} s={s} nbits={nbits} tokens={len(toks)} retokenised={len(retok)} "
              f"same={retok == list(toks)} decoded={len(bits)} roundtrip={bits[:nbits] == list(msg)}", flush=True)
    return out


def main(names=None):
    ref, stable = _import_reference()
    for name, cfg in CRYPTO_CONFIGS.items():
        if names and name not in names:
            continue
        res = run_crypto_config(name, cfg)
        meta = dict(cfg, name=name, kind="crypto", temp=1.0, crypto_quality=cfg["quality"],
                    quality=crypto_rank_quality(cfg["quality"]), logit_seed=LOGIT_SEED,
                    payload_seed=synthetic.PAYLOAD_SEED, context=synthetic.DEFAULT_CONTEXT,
                    reference="src/neuralstego/crypto/arithmetic.py encode_arithmetic / decode_arithmetic")
        np.savez_compressed(
            HERE / f"{name}.npz",
            meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8),
            tokens=np.asarray(res["tokens"], dtype=np.int32), tok_off=np.asarray(res["tok_off"], np.int64),
            consumed=np.asarray(res["cons"], dtype=np.int32),
            payload=np.asarray(res["payload"], dtype=np.uint8), pay_off=np.asarray(res["pay_off"], np.int64),
            decoded=np.asarray(res["decoded"], dtype=np.uint8), dec_off=np.asarray(res["dec_off"], np.int64))
    for name, cfg in CRYPTO_PROVIDER_CONFIGS.items():
        if names and name not in names:
            continue
        res = run_crypto_provider_config(name, cfg)
        meta = dict(cfg, name=name, kind="crypto_provider", crypto_quality=cfg["quality"],
                    quality=crypto_rank_quality(cfg["quality"]), payload_seed=synthetic.PAYLOAD_SEED,
                    context=synthetic.DEFAULT_CONTEXT,
                    reference="src/neuralstego/crypto/arithmetic.py encode_arithmetic / decode_arithmetic over "
                              "tests/golden/providers.py " + cfg["provider"])
        np.savez_compressed(
            HERE / f"{name}.npz",
            meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8),
            tokens=np.asarray(res["tokens"], dtype=np.int32), tok_off=np.asarray(res["tok_off"], np.int64),
            consumed=np.asarray(res["cons"], dtype=np.int32),
            payload=np.asarray(res["payload"], dtype=np.uint8), pay_off=np.asarray(res["pay_off"], np.int64),
            decoded=np.asarray(res["decoded"], dtype=np.uint8), dec_off=np.asarray(res["dec_off"], np.int64))
    for name, cfg in PROVIDER_CONFIGS.items():
        if names and name not in names:
            continue
        res = run_provider_config(name, cfg)
        meta = dict(cfg, name=name, kind="provider", payload_seed=synthetic.PAYLOAD_SEED,
                    context=synthetic.DEFAULT_CONTEXT,
                    reference="src/neuralstego/codec/arithmetic.py encode_with_lm / decode_with_lm over "
                              + ("codec/distribution.py MockLM" if cfg["provider"] == "mock"
                                 else "tests/golden/providers.py " + {"ctxdict": "ContextDictLM",
                                                                      "neartie": "NearTieLM",
                                                                      "neartiedict": "NearTieDictLM"}[cfg["provider"]]))
        np.savez_compressed(
            HERE / f"{name}.npz",
            meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8),
            tokens=np.asarray(res["tokens"], dtype=np.int32), tok_off=np.asarray(res["tok_off"], np.int64),
            consumed=np.asarray(res["cons"], dtype=np.int32),
            payload=np.asarray(res["payload"], dtype=np.uint8), pay_off=np.asarray(res["pay_off"], np.int64),
            decoded=np.asarray(res["decoded"], dtype=np.uint8), dec_off=np.asarray(res["dec_off"], np.int64))
    for name, cfg in RANK_CONFIGS.items():
        if names and name not in names:
            continue
        res = run_rank_config(name, cfg)
        meta = dict(cfg, name=name, kind="rank", logit_seed=LOGIT_SEED, payload_seed=synthetic.PAYLOAD_SEED,
                    context=synthetic.DEFAULT_CONTEXT,
                    reference="src/neuralstego/codec/arithmetic.py encode_with_lm / decode_with_lm")
        np.savez_compressed(
            HERE / f"{name}.npz",
            meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8),
            tokens=np.asarray(res["tokens"], dtype=np.int32), tok_off=np.asarray(res["tok_off"], np.int64),
            consumed=np.asarray(res["cons"], dtype=np.int32),
            payload=np.asarray(res["payload"], dtype=np.uint8), pay_off=np.asarray(res["pay_off"], np.int64),
            decoded=np.asarray(res["decoded"], dtype=np.uint8), dec_off=np.asarray(res["dec_off"], np.int64))
    for name, cfg in COMPAT_CONFIGS.items():
        if names and name not in names:
            continue
        res = run_compat_config(name, cfg, ref, stable)
        meta = dict(cfg, name=name, kind="compat", logit_seed=LOGIT_SEED, payload_seed=synthetic.PAYLOAD_SEED,
                    context=synthetic.DEFAULT_CONTEXT, banned=[cfg["vocab"] - 1, 628], tokenizer="ToyTokenizer",
                    reference="code_base/arithmetic.py encode_arithmetic -> text -> decode_arithmetic",
                    sort="stable (value desc, id asc)")
        meta["boost"] = {str(k): v for k, v in cfg.get("boost", {}).items()}
        np.savez_compressed(
            HERE / f"{name}.npz",
            meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8),
            tokens=np.asarray(res["tokens"], dtype=np.int32), tok_off=np.asarray(res["tok_off"], np.int64),
            bits=np.asarray(res["bits"], dtype=np.uint8), bit_off=np.asarray(res["bit_off"], np.int64),
            msg=np.asarray(res["msg"], dtype=np.uint8), msg_off=np.asarray(res["msg_off"], np.int64),
            stats=np.asarray(res["stats"], dtype=np.float64),
            text=np.asarray(res["text"], dtype=np.uint8), text_off=np.asarray(res["text_off"], np.int64))
    for name, cfg in SAMPLE_CONFIGS.items():
        if names and name not in names:
            continue
        res = run_sample_config(name, cfg, stable)
        meta = dict(cfg, name=name, kind="sample", logit_seed=LOGIT_SEED, torch_seed=SAMPLE_TORCH_SEED,
                    context=synthetic.DEFAULT_CONTEXT, banned=[cfg["vocab"] - 1, 628],
                    reference="code_base/sample.py sample", sort="stable (value desc, id asc)")
        np.savez_compressed(
            HERE / f"{name}.npz",
            meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8),
            tokens=np.asarray(res["tokens"], dtype=np.int32), tok_off=np.asarray(res["tok_off"], np.int64),
            stats=np.asarray(res["stats"], dtype=np.float64))
    for name, cfg in CONFIGS.items():
        if names and name not in names:
            continue
        t0 = time.time()
        res = run_config(name, cfg, ref, stable)
        meta = dict(cfg, name=name, logit_seed=LOGIT_SEED, payload_seed=synthetic.PAYLOAD_SEED,
                    context=synthetic.DEFAULT_CONTEXT, banned=[cfg["vocab"] - 1, 628],
                    reference="code_base/arithmetic.py encode_arithmetic/decode_arithmetic",
                    sort="stable (value desc, id asc)")
        np.savez_compressed(
            HERE / f"{name}.npz",
            meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8),
            tokens=np.asarray(res["tokens"], dtype=np.int32), tok_off=np.asarray(res["tok_off"], np.int64),
            bits=np.asarray(res["bits"], dtype=np.uint8), bit_off=np.asarray(res["bit_off"], np.int64),
            msg=np.asarray(res["msg"], dtype=np.uint8), msg_off=np.asarray(res["msg_off"], np.int64),
            stats=np.asarray(res["stats"], dtype=np.float64),
            tie_free=np.asarray(res["tie_free"], dtype=np.bool_))
        print(f"{name}: {time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
