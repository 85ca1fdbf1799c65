"""Drop-in entry points for callers of the reference's ``code_base/`` scripts (``run_single.py`` & co).

Same names, arguments and return values as ``code_base/arithmetic.py`` (``encode_arithmetic`` :78-217,
``decode_arithmetic`` :220-373) and ``code_base/sample.py`` (``sample`` :6-55), running on the HIP coder with
a KV-cached batched GPT-2 (PyTorch-ROCm).  ``model`` is a Hugging Face GPT-2 (``GPT2LMHeadModel``), an
already built :class:`~neuralsteganography_amd.lm.arithmetic.HipArithmeticLM`, or any batched-logits LM with
the ``prefill``/``step`` protocol; ``enc`` is the tokenizer (``encode``/``decode``).  ``device`` is accepted
for signature compatibility (the coder always runs on the current GPU).

Batched forms (``*_batch``) take lists of messages / texts and run them as one lockstep batch -- the point of
the build; the single-message functions are the batched ones at B = 1.

Behaviour notes (DESIGN.md "Deviations"):
* statistics (avg_NLL, avg_KL, words_per_bit, avg_Hq) are float64 values from fp32 device sums, within
  2e-5 relative of the reference's; tokens and bits are bit-exact;
* the '<eos>' stop of ``arithmetic.py:207-210`` is applied on a 16-token decoded tail per stream;
* ``sample`` draws with a counter-based generator (``seed``; torch.multinomial's stream is not
  reproducible), and also runs ``topk <= 0`` (every id), which the reference's ``sample.py:39`` cannot.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

_PROVIDERS: Dict[int, object] = {}


def _provider(model, enc, logits_dtype: str = "f32"):
    from .lm.arithmetic import HipArithmeticLM

    if isinstance(model, HipArithmeticLM):
        if enc is not None:
            model.tokenizer = enc
        return model
    key = (id(model), id(enc), logits_dtype)
    lm = _PROVIDERS.get(key)
    if lm is None:
        if hasattr(model, "prefill") and hasattr(model, "step"):
            lm = HipArithmeticLM.from_batched(model, enc, logits_dtype=logits_dtype)
        else:
            lm = HipArithmeticLM(model, enc, logits_dtype=logits_dtype)
        _PROVIDERS[key] = lm
    return lm


def _quality(temp, precision, topk, finish_sent=False):
    return {"temp": float(temp), "precision": int(precision), "topk": int(topk), "finish_sent": bool(finish_sent)}


def split_double_newlines(inp: List[int]) -> List[int]:
    """``decode_arithmetic``'s fix-up (arithmetic.py:233-242): token 628 ("\\n\\n") becomes 198, 198."""
    out: List[int] = []
    for t in inp:
        if t == 628:
            out += [198, 198]
        else:
            out.append(int(t))
    return out


def encode_arithmetic_batch(model, enc, messages: Sequence[Sequence[int]], context: Sequence[int],
                            finish_sent: bool = False, device: str = "cuda", temp: float = 1.0,
                            precision: int = 16, topk: int = 50000, stop_text: Optional[str] = "<eos>"
                            ) -> List[Tuple[List[int], float, float, float, float]]:
    """B messages (bit lists) -> per message ``(tokens, avg_NLL, avg_KL, words_per_bit, avg_Hq)``."""
    _ = device
    lm = _provider(model, enc)
    toks, stats = lm.encode_batch([list(m) for m in messages], list(context)[-1022:],
                                  quality=_quality(temp, precision, topk, finish_sent), return_stats=True,
                                  stop_text=stop_text)
    return [(t, s["avg_NLL"], s["avg_KL"], s["words_per_bit"], s["avg_Hq"]) for t, s in zip(toks, stats)]


def encode_arithmetic(model, enc, message: Sequence[int], context: Sequence[int], finish_sent: bool = False,
                      device: str = "cuda", temp: float = 1.0, precision: int = 16, topk: int = 50000):
    """``code_base/arithmetic.py:78`` -- returns ``(output, avg_NLL, avg_KL, words_per_bit, avg_Hq)``."""
    return encode_arithmetic_batch(model, enc, [message], context, finish_sent=finish_sent, device=device,
                                   temp=temp, precision=precision, topk=topk)[0]


def decode_arithmetic_batch(model, enc, texts: Sequence[str], context: Sequence[int], device: str = "cuda",
                            temp: float = 1.0, precision: int = 16, topk: int = 50000) -> List[List[int]]:
    """B cover texts -> the bit list each decodes to (every emitted bit; the caller truncates)."""
    _ = device
    lm = _provider(model, enc)
    token_lists = [split_double_newlines(list(enc.encode(t))) for t in texts]
    return lm.decode_tokens_repair(token_lists, list(context)[-1022:], quality=_quality(temp, precision, topk),
                                   enc=enc)


def decode_arithmetic(model, enc, text: str, context: Sequence[int], device: str = "cuda", temp: float = 1.0,
                      precision: int = 16, topk: int = 50000) -> List[int]:
    """``code_base/arithmetic.py:220`` -- the bit list the cover text decodes to."""
    return decode_arithmetic_batch(model, enc, [text], context, device=device, temp=temp, precision=precision,
                                   topk=topk)[0]


def sample_batch(model, enc, length: int, context: Sequence[int], n: int, temperature: float = 1.0,
                 device: str = "cuda", topk: int = -1, seed: int = 0
                 ) -> List[Tuple[List[int], float, float, float]]:
    """n independent samples -> per sample ``(tokens, avg_NLL, avg_KL, avg_Hq)``."""
    _ = device
    if length <= 0:
        raise ValueError("length must be positive")  # sample.py:7 asserts length > 0
    lm = _provider(model, enc)
    toks, stats = lm.sample_batch(int(n), int(length), list(context)[-1022:], temperature=temperature, topk=topk,
                                  seed=seed)
    return [(t, s["avg_NLL"], s["avg_KL"], s["avg_Hq"]) for t, s in zip(toks, stats)]


def sample(model, enc, length: int, context: Sequence[int], temperature: float = 1.0, device: str = "cuda",
           topk: int = -1, seed: int = 0):
    """``code_base/sample.py:6`` -- returns ``(output, avg_NLL, avg_KL, avg_Hq)``."""
    return sample_batch(model, enc, length, context, 1, temperature=temperature, device=device, topk=topk,
                        seed=seed)[0]


__all__ = ["encode_arithmetic", "decode_arithmetic", "sample", "encode_arithmetic_batch", "decode_arithmetic_batch",
           "sample_batch", "split_double_newlines"]
