"""Provider registry: ``load_lm(name, *, device=None)`` as ``src/neuralstego/lm/__init__.py:16-26``.

Names: ``mock`` (identity, C1); ``gpt2``, ``gpt2-medium``, ``gpt2-fa`` (pretrained weights, loaded
offline-first like the reference's ``utils.get_model``, ``utils.py:12-51``); ``gpt2-random``,
``gpt2-medium-random`` (random-init weights of that architecture, for benchmarking without a network).
Every GPT-2 name returns a :class:`HipArithmeticLM` (HIP coder + batched GPT-2).
"""

from __future__ import annotations

from typing import Optional

from ..exceptions import ConfigurationError
from .mock import MockLM

_MODEL_ALIASES = {"gpt2-fa": "HooshvareLab/gpt2-fa"}


def _load_pretrained(name: str):
    try:
        from transformers import AutoModelForCausalLM, AutoTokenizer

        tok = AutoTokenizer.from_pretrained(name, local_files_only=True)
        model = AutoModelForCausalLM.from_pretrained(name, local_files_only=True)
    except Exception as exc:  # offline image: no weights unless pre-downloaded
        raise ConfigurationError(
            f"pretrained weights for '{name}' are not available offline; use '{name.split('/')[-1]}-random' "
            "or place the checkpoint in the Hugging Face cache") from exc
    model.eval()
    return model, tok


def load_lm(name: str, *, device: Optional[str] = None, logits_dtype: str = "f32", **kwargs):
    name_norm = name.lower()
    if name_norm == "mock":
        return MockLM()
    from .arithmetic import HipArithmeticLM

    if name_norm.endswith("-random"):
        from .gpt2 import random_gpt2

        base = name_norm[: -len("-random")]
        if base not in {"gpt2", "gpt2-medium", "gpt2-fa"}:
            raise ConfigurationError(f"unknown random-init architecture: {name}")
        return HipArithmeticLM(random_gpt2(base), None, device=device, logits_dtype=logits_dtype, **kwargs)
    if name_norm in {"gpt2", "gpt2-medium", "gpt2-fa"}:
        model, tok = _load_pretrained(_MODEL_ALIASES.get(name_norm, name_norm))
        return HipArithmeticLM(model, tok, device=device, logits_dtype=logits_dtype, **kwargs)
    raise ConfigurationError(f"unknown language model provider: {name}")


__all__ = ["load_lm", "MockLM"]
