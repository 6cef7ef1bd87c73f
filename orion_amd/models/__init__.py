"""Decoder-only transformer models built on :mod:`orion_amd.ops`."""
from .gpt2 import GPT, GPTConfig, build_gpt2, PRESETS as GPT2_PRESETS  # noqa: F401
from .llama import Llama, LlamaConfig, build_llama, PRESETS as LLAMA_PRESETS  # noqa: F401


def build_model(name, **overrides):
    """Build any preset by name (gpt2*, llama*)."""
    if name in GPT2_PRESETS:
        return build_gpt2(name, **overrides)
    if name in LLAMA_PRESETS:
        return build_llama(name, **overrides)
    raise KeyError(f"unknown model preset {name!r}; known: {sorted(GPT2_PRESETS) + sorted(LLAMA_PRESETS)}")
