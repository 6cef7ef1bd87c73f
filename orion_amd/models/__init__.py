"""Decoder-only transformer models built on :mod:`orion_amd.ops`."""
from .gpt2 import GPT, GPTConfig, build_gpt2, PRESETS as GPT2_PRESETS  # noqa: F401
