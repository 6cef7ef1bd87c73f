"""Bitwise-reproducible training steps: ``ORION_DETERMINISTIC=1`` or
``torch.use_deterministic_algorithms(True)``.

What it switches (everything else is deterministic by construction -- fixed-order
reductions in the LayerNorm / column-sum / slab-sum / cross-entropy / AdamW kernels):

* attention backward -> the split dK/dV + dQ kernels (no fp32 atomics), also the default;
* linear-layer forward / input-gradient GEMMs -> csrc/gemm.hip (one workgroup per output
  tile, no split-K), instead of hipBLASLt, whose stream-K solutions may combine partial tiles
  in run-dependent order.
"""
from __future__ import annotations

import os

import torch


def deterministic() -> bool:
    return os.environ.get("ORION_DETERMINISTIC") == "1" or torch.are_deterministic_algorithms_enabled()
