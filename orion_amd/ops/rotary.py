"""Rotary embedding autograd wrapper over csrc/rmsnorm_rope.hip (rotate-half form)."""
from __future__ import annotations

import torch

from ._ext import C


class _Rope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, pos0):
        ctx.save_for_backward(cos, sin)
        ctx.pos0 = int(pos0)
        return C().rope(x, cos, sin, int(pos0), 1.0)

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        return C().rope(dy.contiguous(), cos, sin, ctx.pos0, -1.0), None, None, None


def rope_hip(x, cos, sin, pos0=0):
    """x: (B, T, H, D) view with unit stride on D -> contiguous rotated copy."""
    return _Rope.apply(x, cos, sin, pos0)
