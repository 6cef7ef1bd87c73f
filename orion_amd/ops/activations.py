"""GELU(+bias) and SwiGLU autograd wrappers over csrc/activations.hip."""
from __future__ import annotations

import torch

from ._ext import C
from .layernorm import _claim, _notify, _unless, _view


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b):
        bb = None if b is None else b.to(x.dtype)
        y = C().bias_gelu_fwd(x, bb)
        ctx.save_for_backward(x, bb)
        ctx.b_dtype = None if b is None else b.dtype
        ctx.bias = b
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x, bb = ctx.saved_tensors
        (sb,) = _claim((ctx.bias,))
        dx, db = C().bias_gelu_bwd(dy.contiguous(), x, bb, _view(sb))
        _notify(sb)
        db = _unless(db, sb)
        return dx.view(x.shape), (None if db is None else db.to(ctx.b_dtype))


def bias_gelu_hip(x, bias):
    return _BiasGelu.apply(x, bias)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        y = C().swiglu_fwd(gu)
        ctx.save_for_backward(gu)
        return y

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        return C().swiglu_bwd(dy.contiguous(), gu).view(gu.shape)


def swiglu_hip(gate_up):
    """silu(gate) * up on a packed (..., 2F) [gate | up] projection -> (..., F)."""
    return _SwiGLU.apply(gate_up)
