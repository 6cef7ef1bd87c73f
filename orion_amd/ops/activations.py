"""GELU(+bias) and SwiGLU autograd wrappers over csrc/activations.hip, and the fused MLP tail
linear(gelu(a + b_fc)) whose backward is one GEMM (csrc/gemm_phased.hip, EPI_GELU_BWD)."""
from __future__ import annotations

import os

import torch

from ._ext import C
from .gemm import linear_fwd, wgrad, wgrad_into
from .grad_sink import sink_of
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


# ORION_FUSED_MLP=1 routes the GPT-2 MLP tail through _GeluLinear below.  Off by default: on
# MI355X the fused backward GEMM (65536 x 3072 x 768) runs 0.62 ms against 0.59 ms for hipBLASLt's
# dgrad plus the bias_gelu_bwd pass, and the whole GPT-2 step measured 978k vs 990k tok/s (3
# alternating runs each).  The phased kernel's epilogue runs after its MMAs on the same waves
# (one 160 KB-LDS workgroup per CU), so the (M, F) pre-activation read is not overlapped with
# matrix work: +205 us over the plain-store kernel (profiles/gemm_study/epilogue_cost.txt).
_FUSED_MLP = os.environ.get("ORION_FUSED_MLP", "0") != "0"


def fused_mlp_ok(a, weight) -> bool:
    """The fused tail needs bf16 operands the in-tree GEMM takes: a (..., F) contiguous,
    weight (C, F) contiguous with C % 64 == 0 (the reduction dim of the input gradient)."""
    return (_FUSED_MLP and a.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and a.is_contiguous() and weight.is_contiguous() and weight.shape[0] % 64 == 0
            and weight.shape[1] % 8 == 0 and a.data_ptr() % 16 == 0
            and weight.data_ptr() % 16 == 0)


class _GeluLinear(torch.autograd.Function):
    """y = gelu(a + b_fc) W^T + b.  Forward: the bias+GELU kernel, then hipBLASLt.  Backward:
    da = (dy W) * GELU'(a + b_fc) and db_fc = colsum(da) from ONE in-tree GEMM (the GELU
    derivative and the bias-gradient partial sums run in its epilogue), so the (M, F) input
    gradient of the GELU is never written and re-read; dW = dy^T h by the phased weight-
    gradient kernel.  Replaces the bias_gelu -> linear pair of the GPT-2 MLP (SURVEY.md
    section 3, kernel K4: GELU-tanh fused with the bias add)."""

    @staticmethod
    def forward(ctx, a, b_fc, w, b):
        bb = None if b_fc is None else b_fc.to(a.dtype)
        h = C().bias_gelu_fwd(a, bb).view(a.shape)
        ctx.save_for_backward(a, h, w, bb)
        ctx.fc_bias, ctx.bias = b_fc, b
        ctx.sink = sink_of(w)
        return linear_fwd(h, w, b)

    @staticmethod
    def backward(ctx, dy):
        a, h, w, bb = ctx.saved_tensors
        F_ = a.shape[-1]
        dy2 = dy.reshape(-1, dy.shape[-1])
        h2 = h.reshape(-1, F_)
        sfc, sb = _claim((ctx.fc_bias, ctx.bias))
        da, dbfc = C().gemm_gelu_bwd(dy2, w, a.reshape(-1, F_), bb, _view(sfc))
        _notify(sfc)
        dbfc = None if ctx.fc_bias is None else _unless(dbfc, sfc)
        dw = db = None
        if ctx.needs_input_grad[2]:
            if ctx.sink is not None:
                wgrad_into(dy2, h2, ctx.sink.view, ctx.sink.take())
                ctx.sink.notify()
            else:
                dw = wgrad(dy2, h2)
        if ctx.bias is not None and ctx.needs_input_grad[3]:
            db = C().colsum(dy2.contiguous(), _view(sb))
            if sb is not None:
                db = None
            _notify(sb)
        if dbfc is not None:
            dbfc = dbfc.to(ctx.fc_bias.dtype)
        if db is not None:
            db = db.to(ctx.bias.dtype)
        return da.view(a.shape), dbfc, dw, db


def gelu_linear_hip(a, b_fc, weight, bias=None):
    return _GeluLinear.apply(a, b_fc, weight, bias)
