"""LayerNorm / RMSNorm autograd wrappers over the HIP kernels (csrc/layernorm.hip,
csrc/rmsnorm_rope.hip).  Weights may be fp32 (eval/inference) or bf16 (arena);
kernels always see bf16 and gradients are returned in the weight's dtype."""
from __future__ import annotations

import torch

from ._ext import C
from .gemm import WGRAD_FIRST, linear_dgrad, linear_fwd, wgrad, wgrad_into
from .grad_sink import claim, sink_of


def _bf16(t):
    return t if t is None or t.dtype == torch.bfloat16 else t.to(torch.bfloat16)


# small gradients (norm weights, biases) go straight into their gradient-arena slices: the
# reduction kernel's output IS the slice, so no AccumulateGrad add runs (ops/grad_sink.py)
def _claim(params):
    return tuple(claim(p) if p is not None and p.dtype == torch.bfloat16 else None
                 for p in params)


def _view(sink):
    return None if sink is None else sink.view


def _notify(*sinks):
    for sk in sinks:
        if sk is not None:
            sk.notify()


def _unless(g, sink):
    # a gradient written through its sink must not also reach AccumulateGrad (the op may
    # hand back the slice it wrote; ``p.grad += p.grad`` would double it)
    return None if sink is not None else g


def _grad(g, dtype):
    return None if g is None else g.to(dtype)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        xb = _bf16(x)
        y, mean, rstd = C().layernorm_fwd(xb, _bf16(w), _bf16(b), float(eps))
        ctx.save_for_backward(xb, w, mean, rstd)
        ctx.has_bias = b is not None
        ctx.b_dtype = None if b is None else b.dtype
        ctx.x_dtype = x.dtype
        ctx.params = (w, b)
        return y.view(x.shape).to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        xb, w, mean, rstd = ctx.saved_tensors
        sw, sb = _claim(ctx.params)
        dx, dw, db, _ = C().layernorm_bwd(_bf16(dy.contiguous()), xb, _bf16(w), mean, rstd,
                                          ctx.has_bias, None, False, _view(sw), _view(sb))
        _notify(sw, sb)
        dw, db = _unless(dw, sw), _unless(db, sb)
        dx = dx.view(xb.shape).to(ctx.x_dtype)
        return dx, _grad(dw, w.dtype), (_grad(db, ctx.b_dtype) if ctx.has_bias else None), None


def layer_norm_hip(x, weight, bias, eps=1e-5):
    return _LayerNorm.apply(x, weight, bias, eps)


class _AddLayerNorm(torch.autograd.Function):
    """(s, y) = (x + (r + rb), LayerNorm(s)).  ``rb`` is the bias of the branch's output
    projection (added here instead of in the GEMM epilogue).  Backward folds the
    residual-stream gradient ds into the LayerNorm input gradient and produces the
    branch-bias gradient colsum(ds_total) in the same kernel."""

    @staticmethod
    def forward(ctx, x, r, w, b, rb, eps):
        s, y, mean, rstd = C().add_layernorm_fwd(x, r, _bf16(w), _bf16(b), float(eps), _bf16(rb))
        # an unused output (the last block's residual sum) arrives as None, not as a
        # materialised zero tensor (a 100 MB fill + read per step on GPT-2)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(s, w, mean, rstd)
        ctx.has_bias = b is not None
        ctx.b_dtype = None if b is None else b.dtype
        ctx.rb_dtype = None if rb is None else rb.dtype
        ctx.params = (w, b, rb)
        return s.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, ds, dy):
        s, w, mean, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(s)
        dres = None if ds is None else ds.contiguous()
        want_rb = ctx.rb_dtype is not None
        sw, sb, srb = _claim(ctx.params)
        dx, dw, db, drb = C().layernorm_bwd(dy.contiguous(), s, _bf16(w), mean, rstd,
                                            ctx.has_bias, dres, want_rb, _view(sw), _view(sb),
                                            _view(srb))
        _notify(sw, sb, srb)
        dw, db, drb = _unless(dw, sw), _unless(db, sb), _unless(drb, srb)
        dx = dx.view(s.shape)
        return (dx, dx, _grad(dw, w.dtype), (_grad(db, ctx.b_dtype) if ctx.has_bias else None),
                (_grad(drb, ctx.rb_dtype) if want_rb else None), None)


def add_layer_norm_hip(x, r, weight, bias, eps=1e-5, r_bias=None):
    return _AddLayerNorm.apply(x, r, weight, bias, r_bias, eps)


def linear_input_weight_grads(dy2, x, w, sink, need_dx, need_dw):
    """dx = dy W and dW = dy^T x of y = x W^T (dy2: (rows, N)), in the configured order
    (ops.gemm.WGRAD_FIRST); dW goes straight into the gradient arena through ``sink`` when
    there is one (then None is returned for it)."""
    dx = dw = None
    if need_dx and not WGRAD_FIRST:
        dx = linear_dgrad(dy2, w).view(x.shape)
    if need_dw:
        if sink is not None:
            wgrad_into(dy2, x.reshape(-1, x.shape[-1]), sink.view, sink.take())
            sink.notify()
        else:
            dw = wgrad(dy2, x.reshape(-1, x.shape[-1]))
    if need_dx and WGRAD_FIRST:
        dx = linear_dgrad(dy2, w).view(x.shape)
    return dx, dw


class _Linear(torch.autograd.Function):
    """y = x W^T + b on hipBLASLt (or csrc/gemm.hip: ops/gemm.py); backward computes the
    bias gradient with the deterministic two-stage column-sum kernel instead of a generic
    reduction."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.sink = sink_of(w)  # dW straight into the gradient arena (ops/grad_sink.py)
        ctx.bias = b
        return linear_fwd(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        db = None
        bias_grad = ctx.has_bias and ctx.needs_input_grad[2]
        if bias_grad and WGRAD_FIRST:  # dY was just written by the previous kernel: sum it now
            db = _Linear._bias_grad(ctx, dy2)
        dx, dw = linear_input_weight_grads(dy2, x, w, ctx.sink, ctx.needs_input_grad[0],
                                           ctx.needs_input_grad[1])
        if bias_grad and not WGRAD_FIRST:
            db = _Linear._bias_grad(ctx, dy2)
        return dx, dw, db

    @staticmethod
    def _bias_grad(ctx, dy2):
        (sb,) = _claim((ctx.bias,))
        db = C().colsum(dy2.contiguous(), _view(sb))
        if sb is not None:  # written into the arena; never hand the slice back to autograd
            db = None
        _notify(sb)
        return db


def linear_hip(x, weight, bias=None):
    return _Linear.apply(x, weight, bias)


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        xb = _bf16(x)
        y, rstd = C().rmsnorm_fwd(xb, _bf16(w), float(eps))
        ctx.save_for_backward(xb, w, rstd)
        ctx.x_dtype = x.dtype
        ctx.params = (w,)
        return y.view(x.shape).to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        xb, w, rstd = ctx.saved_tensors
        (sw,) = _claim(ctx.params)  # dw straight into the gradient arena (ops/grad_sink.py)
        dx, dw = C().rmsnorm_bwd(_bf16(dy.contiguous()), xb, _bf16(w), rstd, None, _view(sw))
        _notify(sw)
        return dx.view(xb.shape).to(ctx.x_dtype), _grad(_unless(dw, sw), w.dtype), None


def rms_norm_hip(x, weight, eps=1e-5):
    return _RMSNorm.apply(x, weight, eps)


class _AddRMSNorm(torch.autograd.Function):
    """(s, y) = (x + r, RMSNorm(x + r)) with the residual gradient folded into backward."""

    @staticmethod
    def forward(ctx, x, r, w, eps):
        s, y, rstd = C().add_rmsnorm_fwd(x, r, _bf16(w), float(eps))
        ctx.set_materialize_grads(False)  # see _AddLayerNorm
        ctx.save_for_backward(s, w, rstd)
        ctx.params = (w,)
        return s.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, ds, dy):
        s, w, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(s)
        dres = None if ds is None else ds.contiguous()
        (sw,) = _claim(ctx.params)
        dx, dw = C().rmsnorm_bwd(dy.contiguous(), s, _bf16(w), rstd, dres, _view(sw))
        _notify(sw)
        dx = dx.view(s.shape)
        return dx, dx, _grad(_unless(dw, sw), w.dtype), None


def add_rms_norm_hip(x, r, weight, eps=1e-5):
    return _AddRMSNorm.apply(x, r, weight, eps)
