"""GPT-2 residual sites with the branch's output projection doing the residual add (round 6).

Every block has two sites "x = x + branch(h) W^T + b; h = LayerNorm(x)".  The round-2..5 form
ran the projection as a plain GEMM (output o) and folded the add, the projection bias and the
LayerNorm into one kernel that read x and o and wrote x' and h -- 500 MB of HBM traffic per
site at the 124M bench shape.  Here ONE hipBLASLt GEMM writes x' = h_in W^T + b + x (the bias
and the old stream in its epilogue: csrc/blaslt.cpp, ``C().linear_residual``) and the LayerNorm
reads only x': 400 MB, and the projection runs on the wrapper's per-shape measured-fastest
hipBLASLt solution (``scripts/probe_residual_gemm.py``: attn c_proj site 156 -> 131 us, mlp
c_proj site 355 -> 290 us).

Each site is ONE autograd node (forward GEMM + LayerNorm, backward LayerNorm + the branch's
gradients), so the residual-stream gradient still enters the LayerNorm backward kernel (dres)
instead of being summed by autograd, and the branch-bias gradient is still that kernel's
column sum of the total stream gradient:

* ``linear_residual_layer_norm``: the attention site (the branch input is the attention output,
  the projection is c_proj);
* ``mlp_residual_layer_norm``: the MLP site -- the whole fused MLP (fc + bias + GELU epilogue,
  GELU' in the fc2 input-gradient epilogue: ops/activations.py) with fc2 as the residual GEMM.

Reference semantics: nanoGPT's Block (``x = x + attn(ln_1(x)); x = x + mlp(ln_2(x))``).
"""
from __future__ import annotations

import os

import torch

from ._ext import C
from .activations import (mlp_backward, mlp_fc_forward, mlp_ok, swiglu_backward, swiglu_forward,
                          swiglu_mlp_ok)
from .determinism import deterministic
from .grad_sink import sink_of
from .layernorm import _bf16, _claim, _grad, _notify, _unless, _view, linear_input_weight_grads

# ORION_RESID_GEMM=0: the projection as a plain GEMM + the fused add + LayerNorm kernel (A/B);
# =attn: only the attention site
_MODE = os.environ.get("ORION_RESID_GEMM", "1")
_RESID_GEMM = _MODE != "0"
_RESID_MLP = _MODE not in ("0", "attn")


def eligible(x, inp, w, rb, need_bias=True) -> bool:
    if rb is None and need_bias:
        return False
    return (_RESID_GEMM and not deterministic() and x.is_cuda
            and x.dtype == inp.dtype == w.dtype == torch.bfloat16 and x.is_contiguous()
            and inp.is_contiguous() and w.is_contiguous()
            and (rb is None or (rb.dtype == torch.bfloat16 and rb.is_contiguous())))


_CHECKED = set()


def _residual_gemm(inp2, w, rb, x2):
    """C().linear_residual; the first call per shape (when the wrapper picks its hipBLASLt
    solution by timing) is checked against the torch composition, so a solution that accepted
    the problem but computed something else fails loudly instead of training on it."""
    s2 = C().linear_residual(inp2, w, rb, x2)
    key = (inp2.device, tuple(inp2.shape), tuple(w.shape), rb is None)
    if key not in _CHECKED and not torch.cuda.is_current_stream_capturing():
        ref = inp2.float() @ w.float().t() + x2.float()
        if rb is not None:
            ref += rb.float()
        err = ((s2.float() - ref).norm() / ref.norm().clamp_min(1e-30)).item()
        if not err < 1e-2:
            raise RuntimeError(f"linear_residual {tuple(inp2.shape)} x {tuple(w.shape)}: relative error {err:.3g}")
        _CHECKED.add(key)
    return s2


def _ln_forward(ctx, s2, ln_w, ln_b, eps):
    y, mean, rstd = C().layernorm_fwd(s2, _bf16(ln_w), _bf16(ln_b), float(eps))
    ctx.ln = (mean, rstd)
    ctx.has_ln_bias = ln_b is not None
    ctx.ln_b_dtype = None if ln_b is None else ln_b.dtype
    return y


def _ln_backward(ctx, s2, ln_w, ln_b, rb, ds, dy):
    """LayerNorm backward of y = LN(s) plus the stream gradient ds arriving from later sites:
    returns (dsum = d(s) total, dW_ln, db_ln, d rb) with rb's gradient = colsum(dsum)."""
    mean, rstd = ctx.ln
    if dy is None:
        dy = torch.zeros_like(s2)
    dres = None if ds is None else ds.reshape(s2.shape).contiguous()
    sw, sb, srb = _claim((ln_w, ln_b, rb))
    dsum, dw, db, drb = C().layernorm_bwd(dy.reshape(s2.shape).contiguous(), s2, _bf16(ln_w), mean, rstd,
                                          ctx.has_ln_bias, dres, True, _view(sw), _view(sb), _view(srb))
    _notify(sw, sb, srb)
    dw, db, drb = _unless(dw, sw), _unless(db, sb), _unless(drb, srb)
    return (dsum, _grad(dw, ln_w.dtype), (_grad(db, ctx.ln_b_dtype) if ctx.has_ln_bias else None),
            _grad(drb, rb.dtype))


class _LinearResidualLN(torch.autograd.Function):
    """(s, y) = (x + inp W^T + rb, LayerNorm(s))."""

    @staticmethod
    def forward(ctx, x, inp, w, rb, ln_w, ln_b, eps):
        C_ = x.shape[-1]
        inp2 = inp.reshape(-1, inp.shape[-1])
        s2 = _residual_gemm(inp2, w, rb, x.reshape(-1, C_))
        y = _ln_forward(ctx, s2, ln_w, ln_b, eps)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(s2, inp2, w, ln_w)
        ctx.params = (ln_b, rb)
        ctx.sink = sink_of(w)
        ctx.inp_shape = inp.shape
        return s2.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, ds, dy):
        s2, inp2, w, ln_w = ctx.saved_tensors
        ln_b, rb = ctx.params
        dsum, dlw, dlb, drb = _ln_backward(ctx, s2, ln_w, ln_b, rb, ds, dy)
        dinp, dw = linear_input_weight_grads(dsum, inp2, w, ctx.sink, ctx.needs_input_grad[1],
                                             ctx.needs_input_grad[2])
        dx = dsum.view(ctx.inp_shape[:-1] + (s2.shape[-1],)) if ctx.needs_input_grad[0] else None
        dinp = None if dinp is None else dinp.view(ctx.inp_shape)
        return dx, dinp, dw, drb, dlw, dlb, None


class _MLPResidualLN(torch.autograd.Function):
    """(s, y) = (x + gelu(h W_fc^T + b_fc) W_proj^T + b_proj, LayerNorm(s))."""

    @staticmethod
    def forward(ctx, x, h, w_fc, b_fc, w_proj, b_proj, ln_w, ln_b, eps):
        C_ = x.shape[-1]
        h2 = h.reshape(-1, C_)
        a, g, ctx.deriv = mlp_fc_forward(h2, w_fc, b_fc)
        s2 = _residual_gemm(g, w_proj, b_proj, x.reshape(-1, C_))
        y = _ln_forward(ctx, s2, ln_w, ln_b, eps)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(s2, h2, a, g, w_fc, w_proj, ln_w)
        ctx.params = (ln_b, b_fc, b_proj)
        ctx.sinks = (sink_of(w_fc), sink_of(w_proj))
        ctx.x_shape = x.shape
        return s2.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, ds, dy):
        s2, h2, a, g, w_fc, w_proj, ln_w = ctx.saved_tensors
        ln_b, b_fc, b_proj = ctx.params
        dsum, dlw, dlb, dbp = _ln_backward(ctx, s2, ln_w, ln_b, b_proj, ds, dy)
        n = ctx.needs_input_grad
        # mlp_backward's needs: (input h, w_fc, b_fc, w_proj, b_proj -- owned by the LayerNorm)
        dh, dwfc, dbfc, dwp, _ = mlp_backward(dsum, h2, a, g, w_fc, w_proj, (b_fc, b_proj), ctx.sinks,
                                              ctx.deriv, (n[1], n[2], n[3], n[4], False),
                                              proj_bias_grad=False)
        dx = dsum.view(ctx.x_shape) if n[0] else None
        dh = None if dh is None else dh.view(ctx.x_shape)
        return dx, dh, dwfc, dbfc, dwp, dbp, dlw, dlb, None


def linear_residual_layer_norm_hip(x, inp, w, rb, ln_w, ln_b, eps=1e-5):
    return _LinearResidualLN.apply(x, inp, w, rb, ln_w, ln_b, eps)


def mlp_residual_layer_norm_hip(x, h, w_fc, b_fc, w_proj, b_proj, ln_w, ln_b, eps=1e-5):
    return _MLPResidualLN.apply(x, h, w_fc, b_fc, w_proj, b_proj, ln_w, ln_b, eps)


def mlp_eligible(x, h, w_fc, w_proj, b_proj) -> bool:
    return _RESID_MLP and eligible(x, h, w_proj, b_proj) and mlp_ok(h, w_fc, w_proj)


# ---------------------------------------------------------------- Llama: RMSNorm sites (no biases)
def _rms_forward(ctx, s2, w, eps):
    y, rstd = C().rmsnorm_fwd(s2, _bf16(w), float(eps))
    ctx.rstd = rstd
    return y


def _rms_backward(ctx, s2, w, ds, dy):
    if dy is None:
        dy = torch.zeros_like(s2)
    dres = None if ds is None else ds.reshape(s2.shape).contiguous()
    (sw,) = _claim((w,))
    dsum, dw = C().rmsnorm_bwd(dy.reshape(s2.shape).contiguous(), s2, _bf16(w), ctx.rstd, dres, _view(sw))
    _notify(sw)
    return dsum, _grad(_unless(dw, sw), w.dtype)


class _LinearResidualRMS(torch.autograd.Function):
    """(s, y) = (x + inp W^T, RMSNorm(s)): Llama's attention site (o_proj)."""

    @staticmethod
    def forward(ctx, x, inp, w, nw, eps):
        C_ = x.shape[-1]
        inp2 = inp.reshape(-1, inp.shape[-1])
        s2 = _residual_gemm(inp2, w, None, x.reshape(-1, C_))
        y = _rms_forward(ctx, s2, nw, eps)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(s2, inp2, w, nw)
        ctx.sink = sink_of(w)
        ctx.inp_shape = inp.shape
        return s2.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, ds, dy):
        s2, inp2, w, nw = ctx.saved_tensors
        dsum, dnw = _rms_backward(ctx, s2, nw, ds, dy)
        dinp, dw = linear_input_weight_grads(dsum, inp2, w, ctx.sink, ctx.needs_input_grad[1],
                                             ctx.needs_input_grad[2])
        dx = dsum.view(ctx.inp_shape[:-1] + (s2.shape[-1],)) if ctx.needs_input_grad[0] else None
        dinp = None if dinp is None else dinp.view(ctx.inp_shape)
        return dx, dinp, dw, dnw, None


class _SwigluResidualRMS(torch.autograd.Function):
    """(s, y) = (x + swiglu(h W_gu^T) W_down^T, RMSNorm(s)): Llama's feed-forward site (the
    SwiGLU forward in the gate_up epilogue, SwiGLU' in the down_proj input-gradient epilogue:
    ops/activations.py; down_proj is the residual GEMM)."""

    @staticmethod
    def forward(ctx, x, h, w_gu, w_down, nw, eps):
        C_ = x.shape[-1]
        h2 = h.reshape(-1, C_)
        gu, g = swiglu_forward(h2, w_gu)
        s2 = _residual_gemm(g, w_down, None, x.reshape(-1, C_))
        y = _rms_forward(ctx, s2, nw, eps)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(s2, h2, gu, g, w_gu, w_down, nw)
        ctx.sinks = (sink_of(w_gu), sink_of(w_down))
        ctx.x_shape = x.shape
        return s2.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, ds, dy):
        s2, h2, gu, g, w_gu, w_down, nw = ctx.saved_tensors
        dsum, dnw = _rms_backward(ctx, s2, nw, ds, dy)
        n = ctx.needs_input_grad
        dh, dwgu, dwd = swiglu_backward(dsum, h2, gu, g, w_gu, w_down, ctx.sinks, (n[1], n[2], n[3]))
        dx = dsum.view(ctx.x_shape) if n[0] else None
        dh = None if dh is None else dh.view(ctx.x_shape)
        return dx, dh, dwgu, dwd, dnw, None


def linear_residual_rms_norm_hip(x, inp, w, nw, eps=1e-5):
    return _LinearResidualRMS.apply(x, inp, w, nw, eps)


def swiglu_residual_rms_norm_hip(x, h, w_gu, w_down, nw, eps=1e-5):
    return _SwigluResidualRMS.apply(x, h, w_gu, w_down, nw, eps)


def swiglu_eligible(x, h, w_gu, w_down) -> bool:
    return _RESID_MLP and eligible(x, h, w_down, None, need_bias=False) and swiglu_mlp_ok(h, w_gu, w_down)
