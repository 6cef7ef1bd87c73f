"""GELU(+bias) and SwiGLU autograd wrappers over csrc/activations.hip, the fused MLP tail
linear(gelu(a + b_fc)) whose backward is one GEMM (EPI_GELU_BWD), and the fully fused GPT-2
MLP (``mlp_hip``): bias + GELU in the fc GEMM's epilogue, GELU' + the fc-bias gradient in
the projection's input-gradient GEMM (csrc/gemm16.hip) -- no separate GELU pass either way."""
from __future__ import annotations

import os

import torch

from ._ext import C
from .gemm import EPI_BIAS_GELU, linear_dgrad, linear_fwd, wgrad, wgrad_into
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


# ORION_FUSED_MLP (default on since round 3): the GPT-2 MLP as GEMMs with fused epilogues
# (_FusedMLP below; also routes gelu_linear through _GeluLinear).  On the 16x16x32-MFMA kernel
# (csrc/gemm16.hip) the fused forward runs 0.41 ms per layer in the step against 0.39 for
# hipBLASLt + the bias_gelu pass, the fused backward 0.48 against 0.48 -- a wash per layer,
# but with the in-tree input gradients the whole step gains 0.4 % (three alternating runs,
# profiles/ab/ab_gemm_auto_fusedmlp_r03e.log) and two (M, 4C) HBM passes per layer are gone.
# Round 2's 32x32x16 kernel lost (978k vs 990k tok/s): its fused epilogue cost more.
_FUSED_MLP = os.environ.get("ORION_FUSED_MLP", "1") != "0"


def fused_mlp_ok(a, weight) -> bool:
    """The fused tail needs bf16 operands the in-tree GEMM takes: a (..., F) contiguous,
    weight (C, F) contiguous with C % 64 == 0 (the reduction dim of the input gradient)."""
    from .gemm import gemm16_addressable
    return (_FUSED_MLP and a.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and a.is_contiguous() and weight.is_contiguous() and weight.shape[0] % 64 == 0
            and weight.shape[1] % 8 == 0 and a.data_ptr() % 16 == 0
            and weight.data_ptr() % 16 == 0
            and gemm16_addressable(weight.shape[0], weight.shape[0], weight.shape[1], True)
            and gemm16_addressable(weight.shape[1], weight.shape[1], weight.shape[0], False))


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


# ORION_FUSED_MLP=1 (see _FusedMLP): the GPT-2 MLP with both GELU passes inside GEMM epilogues
def mlp_ok(x, w_fc, w_proj) -> bool:
    C_ = x.shape[-1]
    return (_FUSED_MLP and x.dtype == torch.bfloat16 and w_fc.dtype == torch.bfloat16
            and w_proj.dtype == torch.bfloat16 and x.is_contiguous() and w_fc.is_contiguous()
            and w_proj.is_contiguous() and C_ % 64 == 0 and w_fc.shape[0] % 64 == 0
            and w_fc.shape[0] % 8 == 0 and w_proj.shape[0] % 8 == 0
            and x.data_ptr() % 16 == 0 and w_fc.data_ptr() % 16 == 0 and w_proj.data_ptr() % 16 == 0)


class _FusedMLP(torch.autograd.Function):
    """y = gelu(x W_fc^T + b_fc) W_proj^T (+ b_proj), GPT-2's MLP (GELU-tanh
    fused with the bias add), as GEMMs only:

    forward   (a, h) = one in-tree GEMM x W_fc^T whose epilogue adds b_fc and writes both the
              pre-activation a and h = gelu(a) (EPI_BIAS_GELU); y = h W_proj^T;
    backward  (da, db_fc) = one in-tree GEMM dy W_proj whose epilogue multiplies by GELU'(a)
              and emits the column sums of da (EPI_GELU_BWD); dW_proj = dy^T h,
              dx = da W_fc, dW_fc = da^T x (weight gradients straight into the arena).

    Against the unfused bias_gelu -> linear pair this drops two (M, 4C) HBM passes per layer
    (the GELU forward and backward kernels) and the separate fc-bias column sum."""

    @staticmethod
    def forward(ctx, x, w_fc, b_fc, w_proj, b_proj):
        C_ = x.shape[-1]
        x2 = x.reshape(-1, C_)
        a, h, ctx.deriv = mlp_fc_forward(x2, w_fc, b_fc)
        y = linear_fwd(h, w_proj, b_proj)
        ctx.save_for_backward(x2, a, h, w_fc, w_proj)
        ctx.biases = (b_fc, b_proj)
        ctx.sinks = (sink_of(w_fc), sink_of(w_proj))
        ctx.x_shape = x.shape
        return y.view(*x.shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, a, h, w_fc, w_proj = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        grads = mlp_backward(dy2, x2, a, h, w_fc, w_proj, ctx.biases, ctx.sinks, ctx.deriv,
                             ctx.needs_input_grad, proj_bias_grad=True)
        grads[0] = None if grads[0] is None else grads[0].view(ctx.x_shape)
        return tuple(grads)


def mlp_fc_forward(x2, w_fc, b_fc):
    """(a, h, deriv) of the fused MLP's first GEMM: h = gelu(x W_fc^T + b_fc) and a = the
    pre-activation, or GELU'(pre-activation) when ``deriv`` (_GELU_DERIV)."""
    bb = None if b_fc is None else b_fc.to(torch.bfloat16)
    if bb is None:
        a = linear_fwd(x2, w_fc)
        return a, C().bias_gelu_fwd(a, None).view(a.shape), False
    if _GELU_DERIV:  # a = GELU'(x W_fc^T + b_fc): the backward epilogue only multiplies
        a, h = C().gemm(x2, w_fc, False, EPI_BIAS_GELU | GEMM_DERIV, bb, None)
        return a, h, True
    a, h = C().gemm(x2, w_fc, False, EPI_BIAS_GELU, bb, None)
    return a, h, False


def mlp_backward(dy2, x2, a, h, w_fc, w_proj, biases, sinks, deriv, needs, proj_bias_grad=True):
    """Gradients [dx2, dW_fc, db_fc, dW_proj, db_proj] of the fused MLP from dy2 = d(output)
    (rows, C): one in-tree GEMM dy W_proj with GELU' and the fc-bias column sums in its
    epilogue, then the weight gradients (straight into the arena through ``sinks``) and the fc
    input gradient in the _MLP_BWD_ORDER order.  ``needs`` = needs_input_grad of (x, w_fc,
    b_fc, w_proj, b_proj); without ``proj_bias_grad`` the caller owns db_proj."""
    b_fc, b_proj = biases
    s_fc, s_proj = sinks
    sbfc, sbproj = _claim((b_fc, b_proj if proj_bias_grad else None))
    # a already holds the fc bias: GELU'(a), no bias operand (or a IS the derivative)
    da, dbfc = C().gemm_gelu_bwd(dy2, w_proj, a, None, _view(sbfc), deriv)
    _notify(sbfc)
    dbfc = None if b_fc is None else _unless(dbfc, sbfc)
    grads = [None, None, None, None, None]

    def proj_grads():
        if needs[3]:
            if s_proj is not None:
                wgrad_into(dy2, h, s_proj.view, s_proj.take())
                s_proj.notify()
            else:
                grads[3] = wgrad(dy2, h)
        if proj_bias_grad and b_proj is not None and needs[4]:
            db = C().colsum(dy2, _view(sbproj))
            grads[4] = None if sbproj is not None else db.to(b_proj.dtype)
            _notify(sbproj)

    def fc_dgrad():
        if needs[0]:
            grads[0] = linear_dgrad(da, w_fc)

    def fc_wgrad():
        if needs[1]:
            if s_fc is not None:
                wgrad_into(da, x2, s_fc.view, s_fc.take())
                s_fc.notify()
            else:
                grads[1] = wgrad(da, x2)
    for step in {"0": (proj_grads, fc_dgrad, fc_wgrad), "1": (fc_dgrad, fc_wgrad, proj_grads),
                 "2": (fc_wgrad, fc_dgrad, proj_grads)}[_MLP_BWD_ORDER]:
        step()
    if dbfc is not None:
        grads[2] = dbfc.to(b_fc.dtype)
    return grads


# ORION_GELU_DERIV=1 (default, round 5): the fused MLP's forward epilogue stores GELU'(a) in
# place of the pre-activation a (one sigmoid for gelu and GELU'), so the backward epilogue
# multiplies instead of evaluating GELU' (exp + rcp per element) in the store-bound GEMM.
_GELU_DERIV = os.environ.get("ORION_GELU_DERIV", "1") == "1"
GEMM_DERIV = 0x100


# Order of the MLP backward's GEMMs after the fused GELU' one: 1 (default) = the fc input and
# weight gradients first -- the two readers of da (403 MB at GPT-2's shape) back to back, while
# it is still in the caches -- and the fc2 weight gradient / bias last; 0 = fc2 first (round 3);
# 2 = fc weight gradient, fc input gradient, fc2.  GPT-2 step: 1 vs 0 +0.2 % (3 of 3), 2 vs 0
# mixed (profiles/ab/mlp_bwd_order_r04.log).
_MLP_BWD_ORDER = os.environ.get("ORION_MLP_BWD_ORDER", "1")


def mlp_hip(x, w_fc, b_fc, w_proj, b_proj=None):
    return _FusedMLP.apply(x, w_fc, b_fc, w_proj, b_proj)


# ORION_FUSED_SWIGLU=1 (default): Llama's feed-forward with the SwiGLU backward inside the
# down_proj input-gradient GEMM's epilogue (csrc/gemm16.hip EPI_SWIGLU_BWD): per layer the
# (M, F) gradient of the SwiGLU output is never written and re-read, and the separate
# swiglu_bwd pass over (M, 2F) is gone.
_FUSED_SWIGLU = os.environ.get("ORION_FUSED_SWIGLU", "1") != "0"


# Llama feed-forward backward order after the fused SwiGLU' GEMM, as _MLP_BWD_ORDER: here order
# 1 measured neutral (dgu is 721 MB, larger than the caches: profiles/ab/mlp_bwd_order_r04.log),
# so the default stays 0
_SWIGLU_BWD_ORDER = os.environ.get("ORION_SWIGLU_BWD_ORDER", "0")

# ORION_SWIGLU_FWD=gemm (default): the gate_up projection runs on gemm16 with the SwiGLU forward
# in its epilogue (csrc/gemm16.hip EPI_SWIGLU; needs F % 128 == 0): one kernel writes gu and
# h, the separate swiglu_fwd pass over (M, 2F) is gone.  =pass: hipBLASLt
# gate_up + the swiglu_fwd pass.
_SWIGLU_FWD = os.environ.get("ORION_SWIGLU_FWD", "gemm")


def swiglu_mlp_ok(x, w_gu, w_down) -> bool:
    from .gemm import gemm16_addressable
    C_, F2 = x.shape[-1], w_gu.shape[0]
    F_ = F2 // 2
    return (_FUSED_SWIGLU and x.dtype == torch.bfloat16 and w_gu.dtype == torch.bfloat16
            and w_down.dtype == torch.bfloat16 and x.is_contiguous() and w_gu.is_contiguous()
            and w_down.is_contiguous() and F2 % 2 == 0 and w_down.shape == (C_, F_)
            and C_ % 64 == 0 and F_ % 8 == 0 and x.data_ptr() % 16 == 0
            and w_gu.data_ptr() % 16 == 0 and w_down.data_ptr() % 16 == 0
            and gemm16_addressable(C_, C_, F_, True) and gemm16_addressable(2 * F_, 2 * F_, F_, False))


class _SwigluMLP(torch.autograd.Function):
    """y = (silu(x W_g^T) * (x W_u^T)) W_down^T with W_gu = [W_g; W_u] packed, Llama's
    feed-forward.

    forward   (gu, h) = ONE in-tree GEMM x W_gu^T with h = silu(gate) * up in its epilogue
              (_SWIGLU_FWD; else hipBLASLt + the swiglu pass), y = h W_down^T;
    backward  dgu = ONE in-tree GEMM dy W_down whose epilogue reads gate / up from gu and
              writes dgate = dh up silu'(gate), dup = dh silu(gate) straight into the packed
              (M, 2F) gradient; dW_down = dy^T h, dx = dgu W_gu, dW_gu = dgu^T x (weight
              gradients straight into the arena)."""

    @staticmethod
    def forward(ctx, x, w_gu, w_down):
        C_ = x.shape[-1]
        x2 = x.reshape(-1, C_)
        gu, h = swiglu_forward(x2, w_gu)
        y = linear_fwd(h, w_down)
        ctx.save_for_backward(x2, gu, h, w_gu, w_down)
        ctx.sinks = (sink_of(w_gu), sink_of(w_down))
        ctx.x_shape = x.shape
        return y.view(*x.shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, gu, h, w_gu, w_down = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        grads = swiglu_backward(dy2, x2, gu, h, w_gu, w_down, ctx.sinks, ctx.needs_input_grad)
        grads[0] = None if grads[0] is None else grads[0].view(ctx.x_shape)
        return tuple(grads)


def swiglu_forward(x2, w_gu):
    """(gu, h) of Llama's feed-forward input side: gu = x W_gu^T, h = silu(gate) * up."""
    if _SWIGLU_FWD == "gemm" and w_gu.shape[0] % 256 == 0 and w_gu.numel() * 2 < 0xFFFFFF00:
        return tuple(C().gemm_swiglu(x2, w_gu))
    gu = linear_fwd(x2, w_gu)
    return gu, C().swiglu_fwd(gu)


def swiglu_backward(dy2, x2, gu, h, w_gu, w_down, sinks, needs):
    """Gradients [dx2, dW_gu, dW_down] of the feed-forward from dy2 = d(output): ONE in-tree GEMM
    dy W_down whose epilogue applies SwiGLU' (EPI_SWIGLU_BWD), then the weight gradients
    (through ``sinks``) and the input gradient in the _SWIGLU_BWD_ORDER order."""
    s_gu, s_down = sinks
    dgu = C().gemm_swiglu_bwd(dy2, w_down, gu)
    grads = [None, None, None]

    def down_wgrad():
        if needs[2]:
            if s_down is not None:
                wgrad_into(dy2, h, s_down.view, s_down.take())
                s_down.notify()
            else:
                grads[2] = wgrad(dy2, h)

    def gu_dgrad():
        if needs[0]:
            grads[0] = linear_dgrad(dgu, w_gu)

    def gu_wgrad():
        if needs[1]:
            if s_gu is not None:
                wgrad_into(dgu, x2, s_gu.view, s_gu.take())
                s_gu.notify()
            else:
                grads[1] = wgrad(dgu, x2)
    # the same orders as _FusedMLP (_SWIGLU_BWD_ORDER)
    for step in {"0": (down_wgrad, gu_dgrad, gu_wgrad), "1": (gu_dgrad, gu_wgrad, down_wgrad),
                 "2": (gu_wgrad, gu_dgrad, down_wgrad)}[_SWIGLU_BWD_ORDER]:
        step()
    return grads


def swiglu_mlp_hip(x, w_gu, w_down):
    return _SwigluMLP.apply(x, w_gu, w_down)
