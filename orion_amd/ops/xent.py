"""Fused softmax-cross-entropy wrappers over csrc/xent.hip.

``linear_cross_entropy`` fuses the LM head: logits = x W^T (hipBLASLt GEMM),
then one kernel computes the loss AND writes dlogits over the logits buffer,
so backward is two GEMMs on the saved dlogits with the upstream gradient
applied to the small (N, C) / (V, C) results.
"""
from __future__ import annotations

import torch

from ._ext import C
from .gemm import WGRAD_FIRST, linear_dgrad, linear_fwd, wgrad, wgrad_into
from .grad_sink import sink_of

import os

# LM head: weight gradient before the input gradient, so dX (read next by the final LayerNorm's
# backward) is not evicted by the weight gradient's 6.6 GB pass over the logit gradient (A/B;
# defaults to the global ORION_WGRAD_FIRST order)
_LM_WGRAD_FIRST = os.environ.get("ORION_LMHEAD_WGRAD_FIRST", "1" if WGRAD_FIRST else "0") == "1"


class _LinearXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, targets, ignore_index):
        logits = linear_fwd(x, w)
        loss = C().xent_fwd_bwd(logits, targets.contiguous(), int(ignore_index))
        ctx.save_for_backward(x, w, logits)   # logits now hold dlogits / n_valid
        ctx.sink = sink_of(w)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, w, dl = ctx.saved_tensors
        s = g.detach().float().reshape(1).contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0] and not _LM_WGRAD_FIRST:
            dx = linear_dgrad(dl, w)
            C().scale_(dx, s)
        if ctx.needs_input_grad[1]:
            sink = ctx.sink
            if sink is not None:
                wgrad_into(dl, x, sink.view, sink.take(), s)
                sink.notify()
            else:
                dw = wgrad(dl, x, s)
        if ctx.needs_input_grad[0] and _LM_WGRAD_FIRST:
            dx = linear_dgrad(dl, w)
            C().scale_(dx, s)
        return dx, dw, None, None


def linear_cross_entropy_hip(x, w, targets, ignore_index=-1):
    """mean cross-entropy of softmax(x @ w^T) against targets; x (N, C), w (V, C)."""
    return _LinearXent.apply(x, w, targets, ignore_index)


class _Xent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, ignore_index):
        buf = logits.detach().contiguous().clone()
        loss = C().xent_fwd_bwd(buf, targets.contiguous(), int(ignore_index))
        ctx.save_for_backward(buf)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        out = dl.clone()
        C().scale_(out, g.detach().float().reshape(1).contiguous())
        return out, None, None


def fused_cross_entropy(logits, targets, ignore_index=-1):
    return _Xent.apply(logits, targets, ignore_index)
