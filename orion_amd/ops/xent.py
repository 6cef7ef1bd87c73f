"""Fused softmax-cross-entropy wrappers.

``linear_cross_entropy`` fuses the LM head.  Default (``ORION_LMHEAD=exp``,
csrc/lmhead.hip): the in-tree forward GEMM writes E = exp(logits - ref) with
per-row partial sums and the target logits from its epilogue, a fold over the
partials gives the loss and folds the one-hot term into E, and the backward is
dX = s (E W) (row scale in the GEMM epilogue) and dW = E^T (s X) -- no pass over
the (tokens x vocab) buffer besides the three GEMMs.  ``ORION_LMHEAD=rowpass``:
round 4's form, logits = x W^T (hipBLASLt) then one kernel (csrc/xent.hip)
computes the loss and writes dlogits over the logits buffer.
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
        check_targets(targets, w.shape[0], int(ignore_index))
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
    if lmhead_exp_eligible(x, w):
        return _LinearXentExp.apply(x, w, targets, ignore_index)
    return _LinearXent.apply(x, w, targets, ignore_index)


_TGT_CHECK_ALWAYS = os.environ.get("ORION_CHECK_IDS") == "1"
_tgt_checked: set = set()


def check_targets(targets, V, ignore_index):
    """Raise IndexError, as torch's cross_entropy does, when a target other than
    ``ignore_index`` lies outside [0, V).  Host check (one sync) on the first call per device,
    or on every call with ORION_CHECK_IDS=1; after that both kernels skip such a target (no
    loss, no gradient, not counted in n_valid) and raise the device flag read by
    ``ops.embedding.id_error``."""
    key = targets.device
    if key in _tgt_checked and not _TGT_CHECK_ALWAYS:
        return
    _tgt_checked.add(key)
    bad = (targets != ignore_index) & ((targets < 0) | (targets >= V))
    if bool(bad.any()):
        t = targets[bad][0].item()
        raise IndexError(f"Target {t} is out of bounds for {V} classes (ignore_index={ignore_index})")


_LMHEAD = os.environ.get("ORION_LMHEAD", "exp")
# the scaled activations of the LM-head weight gradient written transposed (C, N), so the
# weight gradient reads them as an NT operand (csrc/wgrad.hip, bt); ORION_LMHEAD_XT=0: (N, C)
_LM_XT = os.environ.get("ORION_LMHEAD_XT", "1") == "1"
_CREF = {}


def _cref(dev, w=None):
    """The running exp reference of the LM-head forward with weight ``w`` on ``dev`` (a device
    scalar the fold kernel updates: the largest row log-sum-exp of the previous call), one per
    weight tensor (keyed by its storage), so two models in one process -- a DDP trainer and its
    local reference, say -- do not feed each other's forwards.  Deterministic mode
    (ops/determinism.py) uses a fresh 0 every call instead: the bf16 rounding of exp(logit -
    ref) depends on the reference, so a carried-over one would make two identical runs in one
    process differ in the last bits (rows it does not suit take the exact fixup path).  Any
    value is correct: the reference only decides which rows need the fixup."""
    from .determinism import deterministic
    if deterministic():
        return torch.zeros(1, dtype=torch.float32, device=dev)
    key = (dev, w.data_ptr() if w is not None else 0)
    t = _CREF.get(key)
    if t is None:
        if len(_CREF) >= 64:  # freed weights' storages are reused: keep the table bounded
            _CREF.clear()
        t = _CREF[key] = torch.zeros(1, dtype=torch.float32, device=dev)
    return t


def lmhead_exp_eligible(x, w) -> bool:
    return (_LMHEAD == "exp" and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.dim() == 2 and x.stride(1) == 1 and w.is_contiguous() and x.shape[1] % 64 == 0
            and x.shape[1] <= 16384
            and w.shape[0] % 64 == 0 and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0
            and w.data_ptr() % 16 == 0 and x.shape[0] % 32 == 0)


class _LinearXentExp(torch.autograd.Function):
    """LM head + cross-entropy through the exp-epilogue GEMM (csrc/lmhead.hip)."""

    @staticmethod
    def forward(ctx, x, w, targets, ignore_index):
        t = targets.contiguous()
        check_targets(t, w.shape[0], int(ignore_index))
        loss, e, invz, inv_n = C().lmhead_fwd(x, w, t, int(ignore_index), _cref(x.device, w))
        ctx.save_for_backward(x, w, t, e, invz, inv_n)
        ctx.ignore = int(ignore_index)
        ctx.sink = sink_of(w)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, w, t, e, invz, inv_n = ctx.saved_tensors
        xt = _LM_XT and x.shape[0] % 64 == 0 and x.shape[1] % 64 == 0
        srow, xs = C().lmhead_bwd_prep(x, t, ctx.ignore, w.shape[0], invz, inv_n, g.detach(), xt)
        if xt:
            xs = xs.t()  # (N, C) view of the (C, N) tensor
        one = torch.ones(1, dtype=torch.float32, device=x.device)
        dx = dw = None
        if ctx.needs_input_grad[0] and not _LM_WGRAD_FIRST:
            dx = C().gemm_rowscale(e, w, srow)
        if ctx.needs_input_grad[1]:
            sink = ctx.sink
            if sink is not None:
                wgrad_into(e, xs, sink.view, sink.take(), one)
                sink.notify()
            else:
                dw = wgrad(e, xs, one)
        if ctx.needs_input_grad[0] and _LM_WGRAD_FIRST:
            dx = C().gemm_rowscale(e, w, srow)
        return dx, dw, None, None


class _Xent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, ignore_index):
        check_targets(targets, logits.shape[-1], int(ignore_index))
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
