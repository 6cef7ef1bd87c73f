"""Token + position embedding fused with the first LayerNorm (GPT-2), on the HIP kernels.

Forward (one kernel, csrc/layernorm.hip in gather mode): s = wte[idx] + wpe[t] is formed,
returned (the residual stream) and normalised; it replaces an embedding gather, a
broadcast add and a LayerNorm pass.

Backward: the LayerNorm backward folds the residual-stream gradient into dx (as for every
other add+LayerNorm), then
  * wpe: the column sum of dx over the batch, written into wpe's gradient-arena slice;
  * wte: dx added row by row into the token table's fp32 arena slice with fp32 atomics
    (csrc/embedding.hip).  The table is tied to the LM head, whose weight gradient was
    written into the same slice at the start of the backward; the sink expects both
    producers before it reports the parameter to the data-parallel reducer
    (ops/grad_sink.py).  Deterministic mode and gradient-accumulation steps whose slice
    cannot be written directly use the sort-based dense embedding backward.

Token ids are validated: the first call per device checks ``idx`` against the table on the
host (one ``aminmax``; ``ORION_CHECK_IDS=1`` checks every call, at the price of a sync) and
raises ``IndexError``, and both kernels clamp / skip any id outside ``[0, V)`` and raise a
device flag instead of reading or atomically adding outside the table (``id_error``).
"""
from __future__ import annotations

import os

import torch

from ._ext import C
from .determinism import deterministic
from .grad_sink import sink_of
from .layernorm import _bf16, _claim, _grad, _notify, _unless, _view

_CHECK_ALWAYS = os.environ.get("ORION_CHECK_IDS") == "1"
_checked: set = set()


def check_ids(idx, V):
    """Raise IndexError if any token id is outside [0, V) (synchronises)."""
    lo, hi = torch.aminmax(idx)
    lo, hi = int(lo), int(hi)
    if lo < 0 or hi >= V:
        raise IndexError(f"token id out of range: ids span [{lo}, {hi}] for a table of {V} rows")


def id_error(device=None) -> bool:
    """True if an embedding kernel saw an out-of-range token id, or a cross-entropy kernel an
    out-of-range target (not ignore_index; ``ops.xent.check_targets``), since the last call on
    this device (the flag is cleared; synchronises the current stream)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    return bool(C().embed_id_error(dev.index if dev.index is not None else 0))


def _dense_table_grad(dx2, idx, V):
    return torch.ops.aten.embedding_dense_backward(dx2, idx.reshape(-1), V, -1, False)


class _EmbedLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe, w, b, eps):
        s, y, mean, rstd = C().embed_layernorm_fwd(idx, _bf16(wte), _bf16(wpe), _bf16(w), _bf16(b),
                                                   float(eps))
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(idx, s, w, mean, rstd)
        ctx.has_bias = b is not None
        ctx.b_dtype = None if b is None else b.dtype
        ctx.params = (w, b)
        ctx.tables = (wte, wpe)
        return s, y

    @staticmethod
    def backward(ctx, ds, dy):
        idx, s, w, mean, rstd = ctx.saved_tensors
        wte, wpe = ctx.tables
        B, T, Cc = s.shape
        if dy is None:
            dy = torch.zeros_like(s)
        dres = None if ds is None else ds.contiguous()
        sw, sb = _claim(ctx.params)
        dx, dw, db, _ = C().layernorm_bwd(dy.contiguous(), s, _bf16(w), mean, rstd, ctx.has_bias,
                                          dres, False, _view(sw), _view(sb))
        _notify(sw, sb)
        dw, db = _unless(dw, sw), _unless(db, sb)
        dx2 = dx.view(B * T, Cc)

        # position table: column sums of dx over the batch into rows 0..T-1
        dwpe = None
        if ctx.needs_input_grad[2]:
            (spe,) = _claim((wpe,))
            if spe is not None:
                view = spe.view.view(-1, Cc)
                C().batch_sum_(dx.view(B, T * Cc), view[:T].reshape(-1))
                if view.shape[0] > T:  # positions this step did not use (slice not pre-zeroed)
                    view[T:].zero_()
                spe.notify()
            else:
                dwpe = torch.zeros_like(wpe, dtype=torch.float32)
                dwpe[:T] = dx.float().sum(0)
                dwpe = dwpe.to(wpe.dtype)

        # token table (tied to the LM head)
        dwte = None
        if ctx.needs_input_grad[1]:
            st = sink_of(wte)
            if st is not None and st.view.dtype == torch.float32 and not deterministic():
                view, acc = st.last_use_target()
                if not acc:  # first producer of the step: the slice is not pre-zeroed
                    view.zero_()
                C().embed_scatter_add_(dx2, idx, view.view(-1, Cc))
                st.notify(last=True)
            elif st is not None:
                g = _dense_table_grad(dx2, idx, wte.shape[0])
                view, acc = st.last_use_target()
                if acc:
                    view.view(-1, Cc).add_(g)
                else:
                    view.view(-1, Cc).copy_(g)
                st.notify(last=True)
            else:
                dwte = _dense_table_grad(dx2, idx, wte.shape[0]).to(wte.dtype)
        return (None, dwte, dwpe, _grad(dw, w.dtype),
                (_grad(db, ctx.b_dtype) if ctx.has_bias else None), None)


def embed_layer_norm_hip(idx, wte, wpe, weight, bias, eps=1e-5):
    if _CHECK_ALWAYS or idx.device not in _checked:
        check_ids(idx, wte.shape[0])
        _checked.add(idx.device)
    return _EmbedLayerNorm.apply(idx.long(), wte, wpe, weight, bias, eps)


class _Embedding(torch.autograd.Function):
    """Plain token embedding (Llama): the forward is the gather; the backward adds dy row by row
    into the table's fp32 gradient-arena slice with fp32 atomics (csrc/embedding.hip) instead of
    the sort-based dense backward plus a pass adding it into the arena (Llama-7B: ~1.0 ms ->
    ~0.3 ms per step).  Deterministic mode, a bf16 arena or no arena take the dense backward."""

    @staticmethod
    def forward(ctx, idx, weight):
        ctx.save_for_backward(idx)
        ctx.table = weight
        return torch.nn.functional.embedding(idx, weight)

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        wte = ctx.table
        if not ctx.needs_input_grad[1]:
            return None, None
        Cc = wte.shape[1]
        dy2 = dy.reshape(-1, Cc)
        if dy2.dtype != torch.bfloat16:
            dy2 = dy2.to(torch.bfloat16)
        st = sink_of(wte)
        if st is not None and st.view.dtype == torch.float32 and not deterministic():
            view, acc = st.last_use_target()
            if not acc:  # first producer of the step: the slice is not pre-zeroed
                view.zero_()
            C().embed_scatter_add_(dy2, idx, view.view(-1, Cc))
            st.notify(last=True)
            return None, None
        if st is not None:
            g = _dense_table_grad(dy2, idx, wte.shape[0])
            view, acc = st.last_use_target()
            if acc:
                view.view(-1, Cc).add_(g)
            else:
                view.view(-1, Cc).copy_(g)
            st.notify(last=True)
            return None, None
        return None, _dense_table_grad(dy2, idx, wte.shape[0]).to(wte.dtype)


def embedding_hip(idx, weight):
    if _CHECK_ALWAYS or idx.device not in _checked:
        check_ids(idx, weight.shape[0])
        _checked.add(idx.device)
    return _Embedding.apply(idx.long(), weight)
