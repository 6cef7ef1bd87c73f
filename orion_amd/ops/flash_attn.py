"""Flash-attention autograd wrappers over the HIP kernels: csrc/attn_fwd.hip (forward) and
csrc/attn_bwd_split.hip (delta, dK/dV and dQ kernels, the backward); csrc/attention.hip keeps
the 64-bit-addressed forms for operands beyond the others' 32-bit buffer offsets.

``flash_attention_qkv`` consumes the packed (B, T, 3C) output of a fused QKV
projection through strided views and produces the packed gradient in one
buffer, so there is no split/transpose/concat around the kernels.
"""
from __future__ import annotations

import math
import os

import torch

from ._ext import C
from .determinism import deterministic
from .grad_sink import sink_of


def _bwd_flags() -> int:
    return 4 if deterministic() else 0


class _FlashQKV(torch.autograd.Function):
    """Attention on the packed (B, T, 3C) output of the QKV projection.  ``qkv_bias``: the
    projection's bias, already added to ``qkv`` by a linear that did not track it; its
    gradient colsum(dQKV) is produced here -- by the split backward kernels as fp32 column
    sums per 32-token block (no pass over the packed dQKV) -- and written through the
    bias's gradient sink (ops/grad_sink.py)."""

    @staticmethod
    def forward(ctx, qkv, n_head, causal, qkv_bias):
        B, T, C3 = qkv.shape
        Cm = C3 // 3
        D = Cm // n_head
        v5 = qkv.view(B, T, 3, n_head, D)
        scale = 1.0 / math.sqrt(D)
        o, lse = C().attn_fwd(v5[:, :, 0], v5[:, :, 1], v5[:, :, 2], bool(causal), scale)
        ctx.save_for_backward(qkv, o, lse)
        ctx.meta = (n_head, bool(causal), scale)
        ctx.bias = qkv_bias
        return o.view(B, T, Cm)

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        n_head, causal, scale = ctx.meta
        B, T, C3 = qkv.shape
        D = C3 // 3 // n_head
        v5 = qkv.view(B, T, 3, n_head, D)
        dqkv = torch.empty_like(qkv)
        d5 = dqkv.view(B, T, 3, n_head, D)
        do4 = do.contiguous().view(B, T, n_head, D)
        bias = ctx.bias
        want_db = bias is not None and ctx.needs_input_grad[3]
        sb = db = None
        if want_db:
            from .grad_sink import claim
            sb = claim(bias) if bias.dtype == torch.bfloat16 else None
            db = sb.view if sb is not None else torch.empty(C3, dtype=qkv.dtype, device=qkv.device)
        C().attn_bwd(do4, v5[:, :, 0], v5[:, :, 1], v5[:, :, 2], o, lse, causal, scale,
                     d5[:, :, 0], d5[:, :, 1], d5[:, :, 2], _bwd_flags(), db)
        if sb is not None:  # written into the arena slice; never handed back to autograd
            sb.notify()
            db = None
        elif db is not None:
            db = db.to(bias.dtype)
        return dqkv, None, None, db


def flash_attention_qkv(qkv, n_head, causal=True, qkv_bias=None):
    return _FlashQKV.apply(qkv, n_head, causal, qkv_bias)


class _Flash(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal):
        D = q.shape[-1]
        scale = 1.0 / math.sqrt(D)
        o, lse = C().attn_fwd(q, k, v, bool(causal), scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.meta = (bool(causal), scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        causal, scale = ctx.meta
        dq = torch.empty(q.shape, dtype=q.dtype, device=q.device)
        dk = torch.empty(k.shape, dtype=k.dtype, device=k.device)
        dv = torch.empty(v.shape, dtype=v.dtype, device=v.device)
        C().attn_bwd(do.contiguous(), q, k, v, o, lse, causal, scale, dq, dk, dv, _bwd_flags())
        return dq, dk, dv, None


def flash_attention(q, k, v, causal=True):
    """q (B, T, Hq, D), k/v (B, Tk, Hkv, D) with unit stride on D -> (B, T, Hq, D)."""
    return _Flash.apply(q, k, v, causal)


class _RopeFlashPacked(torch.autograd.Function):
    """RoPE + causal flash attention on a packed (B, T, Hq + 2 Hkv, D) QKV projection.

    Forward: ONE rope launch rotates the adjacent q|k head range into a contiguous
    (B, T, Hq + Hkv, D) buffer; the attention kernel reads q and k as strided views of it
    and v straight from the projection.  Backward: the attention kernels write dq, dk and
    dv into the three head ranges of ONE packed gradient buffer, dq and dk already
    un-rotated (the inverse rotation at the split kernels' stores, csrc/attn_bwd_split.hip
    store_row_grad; the other backward forms run the rope kernel after) -- no zero-fill,
    slice copies, gradient adds or rope pass around the kernels."""

    @staticmethod
    def forward(ctx, qkv, n_q, n_kv, cos, sin, pos0):
        B, T, H3, D = qkv.shape
        qk = C().rope(qkv[:, :, :n_q + n_kv], cos, sin, int(pos0), 1.0)
        scale = 1.0 / math.sqrt(D)
        v = qkv[:, :, n_q + n_kv:]
        o, lse = C().attn_fwd(qk[:, :, :n_q], qk[:, :, n_q:], v, True, scale)
        ctx.save_for_backward(qkv, qk, o, lse, cos, sin)
        ctx.meta = (n_q, n_kv, int(pos0), scale)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, qk, o, lse, cos, sin = ctx.saved_tensors
        n_q, n_kv, pos0, scale = ctx.meta
        dqkv = torch.empty_like(qkv)
        C().attn_bwd(do.contiguous(), qk[:, :, :n_q], qk[:, :, n_q:], qkv[:, :, n_q + n_kv:], o, lse,
                     True, scale, dqkv[:, :, :n_q], dqkv[:, :, n_q:n_q + n_kv], dqkv[:, :, n_q + n_kv:],
                     _bwd_flags(), None, cos, sin, pos0)
        return dqkv, None, None, None, None, None


class _QKVRopeFlash(torch.autograd.Function):
    """Llama's packed QKV projection + RoPE + causal flash attention as ONE node (round 6).

    Forward: the in-tree GEMM (csrc/gemm16.hip EPI_ROPE) writes q and k already rotated -- the
    rotation applied to the fp32 accumulators before the one bf16 rounding -- and v as computed,
    so the separate rope pass (a read and a write of the q | k heads) is gone; the attention
    reads the three head ranges of that buffer.  Backward: as _RopeFlashPacked, the attention
    kernels write dq / dk un-rotated into one packed dqkv, which then feeds the projection's
    input and weight gradients (ops/layernorm.py linear_input_weight_grads)."""

    @staticmethod
    def forward(ctx, x, w, n_q, n_kv, cos, sin, pos0):
        B, T, _ = x.shape
        H3 = n_q + 2 * n_kv
        D = w.shape[0] // H3
        qkv = C().gemm_rope(x, w, cos, sin, int(pos0), T, (n_q + n_kv) * D, D).view(B, T, H3, D)
        scale = 1.0 / math.sqrt(D)
        o, lse = C().attn_fwd(qkv[:, :, :n_q], qkv[:, :, n_q:n_q + n_kv], qkv[:, :, n_q + n_kv:], True, scale)
        ctx.save_for_backward(x, w, qkv, o, lse, cos, sin)
        ctx.meta = (n_q, n_kv, int(pos0), scale)
        ctx.sink = sink_of(w)
        return o

    @staticmethod
    def backward(ctx, do):
        from .layernorm import linear_input_weight_grads
        x, w, qkv, o, lse, cos, sin = ctx.saved_tensors
        n_q, n_kv, pos0, scale = ctx.meta
        dqkv = torch.empty_like(qkv)
        C().attn_bwd(do.contiguous(), qkv[:, :, :n_q], qkv[:, :, n_q:n_q + n_kv], qkv[:, :, n_q + n_kv:], o, lse,
                     True, scale, dqkv[:, :, :n_q], dqkv[:, :, n_q:n_q + n_kv], dqkv[:, :, n_q + n_kv:],
                     _bwd_flags(), None, cos, sin, pos0)
        dx, dw = linear_input_weight_grads(dqkv.view(-1, dqkv.shape[2] * dqkv.shape[3]), x, w, ctx.sink,
                                           ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return dx, dw, None, None, None, None, None


# ORION_QKV_ROPE=0: the projection on its own (hipBLASLt) and the rope pass (A/B)
_QKV_ROPE = os.environ.get("ORION_QKV_ROPE", "1") != "0"


def qkv_rope_eligible(x, w, n_q, n_kv, cos) -> bool:
    from .gemm import gemm16_addressable
    H3 = n_q + 2 * n_kv
    if not (_QKV_ROPE and x.is_cuda and x.dim() == 3 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and w.dim() == 2 and w.shape[0] % H3 == 0 and w.shape[0] // H3 == 128 and x.stride(-1) == 1
            and x.is_contiguous() and w.is_contiguous() and x.shape[-1] % 64 == 0 and x.data_ptr() % 16 == 0
            and w.data_ptr() % 16 == 0 and cos.dtype == torch.float32 and cos.is_contiguous()):
        return False
    return gemm16_addressable(x.shape[-1], x.shape[-1], w.shape[0], False)


def qkv_rope_flash_attention(x, w, n_q, n_kv, cos, sin, pos0=0):
    """x (B, T, C) -> causal attention of rope(q), rope(k), v of the packed projection x w^T."""
    return _QKVRopeFlash.apply(x, w, n_q, n_kv, cos, sin, pos0)


def rope_flash_attention_packed(qkv, n_q, n_kv, cos, sin, pos0=0):
    """qkv (B, T, Hq + 2 Hkv, D) -> causal attention of rope(q), rope(k), v: (B, T, Hq, D)."""
    return _RopeFlashPacked.apply(qkv, n_q, n_kv, cos, sin, pos0)
