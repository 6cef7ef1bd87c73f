"""Plain-PyTorch reference implementations of every fused op.

These are the CPU execution path and the numerics oracle for the HIP kernels
in ``csrc/``.  They favour clarity over speed and compute in fp32 internally.

Layout conventions shared with the HIP kernels:

* ``qkv`` is the raw output of the fused QKV projection, shape ``(B, T, 3*C)``
  and read as ``(B, T, 3, H, D)``; attention output is ``(B, T, H*D)`` so it
  feeds the output projection with no transpose.
* cross-entropy takes ``logits`` ``(N, V)`` and int64 ``targets`` ``(N,)``;
  ``ignore_index`` rows contribute nothing.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def layer_norm(x, weight, bias, eps=1e-5):
    y = F.layer_norm(x.float(), (x.shape[-1],), weight.float(),
                     None if bias is None else bias.float(), eps)
    return y.to(x.dtype)


def rms_norm(x, weight, eps=1e-5):
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * weight.float()
    return y.to(x.dtype)


def gelu_tanh(x):
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


def bias_gelu(x, bias):
    return F.gelu(x.float() + bias.float(), approximate="tanh").to(x.dtype)


def swiglu(gate, up):
    return (F.silu(gate.float()) * up.float()).to(gate.dtype)


def rope_tables(seq_len, head_dim, theta=10000.0, device=None):
    """cos/sin tables of shape (T, D/2), fp32 (computed once on the host side)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(seq_len, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return ang.cos().float().to(device), ang.sin().float().to(device)


def rope(x, cos, sin):
    """Rotate interleaved-half pairs (x[..., :D/2], x[..., D/2:]) of x (B, T, H, D)."""
    xf = x.float()
    d2 = x.shape[-1] // 2
    x1, x2 = xf[..., :d2], xf[..., d2:]
    c = cos[: x.shape[1]].view(1, x.shape[1], 1, d2)
    s = sin[: x.shape[1]].view(1, x.shape[1], 1, d2)
    out = torch.cat([x1 * c - x2 * s, x1 * s + x2 * c], dim=-1)
    return out.to(x.dtype)


def attention_qkv(qkv, n_head, causal=True, scale=None):
    """softmax(Q K^T * scale [+ causal mask]) V for packed qkv (B, T, 3*C)."""
    B, T, C3 = qkv.shape
    C = C3 // 3
    D = C // n_head
    q, k, v = qkv.float().view(B, T, 3, n_head, D).unbind(2)
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))  # (B, H, T, D)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    s = (q @ k.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(T, T, dtype=torch.bool, device=qkv.device).tril()
        s = s.masked_fill(~mask, float("-inf"))
    p = s.softmax(-1)
    o = (p @ v).transpose(1, 2).reshape(B, T, C)
    return o.to(qkv.dtype)


def attention(q, k, v, causal=True, scale=None):
    """softmax attention for separate q (B,T,Hq,D), k/v (B,T,Hkv,D) with GQA."""
    B, T, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    if rep > 1:
        kf = kf.repeat_interleave(rep, dim=1)
        vf = vf.repeat_interleave(rep, dim=1)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    s = (qf @ kf.transpose(-1, -2)) * scale
    if causal:
        Tk = k.shape[1]
        mask = torch.ones(T, Tk, dtype=torch.bool, device=q.device).tril(Tk - T)
        s = s.masked_fill(~mask, float("-inf"))
    o = (s.softmax(-1) @ vf).transpose(1, 2)
    return o.to(q.dtype)


def cross_entropy(logits, targets, ignore_index=-1):
    return F.cross_entropy(logits.float(), targets, ignore_index=ignore_index)


def adamw_step(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step,
               grad_scale=1.0):
    """In-place decoupled-weight-decay Adam on fp32 tensors (torch.optim.AdamW maths)."""
    g = grad.float() * grad_scale
    param.mul_(1.0 - lr * weight_decay)
    exp_avg.mul_(beta1).add_(g, alpha=1.0 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    denom = (exp_avg_sq / bc2).sqrt_().add_(eps)
    param.addcdiv_(exp_avg, denom, value=-lr / bc1)
    return param
