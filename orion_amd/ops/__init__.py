"""Fused-op layer: HIP/CDNA4 kernels on the GPU, plain PyTorch on the CPU.

Every public function here dispatches on the device of its inputs:

* CPU tensors -> :mod:`orion_amd.ops.reference` (the numerics oracle);
* GPU tensors -> the hand-written gfx950 kernels in ``csrc/`` (loaded from the
  in-tree ``orion_amd/_C*.so``), wrapped in ``torch.autograd.Function``s.

There is deliberately no silent fallback on the GPU: if the extension is not
built, a GPU call raises.  ``ORION_AMD_OPS=torch`` (or :func:`set_backend`)
selects stock PyTorch GPU ops instead; it exists only so ``bench.py`` can
measure the stock-PyTorch baseline on the same model.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import reference as ref
from ._ext import ext_available, load_ext

_BACKEND = os.environ.get("ORION_AMD_OPS", "hip")


def set_backend(name: str):
    global _BACKEND
    assert name in ("hip", "torch"), name
    _BACKEND = name


def backend() -> str:
    return _BACKEND


def _gpu(t: torch.Tensor) -> str | None:
    """Return 'hip' / 'torch' for GPU tensors, None for CPU tensors."""
    if not t.is_cuda:
        return None
    if _BACKEND == "hip":
        load_ext(required=True)
        return "hip"
    return "torch"


# --------------------------------------------------------------------------- norms
def layer_norm(x, weight, bias, eps=1e-5):
    b = _gpu(x)
    if b == "hip":
        from .layernorm import layer_norm_hip
        return layer_norm_hip(x, weight, bias, eps)
    if b == "torch":
        return F.layer_norm(x, (x.shape[-1],), weight.to(x.dtype),
                            None if bias is None else bias.to(x.dtype), eps)
    return ref.layer_norm(x, weight, bias, eps)


def add_layer_norm(x, r, weight, bias, eps=1e-5, r_bias=None):
    """Fused residual add + LayerNorm: (s, y) = (x + r [+ r_bias], LayerNorm(s)).
    ``r_bias`` is the bias of the branch's output projection (fused here)."""
    b = _gpu(x)
    if b == "hip":
        from .layernorm import add_layer_norm_hip
        return add_layer_norm_hip(x, r, weight, bias, eps, r_bias)
    if r_bias is not None:
        r = r + r_bias.to(r.dtype)
    s = x + r
    return s, layer_norm(s, weight, bias, eps)


def linear_residual_layer_norm(x, inp, w, rb, ln_w, ln_b, eps=1e-5):
    """A residual site with the branch's output projection: (s, y) = (x + inp W^T + rb,
    LayerNorm(s)).  On the GPU one hipBLASLt GEMM with the bias and the old stream in its
    epilogue, then a LayerNorm that reads only s (ops/residual.py); elsewhere the projection
    then :func:`add_layer_norm`."""
    if _gpu(x) == "hip":
        from .residual import eligible, linear_residual_layer_norm_hip
        if eligible(x, inp, w, rb):
            return linear_residual_layer_norm_hip(x, inp, w, rb, ln_w, ln_b, eps)
    return add_layer_norm(x, linear(inp, w, None), ln_w, ln_b, eps, r_bias=rb)


def mlp_residual_layer_norm(x, h, w_fc, b_fc, w_proj, b_proj, ln_w, ln_b, eps=1e-5):
    """The MLP residual site: (s, y) = (x + mlp(h), LayerNorm(s)) with GPT-2's MLP; on the GPU
    the fused MLP whose fc2 GEMM does the residual add (ops/residual.py)."""
    if _gpu(x) == "hip":
        from .residual import mlp_eligible, mlp_residual_layer_norm_hip
        if mlp_eligible(x, h, w_fc, w_proj, b_proj):
            return mlp_residual_layer_norm_hip(x, h, w_fc, b_fc, w_proj, b_proj, ln_w, ln_b, eps)
    return add_layer_norm(x, mlp(h, w_fc, b_fc, w_proj, None), ln_w, ln_b, eps, r_bias=b_proj)


def linear_residual_rms_norm(x, inp, w, nw, eps=1e-5):
    """Llama's attention site: (s, y) = (x + inp W^T, RMSNorm(s)); on the GPU the o_proj GEMM adds
    the residual stream in its epilogue and the RMSNorm reads only s (ops/residual.py)."""
    if _gpu(x) == "hip":
        from .residual import eligible, linear_residual_rms_norm_hip
        if eligible(x, inp, w, None, need_bias=False):
            return linear_residual_rms_norm_hip(x, inp, w, nw, eps)
    return add_rms_norm(x, linear(inp, w), nw, eps)


def swiglu_residual_rms_norm(x, h, w_gate_up, w_down, nw, eps=1e-5):
    """Llama's feed-forward site: (s, y) = (x + swiglu_mlp(h), RMSNorm(s)); on the GPU down_proj
    adds the residual stream in its epilogue (ops/residual.py)."""
    if _gpu(x) == "hip":
        from .residual import swiglu_eligible, swiglu_residual_rms_norm_hip
        if swiglu_eligible(x, h, w_gate_up, w_down):
            return swiglu_residual_rms_norm_hip(x, h, w_gate_up, w_down, nw, eps)
    return add_rms_norm(x, swiglu_mlp(h, w_gate_up, w_down), nw, eps)


def add_rms_norm(x, r, weight, eps=1e-5):
    """Fused residual add + RMSNorm: (s, y) = (x + r, RMSNorm(x + r))."""
    b = _gpu(x)
    if b == "hip":
        from .layernorm import add_rms_norm_hip
        return add_rms_norm_hip(x, r, weight, eps)
    s = x + r
    return s, rms_norm(s, weight, eps)


def linear(x, weight, bias=None):
    """x W^T + b (hipBLASLt GEMM; bias gradient by the HIP column-sum kernel)."""
    b = _gpu(x)
    if b == "hip":
        from .layernorm import linear_hip
        return linear_hip(x, weight, bias)
    return F.linear(x, weight.to(x.dtype), None if bias is None else bias.to(x.dtype))


def rms_norm(x, weight, eps=1e-5):
    b = _gpu(x)
    if b == "hip":
        from .rmsnorm import rms_norm_hip
        return rms_norm_hip(x, weight, eps)
    if b == "torch":
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype) * weight.to(x.dtype)
    return ref.rms_norm(x, weight, eps)


# --------------------------------------------------------------------------- activations
def gelu(x):
    b = _gpu(x)
    if b == "hip":
        from .activations import bias_gelu_hip
        return bias_gelu_hip(x, None)
    if b == "torch":
        return F.gelu(x, approximate="tanh")
    return ref.gelu_tanh(x)


def bias_gelu(x, bias):
    b = _gpu(x)
    if b == "hip":
        from .activations import bias_gelu_hip
        return bias_gelu_hip(x, bias)
    if b == "torch":
        return F.gelu(x + bias.to(x.dtype), approximate="tanh")
    return ref.bias_gelu(x, bias)


def gelu_linear(a, fc_bias, weight, bias=None):
    """linear(gelu(a + fc_bias), weight, bias): the MLP tail.  On the GPU one autograd node
    whose backward is a single GEMM with the GELU derivative and the fc-bias gradient fused
    into its epilogue (ops/activations.py); elsewhere bias_gelu then linear."""
    b = _gpu(a)
    if b == "hip":
        from .activations import fused_mlp_ok, gelu_linear_hip
        if fused_mlp_ok(a, weight):
            return gelu_linear_hip(a, fc_bias, weight, bias)
    h = gelu(a) if fc_bias is None else bias_gelu(a, fc_bias)
    return linear(h, weight, bias)


def mlp(x, w_fc, b_fc, w_proj, b_proj=None):
    """GPT-2's MLP: linear(gelu(x W_fc^T + b_fc), W_proj, b_proj).  On the GPT-2 GPU path
    (``ORION_FUSED_MLP``) both GELU passes live in GEMM epilogues (ops/activations.py
    ``_FusedMLP``); otherwise the fc GEMM then :func:`gelu_linear`."""
    b = _gpu(x)
    if b == "hip":
        from .activations import mlp_hip, mlp_ok
        if mlp_ok(x, w_fc, w_proj):
            return mlp_hip(x, w_fc, b_fc, w_proj, b_proj)
    return gelu_linear(linear(x, w_fc), b_fc, w_proj, b_proj)


def swiglu_mlp(x, w_gate_up, w_down):
    """Llama's feed-forward: linear(swiglu(x W_gu^T), W_down) with W_gu = [W_gate; W_up].  On
    the GPU path the SwiGLU backward runs in the down_proj input-gradient GEMM's epilogue
    (ops/activations.py ``_SwigluMLP``)."""
    b = _gpu(x)
    if b == "hip":
        from .activations import swiglu_mlp_hip, swiglu_mlp_ok
        if swiglu_mlp_ok(x, w_gate_up, w_down):
            return swiglu_mlp_hip(x, w_gate_up, w_down)
    return linear(swiglu(linear(x, w_gate_up)), w_down)


def swiglu(gate_up):
    """silu(gate) * up on a packed (..., 2F) [gate | up] projection -> (..., F)."""
    b = _gpu(gate_up)
    if b == "hip":
        from .activations import swiglu_hip
        return swiglu_hip(gate_up)
    gate, up = gate_up.chunk(2, dim=-1)
    if b == "torch":
        return F.silu(gate) * up
    return ref.swiglu(gate, up)


def embed_layer_norm(idx, wte, wpe, weight, bias, eps=1e-5):
    """GPT-2's input: (x, h) = (wte[idx] + wpe[:T], LayerNorm(x)) for idx (B, T).  On the GPU
    one kernel forward; backward writes the token-table gradient straight into its (tied)
    gradient-arena slice (ops/embedding.py)."""
    b = _gpu(wte)
    if b == "hip" and wte.shape[1] % 8 == 0 and wte.shape[1] <= 2048:
        from .embedding import embed_layer_norm_hip
        return embed_layer_norm_hip(idx, wte, wpe, weight, bias, eps)
    x = add_broadcast(F.embedding(idx, wte), wpe[:idx.shape[1]])
    return x, layer_norm(x, weight, bias, eps)


_TORCH_EMBEDDING = os.environ.get("ORION_EMBEDDING") == "torch"  # A/B: PyTorch's embedding backward


def token_embedding(idx, weight):
    """weight[idx] (Llama's token embedding; ``embedding`` is the submodule's name).  On the GPU
    the backward adds into the table's gradient-arena slice directly (ops/embedding.py)."""
    b = _gpu(weight)
    if b == "hip" and weight.shape[1] % 8 == 0 and weight.dtype == torch.bfloat16 and not _TORCH_EMBEDDING:
        from .embedding import embedding_hip
        return embedding_hip(idx, weight)
    return F.embedding(idx, weight)


def add_broadcast(x, pos):
    """x (B, T, C) + pos (T, C); kept as one op so the GPU path is one kernel."""
    return x + pos.to(x.dtype)


# --------------------------------------------------------------------------- rope
def rope(x, cos, sin, pos0=0):
    """Rotate-half RoPE of x (B, T, H, D) at positions pos0..pos0+T-1 (fp32 tables (Tmax, D/2))."""
    b = _gpu(x)
    if b == "hip":
        from .rotary import rope_hip
        return rope_hip(x, cos, sin, pos0)
    return ref.rope(x, cos[pos0:], sin[pos0:])


def linear_rope_attention(x, weight, n_q, n_kv, cos, sin, pos0=0):
    """Causal attention of (rope(q), rope(k), v) of the packed projection x W^T, W (Hq + 2 Hkv)
    D rows -> (B, T, Hq, D).  GPU path with head dim 128: one fused node, the rotation in the
    projection GEMM's epilogue (flash_attn.qkv_rope_flash_attention); otherwise the projection
    then rope_attention_packed."""
    if _gpu(x) == "hip":
        from .flash_attn import qkv_rope_eligible, qkv_rope_flash_attention
        if qkv_rope_eligible(x, weight, n_q, n_kv, cos):
            return qkv_rope_flash_attention(x, weight, n_q, n_kv, cos, sin, pos0)
    B, T, _ = x.shape
    qkv = linear(x, weight).view(B, T, n_q + 2 * n_kv, weight.shape[0] // (n_q + 2 * n_kv))
    return rope_attention_packed(qkv, n_q, n_kv, cos, sin, pos0)


def rope_attention_packed(qkv, n_q, n_kv, cos, sin, pos0=0):
    """Causal attention of (rope(q), rope(k), v) on a packed (B, T, Hq + 2 Hkv, D) projection
    -> (B, T, Hq, D).  The GPU path is one fused autograd node (no per-view glue)."""
    b = _gpu(qkv)
    if b == "hip":
        from .flash_attn import rope_flash_attention_packed
        return rope_flash_attention_packed(qkv, n_q, n_kv, cos, sin, pos0)
    q = rope(qkv[:, :, :n_q], cos, sin, pos0)
    k = rope(qkv[:, :, n_q:n_q + n_kv], cos, sin, pos0)
    return attention(q, k, qkv[:, :, n_q + n_kv:], causal=True)


# --------------------------------------------------------------------------- attention
def attention_qkv(qkv, n_head, causal=True):
    """Causal self-attention on a packed (B, T, 3C) projection -> (B, T, C)."""
    b = _gpu(qkv)
    if b == "hip":
        from .flash_attn import flash_attention_qkv
        return flash_attention_qkv(qkv, n_head, causal)
    if b == "torch":
        B, T, C3 = qkv.shape
        C = C3 // 3
        q, k, v = qkv.view(B, T, 3, n_head, C // n_head).unbind(2)
        y = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2),
                                           v.transpose(1, 2), is_causal=causal)
        return y.transpose(1, 2).reshape(B, T, C)
    return ref.attention_qkv(qkv, n_head, causal)


def linear_attention_qkv(x, weight, bias, n_head, causal=True):
    """Causal self-attention of the QKV projection x W^T + b -> (B, T, C).  On the HIP path
    the projection's bias gradient comes out of the attention backward (column sums fused
    into the split kernels) instead of a column-sum pass over the packed dQKV."""
    if _gpu(x) == "hip" and bias is not None:
        from .flash_attn import flash_attention_qkv
        from .layernorm import linear_hip
        qkv = linear_hip(x, weight, bias.detach())
        return flash_attention_qkv(qkv, n_head, causal, bias)
    return attention_qkv(linear(x, weight, bias), n_head, causal)


def attention(q, k, v, causal=True):
    """Attention on (B, T, H, D) tensors (GQA when k/v have fewer heads)."""
    b = _gpu(q)
    if b == "hip":
        from .flash_attn import flash_attention
        return flash_attention(q, k, v, causal)
    if b == "torch":
        rep = q.shape[2] // k.shape[2]
        kk = k.repeat_interleave(rep, 2) if rep > 1 else k
        vv = v.repeat_interleave(rep, 2) if rep > 1 else v
        y = F.scaled_dot_product_attention(q.transpose(1, 2), kk.transpose(1, 2),
                                           vv.transpose(1, 2), is_causal=causal)
        return y.transpose(1, 2)
    return ref.attention(q, k, v, causal)


# --------------------------------------------------------------------------- loss
def cross_entropy(logits, targets, ignore_index=-1):
    b = _gpu(logits)
    if b == "hip":
        from .xent import fused_cross_entropy
        return fused_cross_entropy(logits, targets, ignore_index)
    if b == "torch":
        return F.cross_entropy(logits.float(), targets, ignore_index=ignore_index)
    return ref.cross_entropy(logits, targets, ignore_index)


def linear_cross_entropy(x, weight, targets, ignore_index=-1):
    """mean CE of softmax(x @ weight^T); x (N, C), weight (V, C) -- the fused LM head + loss."""
    b = _gpu(x)
    if b == "hip":
        from .xent import linear_cross_entropy_hip
        return linear_cross_entropy_hip(x, weight, targets, ignore_index)
    logits = F.linear(x, weight.to(x.dtype))
    if b == "torch":
        return F.cross_entropy(logits.float(), targets, ignore_index=ignore_index)
    return ref.cross_entropy(logits, targets, ignore_index)


__all__ = [
    "set_backend", "backend", "ext_available", "load_ext",
    "layer_norm", "rms_norm", "gelu", "bias_gelu", "swiglu", "add_broadcast", "embed_layer_norm",
    "token_embedding", "rope",
    "attention_qkv", "linear_attention_qkv", "attention", "rope_attention_packed", "linear_rope_attention",
    "cross_entropy", "swiglu_mlp", "linear_residual_layer_norm", "mlp_residual_layer_norm",
    "linear_residual_rms_norm", "swiglu_residual_rms_norm",
    "linear_cross_entropy",
]


# ------------------------------------------------------------------ parameter-read guards
# ZeRO-1 leaves the weight all-gathers of the previous optimizer step in flight
# (parallel/ddp.py ShardedGradReducer.gather_params).  The fused ops read weights of several
# modules at once from the model's top-level forward (block i's add+LayerNorm takes block
# i+1's ln_1, the embedding takes block 0's), so module forward hooks alone cannot say when a
# weight is first read: every op here that takes weights first hands its arguments to the
# registered guards, which wait for the gathers of the buckets those tensors live in.
_PARAM_GUARDS: list = []


def add_param_guard(fn):
    """Register ``fn(tensors)`` to run before any weight-taking op; returns a remover.  A
    bound method is held weakly (a dropped reducer unregisters itself)."""
    import weakref
    ref_ = weakref.WeakMethod(fn) if hasattr(fn, "__self__") else (lambda: fn)
    _PARAM_GUARDS.append(ref_)

    def remove():
        if ref_ in _PARAM_GUARDS:
            _PARAM_GUARDS.remove(ref_)
    return remove


def _guarded(fn):
    import functools

    @functools.wraps(fn)
    def run(*args, **kw):
        if _PARAM_GUARDS:
            ts = [a for a in args if isinstance(a, torch.Tensor)]
            ts += [a for a in kw.values() if isinstance(a, torch.Tensor)]
            for g in list(_PARAM_GUARDS):
                f = g()
                if f is None:
                    _PARAM_GUARDS.remove(g)
                else:
                    f(ts)
        return fn(*args, **kw)
    run.__wrapped_op__ = fn
    return run


for _name in ("layer_norm", "add_layer_norm", "add_rms_norm", "linear", "rms_norm", "bias_gelu",
              "gelu_linear", "mlp", "swiglu_mlp", "embed_layer_norm", "token_embedding", "add_broadcast",
              "linear_attention_qkv", "linear_rope_attention",
              "linear_cross_entropy"):
    globals()[_name] = _guarded(globals()[_name])
del _name
