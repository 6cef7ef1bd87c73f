"""Llama-family decoder (RMSNorm, RoPE, SwiGLU, GQA) on the orion_amd op layer.

BASELINE.json configs 4/5 name a Llama-2-7B-shape model at seq 4096 (SURVEY.md
§2.11: L=32, d=4096, H=32, head_dim=128, FFN 11008, vocab 32000, RoPE theta
1e4).  MI355X-first layout:

* ONE fused QKV projection ``(B, T, (Hq + 2 Hkv) D)``; RoPE reads the q/k
  slices through strides and writes contiguous rotated copies; V is consumed
  in place by the flash-attention kernel (strided view) -- no split/transpose;
* ONE fused gate|up projection ``(B, T, 2F)`` feeding the packed SwiGLU kernel;
* residual add + RMSNorm fused (one kernel forward, one backward), like GPT-2's
  add+LayerNorm;
* parameter names follow the Hugging Face Llama layout where the shapes allow
  (``model.layers.{i}.self_attn.o_proj`` ...), with the fused ``qkv_proj`` /
  ``gate_up_proj`` documented in :func:`split_fused_state_dict`.
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass

import torch
import torch.nn as nn

from .. import ops
from ..ops import reference as ref


@dataclass
class LlamaConfig:
    vocab_size: int = 32000
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 32
    ffn_dim: int = 11008
    max_seq_len: int = 4096
    rope_theta: float = 10000.0
    norm_eps: float = 1e-5
    tie_embeddings: bool = False

    @property
    def head_dim(self):
        return self.dim // self.n_heads

    def to_dict(self):
        return asdict(self)


PRESETS = {
    "llama-tiny": dict(vocab_size=512, dim=256, n_layers=2, n_heads=4, n_kv_heads=2, ffn_dim=512,
                       max_seq_len=256),
    "llama2-7b": dict(),
    "llama2-13b": dict(dim=5120, n_layers=40, n_heads=40, n_kv_heads=40, ffn_dim=13824),
    "llama3-8b": dict(vocab_size=128256, n_kv_heads=8, ffn_dim=14336, max_seq_len=8192,
                      rope_theta=500000.0),
    "llama-1b-gqa": dict(dim=2048, n_layers=16, n_heads=16, n_kv_heads=4, ffn_dim=5632),
}


class RMSNorm(nn.Module):
    def __init__(self, dim, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.eps = eps

    def forward(self, x):
        return ops.rms_norm(x, self.weight, self.eps)


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.n_heads, self.n_kv, self.hd = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
        self.qkv_proj = nn.Linear(cfg.dim, (cfg.n_heads + 2 * cfg.n_kv_heads) * cfg.head_dim, bias=False)
        self.o_proj = nn.Linear(cfg.n_heads * cfg.head_dim, cfg.dim, bias=False)

    def attend(self, x, cos, sin, pos0=0):
        """QKV projection + RoPE + attention, before o_proj: (B, T, Hq * D).  On the GPU with
        D = 128 the rotation rides in the projection's epilogue."""
        B, T, _ = x.shape
        o = ops.linear_rope_attention(x, self.qkv_proj.weight, self.n_heads, self.n_kv, cos, sin, pos0)
        return o.reshape(B, T, -1)

    def forward(self, x, cos, sin, pos0=0):
        return ops.linear(self.attend(x, cos, sin, pos0), self.o_proj.weight)


class FeedForward(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.gate_up_proj = nn.Linear(cfg.dim, 2 * cfg.ffn_dim, bias=False)
        self.down_proj = nn.Linear(cfg.ffn_dim, cfg.dim, bias=False)

    def forward(self, x):
        return ops.swiglu_mlp(x, self.gate_up_proj.weight, self.down_proj.weight)


class DecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.self_attn = Attention(cfg)
        self.post_attention_layernorm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.mlp = FeedForward(cfg)


class Llama(nn.Module):
    """``forward(idx, targets)`` -> (logits|None, loss|None), same contract as GPT."""

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.config = cfg
        self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.dim)
        self.layers = nn.ModuleList([DecoderLayer(cfg) for _ in range(cfg.n_layers)])
        self.norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.lm_head = nn.Linear(cfg.dim, cfg.vocab_size, bias=False)
        if cfg.tie_embeddings:
            self.lm_head.weight = self.embed_tokens.weight
        cos, sin = ref.rope_tables(cfg.max_seq_len, cfg.head_dim, cfg.rope_theta)
        self.register_buffer("rope_cos", cos, persistent=False)
        self.register_buffer("rope_sin", sin, persistent=False)
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        std = 0.02
        for name, p in self.named_parameters():
            if p.dim() == 1:
                p.fill_(1.0)
            elif name.endswith(("o_proj.weight", "down_proj.weight")):
                p.normal_(0.0, std / math.sqrt(2 * self.config.n_layers))
            else:
                p.normal_(0.0, std)

    def num_params(self, non_embedding=False):
        n = sum(p.numel() for p in self.parameters())
        if non_embedding:
            n -= self.embed_tokens.weight.numel()
        return n

    def flops_per_token(self, seq_len=None):
        cfg = self.config
        T = seq_len or cfg.max_seq_len
        return 6 * self.num_params(non_embedding=True) + 12 * cfg.n_layers * cfg.dim * T

    def forward(self, idx, targets=None, pos0=0):
        B, T = idx.shape
        assert pos0 + T <= self.config.max_seq_len
        x = ops.token_embedding(idx, self.embed_tokens.weight)
        cos, sin = self.rope_cos, self.rope_sin
        layers = self.layers
        h = layers[0].input_layernorm(x)
        # the o_proj / down_proj GEMMs add the residual stream in their epilogue and the
        # RMSNorm reads only the new stream (ops/residual.py; other backends: add_rms_norm)
        for i, layer in enumerate(layers):
            at, ff, pln = layer.self_attn, layer.mlp, layer.post_attention_layernorm
            x, h = ops.linear_residual_rms_norm(x, at.attend(h, cos, sin, pos0), at.o_proj.weight,
                                                pln.weight, pln.eps)
            nxt = layers[i + 1].input_layernorm if i + 1 < len(layers) else self.norm
            x, h = ops.swiglu_residual_rms_norm(x, h, ff.gate_up_proj.weight, ff.down_proj.weight,
                                                nxt.weight, nxt.eps)
        if targets is not None:
            loss = ops.linear_cross_entropy(h.reshape(B * T, -1), self.lm_head.weight,
                                            targets.reshape(-1), ignore_index=-1)
            return None, loss
        logits = ops.linear(h[:, [-1], :], self.lm_head.weight)
        return logits, None

    @torch.no_grad()
    def generate(self, idx, max_new_tokens, temperature=1.0, top_k=None):
        for _ in range(max_new_tokens):
            cond = idx[:, -self.config.max_seq_len:]
            logits, _ = self(cond)
            logits = logits[:, -1, :].float() / max(temperature, 1e-6)
            if top_k is not None:
                v, _ = torch.topk(logits, min(top_k, logits.size(-1)))
                logits[logits < v[:, [-1]]] = -float("inf")
            idx = torch.cat((idx, torch.multinomial(torch.softmax(logits, -1), 1)), dim=1)
        return idx


def build_llama(preset="llama2-7b", **overrides):
    kw = dict(PRESETS[preset])
    kw.update(overrides)
    return Llama(LlamaConfig(**kw))


def split_fused_state_dict(sd, cfg: LlamaConfig):
    """Fused qkv_proj / gate_up_proj -> Hugging Face q/k/v_proj, gate/up_proj tensors."""
    out = {}
    hq, hk, hd = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
    for k, v in sd.items():
        if k.endswith("qkv_proj.weight"):
            base = k[: -len("qkv_proj.weight")]
            q, kk, vv = torch.split(v, [hq * hd, hk * hd, hk * hd], dim=0)
            out[base + "q_proj.weight"], out[base + "k_proj.weight"], out[base + "v_proj.weight"] = q, kk, vv
        elif k.endswith("gate_up_proj.weight"):
            base = k[: -len("gate_up_proj.weight")]
            g, u = v.chunk(2, dim=0)
            out[base + "gate_proj.weight"], out[base + "up_proj.weight"] = g, u
        else:
            out[k] = v
    return out
