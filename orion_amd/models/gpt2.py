"""GPT-2 decoder (nanoGPT-compatible parameter names) on the orion_amd op layer.

Parameter names follow the public nanoGPT/HF-GPT-2 layout (``transformer.wte``,
``transformer.h.{i}.attn.c_attn`` ...) so ``ckpt.pt`` files written by
``orion_amd.train.ckpt`` load into nanoGPT-style code and vice versa.

MI355X-first choices (not in the reference, which has no model at all --
SURVEY.md §2.11 [north-star]):

* the QKV projection output ``(B, T, 3C)`` is consumed by the flash-attention
  kernel in place (no head transposes); the kernel writes ``(B, T, C)`` for
  ``c_proj``;
* ``c_fc`` bias + GELU-tanh run as one fused HIP kernel after a bias-less GEMM;
* the loss is a fused softmax-cross-entropy that emits dlogits in its forward
  pass, so the ``(B*T, 50304)`` fp32 probabilities are never materialised.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, asdict

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


@dataclass
class GPTConfig:
    block_size: int = 1024
    vocab_size: int = 50304  # GPT-2's 50257 padded to a multiple of 64
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    dropout: float = 0.0
    bias: bool = True

    def to_dict(self):
        return asdict(self)

    @property
    def head_dim(self):
        return self.n_embd // self.n_head


PRESETS = {
    # BASELINE.json config 1: CPU plumbing model
    "gpt2-tiny": dict(n_layer=2, n_head=2, n_embd=128, block_size=256),  # head dim 64 (HIP attention: 64/128)
    "gpt2": dict(n_layer=12, n_head=12, n_embd=768),            # 124M
    "gpt2-medium": dict(n_layer=24, n_head=16, n_embd=1024),    # 350M
    "gpt2-large": dict(n_layer=36, n_head=20, n_embd=1280),     # 774M
    "gpt2-xl": dict(n_layer=48, n_head=25, n_embd=1600),        # 1558M
}


class LayerNorm(nn.Module):
    def __init__(self, ndim, bias):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(ndim))
        self.bias = nn.Parameter(torch.zeros(ndim)) if bias else None

    def forward(self, x):
        return ops.layer_norm(x, self.weight, self.bias, 1e-5)


class CausalSelfAttention(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        assert cfg.n_embd % cfg.n_head == 0
        self.c_attn = nn.Linear(cfg.n_embd, 3 * cfg.n_embd, bias=cfg.bias)
        self.c_proj = nn.Linear(cfg.n_embd, cfg.n_embd, bias=cfg.bias)
        self.n_head = cfg.n_head
        self.dropout = cfg.dropout

    def attend(self, x):
        """QKV projection + attention, before the output projection (B, T, C); the QKV bias
        gradient is summed inside the attention backward on the HIP path."""
        return ops.linear_attention_qkv(x, self.c_attn.weight, self.c_attn.bias, self.n_head)

    def forward(self, x, fuse_out_bias=False):
        y = self.attend(x)
        # with fuse_out_bias the caller adds c_proj.bias inside its add+LayerNorm kernel
        y = ops.linear(y, self.c_proj.weight, None if fuse_out_bias else self.c_proj.bias)
        if self.dropout and self.training:
            y = F.dropout(y, self.dropout)
        return y


class MLP(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.c_fc = nn.Linear(cfg.n_embd, 4 * cfg.n_embd, bias=cfg.bias)
        self.c_proj = nn.Linear(4 * cfg.n_embd, cfg.n_embd, bias=cfg.bias)
        self.dropout = cfg.dropout

    def forward(self, x, fuse_out_bias=False):
        y = ops.mlp(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight,
                    None if fuse_out_bias else self.c_proj.bias)
        if self.dropout and self.training:
            y = F.dropout(y, self.dropout)
        return y


class Block(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.ln_1 = LayerNorm(cfg.n_embd, cfg.bias)
        self.attn = CausalSelfAttention(cfg)
        self.ln_2 = LayerNorm(cfg.n_embd, cfg.bias)
        self.mlp = MLP(cfg)

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        x = x + self.mlp(self.ln_2(x))
        return x


class GPT(nn.Module):
    """GPT-2 language model.  ``forward(idx, targets)`` -> (logits|None, loss|None)."""

    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.config = cfg
        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(cfg.vocab_size, cfg.n_embd),
            wpe=nn.Embedding(cfg.block_size, cfg.n_embd),
            h=nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)]),
            ln_f=LayerNorm(cfg.n_embd, cfg.bias),
        ))
        self.lm_head = nn.Linear(cfg.n_embd, cfg.vocab_size, bias=False)
        self.transformer.wte.weight = self.lm_head.weight  # weight tying
        self.apply(self._init_weights)
        for pn, p in self.named_parameters():
            if pn.endswith("c_proj.weight"):
                nn.init.normal_(p, mean=0.0, std=0.02 / math.sqrt(2 * cfg.n_layer))

    @staticmethod
    def _init_weights(module):
        if isinstance(module, nn.Linear):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)
            if module.bias is not None:
                nn.init.zeros_(module.bias)
        elif isinstance(module, nn.Embedding):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)

    def num_params(self, non_embedding=True):
        n = sum(p.numel() for p in self.parameters())
        if non_embedding:
            n -= self.transformer.wpe.weight.numel()
        return n

    def flops_per_token(self, seq_len=None):
        """Training FLOPs per token (6N + attention), as in the PaLM MFU formula."""
        cfg = self.config
        T = seq_len or cfg.block_size
        N = self.num_params()
        return 6 * N + 12 * cfg.n_layer * cfg.n_embd * T

    def forward(self, idx, targets=None):
        B, T = idx.shape
        assert T <= self.config.block_size, f"sequence {T} > block_size {self.config.block_size}"
        blocks = self.transformer.h
        if self.config.dropout and self.training:
            tok = self.transformer.wte(idx)
            x = ops.add_broadcast(tok, self.transformer.wpe.weight[:T])
            x = F.dropout(x, self.config.dropout)
            h = blocks[0].ln_1(x)
        else:
            # token + position embedding and block 0's ln_1 in one op (ops/embedding.py)
            ln = blocks[0].ln_1
            x, h = ops.embed_layer_norm(idx, self.transformer.wte.weight, self.transformer.wpe.weight,
                                        ln.weight, ln.bias)
        # Residual stream with every "x = x + branch; h = LN(x)" pair fused into one kernel
        # (forward and backward): block i's second add feeds block i+1's ln_1 (ln_f at the end).
        # The branch output-projection biases are folded into the same kernel
        # (forward: added before the residual sum; backward: their gradient is a
        # column sum of the residual-stream gradient the kernel already holds).
        # Without dropout the branch output projections do the residual add themselves (one
        # GEMM with the bias and the old stream in its epilogue; the LayerNorm then reads only
        # the new stream: ops/residual.py).
        fused_sites = not (self.config.dropout and self.training)
        for i, block in enumerate(blocks):
            nxt = blocks[i + 1].ln_1 if i + 1 < len(blocks) else self.transformer.ln_f
            at, ml = block.attn, block.mlp
            if fused_sites:
                x, h = ops.linear_residual_layer_norm(x, at.attend(h), at.c_proj.weight, at.c_proj.bias,
                                                      block.ln_2.weight, block.ln_2.bias)
                x, h = ops.mlp_residual_layer_norm(x, h, ml.c_fc.weight, ml.c_fc.bias, ml.c_proj.weight,
                                                   ml.c_proj.bias, nxt.weight, nxt.bias)
                continue
            a = at(h, fuse_out_bias=True)
            x, h = ops.add_layer_norm(x, a, block.ln_2.weight, block.ln_2.bias, r_bias=at.c_proj.bias)
            m = ml(h, fuse_out_bias=True)
            x, h = ops.add_layer_norm(x, m, nxt.weight, nxt.bias, r_bias=ml.c_proj.bias)
        x = h
        if targets is not None:
            loss = ops.linear_cross_entropy(x.reshape(B * T, -1), self.lm_head.weight,
                                            targets.reshape(-1), ignore_index=-1)
            return None, loss
        logits = self.lm_head(x[:, [-1], :])
        return logits, None

    @torch.no_grad()
    def generate(self, idx, max_new_tokens, temperature=1.0, top_k=None):
        for _ in range(max_new_tokens):
            idx_cond = idx if idx.size(1) <= self.config.block_size else idx[:, -self.config.block_size:]
            logits, _ = self(idx_cond)
            logits = logits[:, -1, :].float() / max(temperature, 1e-6)
            if top_k is not None:
                v, _ = torch.topk(logits, min(top_k, logits.size(-1)))
                logits[logits < v[:, [-1]]] = -float("inf")
            probs = F.softmax(logits, dim=-1)
            idx_next = torch.multinomial(probs, num_samples=1)
            idx = torch.cat((idx, idx_next), dim=1)
        return idx


def build_gpt2(preset="gpt2", **overrides):
    kw = dict(PRESETS[preset])
    kw.update(overrides)
    return GPT(GPTConfig(**kw))
