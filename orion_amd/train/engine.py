"""Training-step engine: flat bf16 arena + fused AdamW + optional RCCL DDP.

``Trainer.step(batches)`` runs ``len(batches)`` micro-steps of forward and
backward (gradient accumulation into the flat arena), reduces gradients across
data-parallel ranks with backward overlap on the last micro-step, then applies
one fused AdamW step.  Nothing in the step synchronises with the host; the loss
is returned as a device tensor.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .flat import FlatArena
from .optim import FlatAdamW


@dataclass
class OptimConfig:
    learning_rate: float = 6e-4
    weight_decay: float = 0.1
    beta1: float = 0.9
    beta2: float = 0.95
    grad_clip: float = 1.0
    warmup_iters: int = 2000
    lr_decay_iters: int = 600000
    min_lr: float = 6e-5
    decay_lr: bool = True


def cosine_lr(it: int, cfg: OptimConfig) -> float:
    """nanoGPT's schedule: linear warmup, cosine decay to min_lr."""
    if not cfg.decay_lr:
        return cfg.learning_rate
    if it < cfg.warmup_iters:
        return cfg.learning_rate * (it + 1) / (cfg.warmup_iters + 1)
    if it > cfg.lr_decay_iters:
        return cfg.min_lr
    ratio = (it - cfg.warmup_iters) / max(1, cfg.lr_decay_iters - cfg.warmup_iters)
    coeff = 0.5 * (1.0 + math.cos(math.pi * ratio))
    return cfg.min_lr + coeff * (cfg.learning_rate - cfg.min_lr)


class Trainer:
    def __init__(self, model: torch.nn.Module, optim: OptimConfig | None = None,
                 ddp: bool | None = None, bucket_mb: float = 64.0, arena_dtype=None):
        self.model = model
        self.cfg = optim or OptimConfig()
        dev = next(model.parameters()).device
        if arena_dtype is None:
            arena_dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
        self.arena = FlatArena(model, dtype=arena_dtype)
        self.opt = FlatAdamW(self.arena, lr=self.cfg.learning_rate,
                             betas=(self.cfg.beta1, self.cfg.beta2),
                             weight_decay=self.cfg.weight_decay, grad_clip=self.cfg.grad_clip)
        if ddp is None:
            ddp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.reducer = None
        if ddp:
            from ..parallel.ddp import GradBucketReducer
            self.reducer = GradBucketReducer(self.arena, bucket_mb=bucket_mb)
            # R1: every rank starts from rank 0's exact fp32 weights
            dist.broadcast(self.opt.master, 0)
            with torch.no_grad():
                self.arena.params.copy_(self.opt.master)
        self.iter_num = 0

    def step(self, batches):
        """batches: sequence of (idx, targets) micro-batches.  Returns mean loss (device)."""
        self.opt.set_lr(cosine_lr(self.iter_num, self.cfg))
        self.arena.zero_grad()
        n = len(batches)
        losses = []
        for i, (x, y) in enumerate(batches):
            if self.reducer is not None:
                self.reducer.set_sync(i == n - 1)
            _, loss = self.model(x, y)
            (loss / n).backward()
            losses.append(loss.detach())
        if self.reducer is not None:
            self.reducer.finish()
        self.opt.step()
        self.iter_num += 1
        return torch.stack(losses).mean()

    def state_dict(self):
        return dict(model=self.arena.state_dict_fp32(self.opt.master),
                    optimizer=self.opt.state_dict(), iter_num=self.iter_num)
