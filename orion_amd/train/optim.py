"""Fused AdamW over a :class:`~orion_amd.train.flat.FlatArena`.

State layout: fp32 master weights, fp32 ``exp_avg`` and ``exp_avg_sq``, all
flat and aligned with the arena.  One step on the GPU is two kernels:

1. ``grad_sumsq``  -- one pass over the gradient arena, result stays on device;
2. ``adamw_flat``  -- reads grad (bf16), master/m/v (fp32), the weight-decay
   flag of each 2048-element chunk and the clip coefficient derived from (1);
   writes master/m/v and the bf16 compute copy.  No host synchronisation, so
   the whole training step can be captured in a HIP graph.

The math is exactly ``torch.optim.AdamW`` (decoupled weight decay, bias
correction) applied after global-norm gradient clipping.
"""
from __future__ import annotations

import math

import torch

from ..ops._ext import C
from .flat import FlatArena, ALIGN


class FlatAdamW:
    def __init__(self, arena: FlatArena, lr=6e-4, betas=(0.9, 0.95), eps=1e-8,
                 weight_decay=0.1, grad_clip=1.0):
        self.arena = arena
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.grad_clip = grad_clip
        self.step_count = 0
        dev = arena.device
        init = getattr(arena, "init_fp32", None)
        self.master = init if init is not None else arena.params.float().clone()
        arena.init_fp32 = None
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        # device-resident step scalars so a captured graph replays with fresh values
        self._hyper = torch.zeros(8, dtype=torch.float32, device=dev)
        self._use_hip = dev.type == "cuda"
        self._decay_mask = None
        # ZeRO-1: the squared gradient norm of this rank's shard is summed over the ranks
        # (in place, on the device) before it sets the clip coefficient
        self.sumsq_hook = None

    # ------------------------------------------------------------------ helpers
    def _decay_mask_full(self):
        if self._decay_mask is None:
            self._decay_mask = self.arena.decay_flags.repeat_interleave(ALIGN).to(torch.float32)
        return self._decay_mask

    def set_lr(self, lr):
        self.lr = lr

    def hyper_tensor(self):
        """Fill the device hyper-parameter vector for the NEXT step (host -> device)."""
        t = self.step_count + 1
        b1, b2 = self.betas
        # pinned + non_blocking: a pageable copy would make the host wait for the whole
        # backward before it launched the optimizer (a ~40 us idle gap per step in the kernel
        # trace); the caching host allocator keeps the pinned block until its copy has run
        vals = torch.tensor([self.lr, b1, b2, self.eps, self.weight_decay,
                             1.0 - b1 ** t, 1.0 - b2 ** t,
                             self.grad_clip if self.grad_clip else 0.0], dtype=torch.float32,
                            pin_memory=self._use_hip)
        self._hyper.copy_(vals, non_blocking=self._use_hip)
        return self._hyper

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def step(self, hyper_prefilled=False):
        a = self.arena
        if self._use_hip:
            if not hyper_prefilled:
                self.hyper_tensor()
            ops = C()
            ops.grad_sumsq(a.grads, self._sumsq)
            if self.sumsq_hook is not None:
                self.sumsq_hook(self._sumsq)
            ops.adamw_flat(a.params, self.master, self.exp_avg, self.exp_avg_sq, a.grads,
                           a.decay_flags, self._hyper, self._sumsq)
        else:
            self._step_reference()
        self.step_count += 1

    def _step_reference(self):
        a = self.arena
        g = a.grads.float()
        sumsq = (g * g).sum().reshape(1)
        if self.sumsq_hook is not None:
            self.sumsq_hook(sumsq)
        self._sumsq.copy_(sumsq)
        if self.grad_clip:
            norm = float(sumsq.sqrt())
            g = g * min(1.0, self.grad_clip / (norm + 1e-6))
        b1, b2 = self.betas
        t = self.step_count + 1
        decay = self._decay_mask_full()
        self.master.mul_(1.0 - self.lr * self.weight_decay * decay)
        self.exp_avg.mul_(b1).add_(g, alpha=1 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (self.exp_avg_sq / (1 - b2 ** t)).sqrt_().add_(self.eps)
        self.master.addcdiv_(self.exp_avg, denom, value=-self.lr / (1 - b1 ** t))
        a.params.copy_(self.master)

    def grad_norm(self):
        """Global L2 gradient norm of the last step (syncs)."""
        return math.sqrt(float(self._sumsq))

    def state_dict(self):
        return dict(step=self.step_count, lr=self.lr, betas=self.betas, eps=self.eps,
                    weight_decay=self.weight_decay, grad_clip=self.grad_clip,
                    master=self.master, exp_avg=self.exp_avg, exp_avg_sq=self.exp_avg_sq)

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.lr = sd["lr"]
        self.betas = tuple(sd["betas"])
        self.eps = sd["eps"]
        self.weight_decay = sd["weight_decay"]
        self.grad_clip = sd["grad_clip"]
        self.master.copy_(sd["master"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.arena.params.copy_(self.master)
