"""Flat parameter / gradient arenas.

All trainable parameters of a model are re-homed into ONE contiguous bf16
buffer (what the GEMMs read) and their gradients into ONE contiguous buffer
(what autograd accumulates into and what RCCL reduces).  Consequences:

* the optimizer is a single fused HIP kernel over ``numel`` elements, not a
  multi-tensor launch per parameter;
* data-parallel gradient buckets are contiguous *slices* of the gradient
  arena -- an all-reduce needs no copy-in/copy-out;
* every parameter starts at a multiple of ``ALIGN`` elements, so the fused
  AdamW kernel can look up a parameter's weight-decay flag per 2048-element
  chunk with one byte load.

Gradient dtype: the gradient arena is fp32 by default on the GPU (``Trainer``), so
accumulation over micro-batches and the data-parallel all-reduce keep fp32
precision (nanoGPT's fp32-gradient numerics) while the compute copy of the weights
stays bf16.  A bf16 parameter cannot have an fp32 ``.grad``, so in that mode
``p.grad`` is NOT bound to the arena: weight gradients reach their fp32 slice
through the parameter's :class:`~orion_amd.ops.grad_sink.GradSink` (the GEMM /
reduction kernel writes the slice directly, overwriting on the first write of a
step and accumulating in its epilogue afterwards), and any gradient that still
arrives through ``AccumulateGrad`` (tied weights, embeddings, ops without a sink)
is folded into the slice by a post-accumulate hook and released.
``grad_dtype=torch.bfloat16`` restores the all-bf16 arena.

Parameters are laid out in *reverse* module-registration order, which is
approximately the order backward produces their gradients, so the gradient
buckets at the front of the arena fill first (see ``parallel/ddp.py``).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from ..ops import grad_sink

ALIGN = 2048  # elements; also the AdamW weight-decay chunk size


def _round_up(n, a):
    return (n + a - 1) // a * a


@dataclass
class ParamSlot:
    name: str
    param: nn.Parameter
    offset: int
    numel: int
    decay: bool


def arena_order(model: nn.Module):
    """(name, parameter) pairs in arena order -- trainable, deduplicated, reverse registration
    order -- and the number of uses of each parameter (id -> count; > 1 for tied weights)."""
    uses: dict[int, int] = {}
    for _, p in model.named_parameters(remove_duplicate=False):
        uses[id(p)] = uses.get(id(p), 0) + 1
    seen = set()
    named = []
    for name, p in model.named_parameters():
        if not p.requires_grad or id(p) in seen:
            continue
        seen.add(id(p))
        named.append((name, p))
    named.reverse()
    return named, uses


class FlatArena:
    """Owns the flat param/grad buffers of ``model``; rebinds ``p.data``/``p.grad``.

    ``pad_after`` / ``pad_to``: after each named parameter the next offset is rounded up to a
    multiple of ``pad_to`` elements (ZeRO-1: every data-parallel bucket then splits into
    ``world`` equal, ALIGN-aligned shards; ``parallel/ddp.py``)."""

    SKIP_ZERO_MIN = 1 << 16  # elements: sink slices at least this large are not pre-zeroed

    def __init__(self, model: nn.Module, dtype=torch.bfloat16, grad_dtype=None,
                 device=None, decay_filter=None, pad_after=(), pad_to: int = ALIGN):
        device = device or next(model.parameters()).device
        grad_dtype = grad_dtype or dtype
        decay_filter = decay_filter or (lambda name, p: p.dim() >= 2)
        named, uses = arena_order(model)
        pad_after = set(pad_after)
        if pad_to % ALIGN:
            raise ValueError(f"pad_to must be a multiple of {ALIGN}")
        slots, off = [], 0
        for name, p in named:
            slots.append(ParamSlot(name, p, off, p.numel(), bool(decay_filter(name, p))))
            off = _round_up(off + p.numel(), pad_to if name in pad_after else ALIGN)
        self.numel = off
        self.slots = slots
        # parameters used by more than one module (GPT-2's wte / LM head): their gradient is
        # complete only after the LAST use's backward (the embedding, at the very end)
        self.shared = {id(p) for _, p in named if uses.get(id(p), 1) > 1}
        self.dtype = dtype
        self.grad_dtype = grad_dtype
        self.device = device
        self.params = torch.zeros(off, dtype=dtype, device=device)
        self.grads = torch.zeros(off, dtype=grad_dtype, device=device)
        # p.grad can alias the arena only when the dtypes agree (see module docstring)
        self.bound = grad_dtype == dtype
        # per-ALIGN-chunk weight-decay flag (uint8) consumed by the fused AdamW kernel
        flags = torch.zeros(off // ALIGN, dtype=torch.uint8)
        for s in slots:
            if s.decay:
                flags[s.offset // ALIGN: _round_up(s.offset + s.numel, ALIGN) // ALIGN] = 1
        self.decay_flags = flags.to(device)
        # exact fp32 copy of the initial weights: seeds the optimizer's master weights
        # (the compute arena itself is rounded to ``dtype``); released by the optimizer
        self.init_fp32 = torch.zeros(off, dtype=torch.float32, device=device)
        with torch.no_grad():
            for s in slots:
                view = self.params[s.offset: s.offset + s.numel].view_as(s.param)
                view.copy_(s.param.data)
                self.init_fp32[s.offset: s.offset + s.numel].copy_(s.param.data.reshape(-1))
                s.param.data = view
                s.param.grad = self.grad_view(s).view_as(s.param) if self.bound else None
        # direct-to-arena weight gradients (ops/grad_sink.py); a tied parameter's sink expects
        # one producer per use
        self.grad_listeners: list = []
        self.sinks = []
        for s in slots:
            sk = grad_sink.attach(s.param, self.grad_view(s).view_as(s.param),
                                  self.grad_listeners, expect=uses.get(id(s.param), 1))
            if sk is not None:
                self.sinks.append(sk)
        # zero_grad skips the slices of large sink-written weights: their first write of a
        # step overwrites (GradSink.fresh), so zeroing them first is a wasted HBM pass (27 GB
        # per step for Llama-7B's fp32 arena).  Everything else -- padding, small and tied
        # parameters, AccumulateGrad targets -- is zeroed with one multi-tensor launch;
        # ``finish_grads`` zeroes any skipped slice that no kernel wrote this step.
        skip = sorted((s.offset, s.offset + s.numel) for s in slots
                      if getattr(s.param, "_orion_sink", None) is not None
                      and s.numel >= self.SKIP_ZERO_MIN)
        self._skipped = [s.param._orion_sink for s in slots
                         if getattr(s.param, "_orion_sink", None) is not None
                         and s.numel >= self.SKIP_ZERO_MIN]
        self._zero_views, pos = [], 0
        for a, b in skip + [(off, off)]:
            if a > pos:
                self._zero_views.append(self.grads[pos:a])
            pos = max(pos, b)
        # a skipped slice can still receive an AccumulateGrad result (an embedding: no kernel
        # writes its sink): the pre-accumulate hook zeroes it first if nothing wrote it yet
        self._prezero_hooks = [sk._param().register_hook(self._make_prezero(sk))
                               for sk in self._skipped]
        # unbound mode: fold AccumulateGrad results into the fp32 slice (registered before
        # any reducer hook, so the reducer sees the folded slice)
        self._fold_hooks = []
        if not self.bound:
            for s in slots:
                self._fold_hooks.append(s.param.register_post_accumulate_grad_hook(
                    self._make_fold(self.grad_view(s))))

    @staticmethod
    def _make_prezero(sk):
        def prezero(g):
            if sk.fresh:
                sk.view.zero_()
                sk.fresh = False
            return None
        return prezero

    @staticmethod
    def _make_fold(dst):
        def fold(p):
            g = p.grad
            if g is not None:
                dst.add_(g.reshape(-1))
                p.grad = None
        return fold

    def param_view(self, slot: ParamSlot):
        return self.params[slot.offset: slot.offset + slot.numel]

    def grad_view(self, slot: ParamSlot):
        return self.grads[slot.offset: slot.offset + slot.numel]

    def zero_grad(self):
        if len(self._zero_views) == 1 and self._zero_views[0].numel() == self.numel:
            self.grads.zero_()
        elif self._zero_views:
            torch._foreach_zero_(self._zero_views)
        for sk in self.sinks:
            sk.reset()

    def finish_grads(self):
        """After the last backward of a step: zero the skipped sink slices that no kernel
        wrote (parameters unused this step)."""
        for sk in self._skipped:
            if sk.fresh:
                sk.view.zero_()

    def detach_sinks(self):
        """Stop direct gradient writes (params then take the AccumulateGrad path)."""
        for s in self.slots:
            grad_sink.detach(s.param)
        self.sinks = []
        self._skipped = []
        self._zero_views = [self.grads]
        for h in self._prezero_hooks:
            h.remove()
        self._prezero_hooks = []

    def rebind_grads(self):
        """Re-point ``p.grad`` at the arena (after anything replaced it); unbound arenas
        (fp32 gradients for bf16 parameters) keep ``p.grad`` empty instead."""
        for s in self.slots:
            if not self.bound:
                s.param.grad = None
                continue
            g = s.param.grad
            if g is None or g.data_ptr() != self.grads[s.offset:].data_ptr():
                s.param.grad = self.grads[s.offset: s.offset + s.numel].view_as(s.param)

    def state_dict_fp32(self, master: torch.Tensor | None = None):
        src = master if master is not None else self.params
        return {s.name: src[s.offset: s.offset + s.numel].view(s.param.shape).float().clone()
                for s in self.slots}
