"""Direct-to-arena weight gradients.

With a flat gradient arena (``train/flat.py``) every parameter's ``.grad`` is a view
into one buffer.  Returning a weight gradient from an autograd ``Function`` makes
PyTorch's ``AccumulateGrad`` run ``p.grad += dW`` -- a separate elementwise kernel that
re-reads the new gradient and the arena slice and writes the slice back (for
Llama-7B at 16k tokens per micro-batch: ~20 ms per step, ~2.4 % of it).

Instead, the arena attaches a :class:`GradSink` to each parameter it owns, and the
GEMM-backed backward functions (``ops.layernorm._Linear``, the fused LM head in
``ops.xent``) write ``dW`` straight into the arena slice -- overwriting it on the first
write of a step, accumulating in the GEMM epilogue afterwards (gradient accumulation
over micro-batches) -- and return ``None`` for the weight.  Because no
``AccumulateGrad`` runs, the sink then notifies the arena's gradient listeners (the
data-parallel reducer's bucket counter) itself.

Tied parameters (used by ``uses`` > 1 modules, e.g. GPT-2's ``wte`` = LM head) get a sink
too: the first write of a step overwrites, every later one accumulates (``take``).  A
producer that is not the parameter's last use in the backward (the LM head) calls
``notify()``, which only counts.  The last use (GPT-2's fused embedding, the final kernel of
the backward) calls ``notify(last=True)``: the parameter is reported once every ``expect``
producer of this micro-step has written through the sink.  When some use of the micro-step
did not (a dropout path's plain embedding goes through ``AccumulateGrad`` and the arena's
fold hook, and never calls ``notify(last=True)``), nothing is reported here and the
post-accumulate-grad hook reports the parameter after that last contribution instead.
Either way a data-parallel bucket is never launched between the LM head's and the
embedding's writes -- and, since ``AccumulateGrad`` runs no hook for an undefined
gradient, the all-sink case is reported during the backward rather than only at
``finish()``.
``ORION_DIRECT_GRADS=0`` disables the mechanism.
"""
from __future__ import annotations

import os
import weakref

import torch

ENABLED = os.environ.get("ORION_DIRECT_GRADS", "1") != "0"


class GradSink:
    __slots__ = ("view", "fresh", "expect", "notes", "_micro", "_param", "_listeners",
                 "tail", "tail_cb", "__weakref__")

    def __init__(self, param: torch.Tensor, view: torch.Tensor, listeners: list, expect: int = 1):
        self.view = view            # the parameter's slice of the gradient arena, param-shaped
        self.fresh = True           # no write yet this step -> the next write may overwrite
        self.expect = expect        # producers per micro-step (uses of a tied parameter)
        self.notes = 0              # notify() calls since the step began
        self._micro = 0             # notify() calls since the last use's notify(last=True)
        self._param = weakref.ref(param)
        self._listeners = listeners  # shared with the owning arena
        # split tied gradient (parallel/ddp.py, tied_bf16): while set by the data-parallel
        # reducer, the LAST use writes its contribution here (param-shaped fp32, overwritten)
        # instead of accumulating into ``view``, the earlier uses' notify() reports the
        # parameter at once (its arena bucket can be reduced under the rest of the backward)
        # and the last use's notify(last=True) calls ``tail_cb(param)``
        self.tail = None
        self.tail_cb = None

    def reset(self):
        """Start of an optimizer step (the arena's zero_grad)."""
        self.fresh = True
        self.notes = 0
        self._micro = 0

    def take(self) -> bool:
        """Claim the slice for one write; returns True if the write must accumulate."""
        acc = not self.fresh
        self.fresh = False
        return acc

    def last_use_target(self):
        """(tensor, accumulate) for the parameter's LAST use (the embedding of a tied table):
        the split tail when the reducer set one (overwrite), else the arena slice
        (``take()``)."""
        if self.tail is not None:
            return self.tail, False
        return self.view, self.take()

    def notify(self, last: bool = False):
        """One producer wrote its gradient through the sink.  ``last``: the producer is the
        parameter's last use in the backward (only meaningful for tied parameters)."""
        self.notes += 1
        self._micro += 1
        if self.expect > 1 and self.tail is not None:
            p = self._param()
            if p is None:
                return
            if last:
                self._micro = 0
                self.tail_cb(p)
            else:
                for cb in self._listeners:
                    cb(p)
            return
        if self.expect > 1:
            if not last:
                return
            complete = self._micro >= self.expect
            self._micro = 0
            if not complete:  # some use went through AccumulateGrad: its hook reports
                return
        p = self._param()
        if p is not None:
            for cb in self._listeners:
                cb(p)


def attach(param: torch.Tensor, view: torch.Tensor, listeners: list,
           expect: int = 1) -> GradSink | None:
    if not ENABLED or view.dtype not in (torch.bfloat16, torch.float32) or not view.is_cuda:
        return None
    sink = GradSink(param, view, listeners, expect)
    param._orion_sink = sink
    return sink


def detach(param: torch.Tensor):
    if hasattr(param, "_orion_sink"):
        del param._orion_sink


def sink_of(param: torch.Tensor) -> GradSink | None:
    """The arena sink of ``param``, or None (not arena-owned, tied, or disabled)."""
    return getattr(param, "_orion_sink", None)


def claim(param: torch.Tensor | None) -> GradSink | None:
    """The sink of ``param`` if its gradient can be written straight into the arena by the
    next kernel: only the first write of a step (it overwrites).  Later writes (gradient
    accumulation) return the gradient and take the ``AccumulateGrad`` path instead.  The
    caller passes ``sink.view`` as the kernel's output, then calls ``sink.notify()`` and
    returns ``None`` for that gradient."""
    sk = None if param is None else sink_of(param)
    if sk is None or not sk.fresh:
        return None
    sk.fresh = False
    return sk
