"""Error budgets for the GPU kernel tests, pinned to what stock PyTorch in bf16 achieves.

A fixed relative-error threshold (3e-2, 8e-2, ...) against an fp32 reference says nothing
about whether a kernel is as accurate as it should be: bf16 rounding of the output alone is
~4e-3, so an error that corrupts a few percent of one tile would still pass (VERDICT r3,
weak item 8).  Every kernel test therefore also computes the same op with stock PyTorch on
the bf16 inputs (PyTorch's own bf16 kernels: F.layer_norm, F.scaled_dot_product_attention,
matmul, ...) and asserts

    err(HIP vs fp32 reference) <= FACTOR * err(PyTorch-bf16 vs fp32 reference) + FLOOR

with FACTOR = 2 and FLOOR = 1e-3: the in-tree kernel may be at most twice as far from the
exact result as PyTorch's bf16 path is, plus a small absolute floor for outputs whose bf16
baseline is exact (e.g. sums that round the same way).
"""
from __future__ import annotations

import torch

FACTOR = 2.0
FLOOR = 1e-3


def rel_err(a, b) -> float:
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def within_bf16_budget(name, got, ref32, base_bf16, factor=FACTOR, floor=FLOOR):
    """Assert the budget above for one tensor; returns (err, baseline err)."""
    e = rel_err(got, ref32)
    b = rel_err(base_bf16, ref32)
    assert e <= factor * b + floor, (f"{name}: rel err {e:.3e} vs fp32 exceeds {factor} x the "
                                     f"PyTorch-bf16 error {b:.3e} + {floor:.0e}")
    return e, b


def check_all(names, gots, refs, bases, factor=FACTOR, floor=FLOOR):
    """``within_bf16_budget`` over parallel sequences (outputs and gradients)."""
    out = {}
    for n, g, r, b in zip(names, gots, refs, bases):
        out[n] = within_bf16_budget(n, g, r, b, factor, floor)
    return out


def torch_bf16(fn, inputs, grad_out=None):
    """Run ``fn`` (stock PyTorch ops) on detached bf16 copies of ``inputs`` (tensors that
    require grad get grads) -> (output, [input grads]).  The bf16 baseline of a test."""
    xs = [t.detach().to(torch.bfloat16).requires_grad_(t.requires_grad) if torch.is_tensor(t) else t
          for t in inputs]
    y = fn(*xs)
    grads = []
    if grad_out is not None:
        y.backward(grad_out.to(y.dtype))
        grads = [x.grad if torch.is_tensor(x) and x.requires_grad else None for x in xs]
    return y, grads
