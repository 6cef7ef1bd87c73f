"""Linear-layer GEMMs: forward x W^T (+ bias), input gradient dy W, weight gradient dy^T x.

The in-tree kernel is ``csrc/gemm16.hip`` (v_mfma_f32_16x16x32_bf16, 256 x 256 tiles, one
persistent 512-thread workgroup per CU walking its work items with one continuous LDS-DMA
stream, fused bias / GELU / GELU' / column-sum epilogues).  It serves:

* every input gradient (``linear_dgrad``) and the fused MLP GEMMs (ops/activations.py);
* every weight gradient (``wgrad`` / ``wgrad_into``: k-major operands, split-K work items
  into fp32 slabs folded by ``slab_sum``, or straight into the fp32 gradient arena);
* the plain forwards under ``ORION_GEMM=hip``, inside a HIP-graph capture (``hip_gemms()``)
  and in the deterministic mode -- otherwise the plain forwards run on hipBLASLt
  (``ORION_GEMM=auto``, the default; profiles/gemm16/).

``csrc/wgrad.hip`` keeps one MFMA weight-gradient kernel for token counts that are not a
multiple of 64 (gemm16 stages 64-token k-tiles).  ``ORION_WGRAD=bmm`` is the library
alternative (batched hipBLASLt GEMM over token chunks + ``slab_sum``), kept for A/B runs.
"""
from __future__ import annotations

import contextlib
import os

import torch

from ._ext import C
from .determinism import deterministic

# ------------------------------------------------------------------ forward / dgrad GEMMs
# Linear-layer forward (x W^T [+ b]) and input gradient (dy W).  ORION_GEMM=auto (default):
# every input gradient on csrc/gemm16.hip, plain forward GEMMs on hipBLASLt.
# ORION_GEMM=blas: hipBLASLt for all; ORION_GEMM=hip: every eligible GEMM in-tree.  Inside a
# HIP-graph capture (``hip_gemms()``) every eligible GEMM is in-tree (no library-side host
# state between replays), and so in the deterministic mode (ops/determinism.py): one work
# item per output tile, no split-K.
_GEMM_IMPL = os.environ.get("ORION_GEMM", "auto")  # "auto" | "blas" | "hip"
_FORCE_HIP = 0

EPI_STORE, EPI_BIAS, EPI_BIAS_GELU, EPI_GELU_BWD = 0, 1, 2, 3


# GEMMs that fell back to a library call inside ``hip_gemms()`` (ineligible shape, stride or
# alignment): (kind, shape) records.  A captured HIP graph must not contain library GEMMs
# (round 1: captured hipBLASLt GEMMs faulted on replay at 65k tokens), so the trainer checks
# this after its warm-up steps and stays eager, with a warning, when anything fell back.
_FORCED_FALLBACKS: list = []


@contextlib.contextmanager
def hip_gemms():
    """Route eligible linear-layer GEMMs to the in-tree kernel (csrc/gemm16.hip) inside the
    block: a captured HIP graph then holds no library GEMM (no library-side host state)."""
    global _FORCE_HIP
    _FORCE_HIP += 1
    try:
        yield
    finally:
        _FORCE_HIP -= 1


def forced_fallbacks(clear: bool = False) -> list:
    """The library fallbacks recorded inside ``hip_gemms()`` so far (see above)."""
    out = list(_FORCED_FALLBACKS)
    if clear:
        _FORCED_FALLBACKS.clear()
    return out


def _note_fallback(kind: str, *tensors):
    if _FORCE_HIP and len(_FORCED_FALLBACKS) < 64:
        _FORCED_FALLBACKS.append((kind, tuple(tuple(t.shape) for t in tensors)))


_OFF_LIMIT = 0xFFFFFF00  # gemm16's buffer resources: 32-bit byte offsets per work item


def gemm16_addressable(ldx: int, K: int, N: int, w_kmajor: bool) -> bool:
    """csrc/gemm16.hip bases its buffer resources at the work item's tile: one 256-row band
    of X / the outputs / the pre-activation, and the whole [K][N] weight when it is k-major,
    must fit 32-bit offsets (gemm16_ok).  Outside that the caller takes hipBLASLt."""
    bands = 256 * 2 * max(ldx, N, 1)
    wb = K * N * 2 if w_kmajor else 256 * 2 * K
    return bands < _OFF_LIMIT and wb < _OFF_LIMIT


def _hip_eligible(x: torch.Tensor, w: torch.Tensor, w_kmajor: bool) -> bool:
    K = x.shape[-1]
    N = w.shape[1] if w_kmajor else w.shape[0]
    ldx = x.stride(0) if x.dim() == 2 else K
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and K % 64 == 0 and N % 8 == 0 and w.is_contiguous() and x.stride(-1) == 1
            and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0
            and (x.dim() == 2 and x.stride(0) % 8 == 0 or x.is_contiguous())
            and gemm16_addressable(ldx, K, N, w_kmajor))


# gemm16's work walk.  Persistent (default): one workgroup per CU for the whole GEMM, all
# 160 KB of LDS held.  A kernel that needs LDS -- RCCL's collectives do -- gets a CU only when a
# gemm16 workgroup exits, i.e. at the end of the GEMM; one workgroup per work item frees each CU
# every item (~20-40 us).  Under data parallelism the bucketed all-reduces / reduce-scatters
# run beside the backward GEMMs, so the trainer switches to per-item walks when it has a
# reducer over more than one rank (ORION_GEMM_DDP_PERSISTENT=1 keeps the persistent walk);
# the per-item walk costs 1-6 % on the isolated GPT-2 shapes
# (profiles/ab/gemm16_persistent_stagger_peritem_r04.log, column cfgs_TFs).
_PER_ITEM = False      # the explicit setting (set_per_item_walk)
_PER_ITEM_REFS = 0     # live requests (request_per_item_walk): DDP trainers over > 1 rank


def _apply_walk():
    on = _PER_ITEM or _PER_ITEM_REFS > 0
    cur = C().gemm_diag(-1)  # query
    C().gemm_diag((cur | 64) if on else (cur & ~64))


def set_per_item_walk(on: bool) -> bool:
    """Select gemm16's one-workgroup-per-item walk (True) or the persistent walk (False) as the
    explicit setting; live :func:`request_per_item_walk` requests keep the per-item walk on
    regardless.  Only the walk bit (64) of the diagnostic flags changes; returns the previous
    explicit setting."""
    global _PER_ITEM
    prev = _PER_ITEM
    _PER_ITEM = bool(on)
    _apply_walk()
    return prev


def request_per_item_walk():
    """Turn the per-item walk on for as long as the returned release callable has not run
    (reference counted: overlapping requesters -- two DDP trainers, say -- keep it on until
    the LAST one releases; then the explicit setting comes back).  The release is idempotent."""
    global _PER_ITEM_REFS
    _PER_ITEM_REFS += 1
    _apply_walk()
    done = []

    def release():
        global _PER_ITEM_REFS
        if done:
            return
        done.append(1)
        _PER_ITEM_REFS -= 1
        _apply_walk()
    return release


def per_item_walk() -> bool:
    return _PER_ITEM or _PER_ITEM_REFS > 0


def _hip_wins(x: torch.Tensor, w: torch.Tensor, w_kmajor: bool) -> bool:
    # Plain forwards stay on hipBLASLt.  The short-K ones (GPT-2 qkv + bias, attn-proj) are
    # faster in-tree in isolation since the persistent walk (988 / 912 vs 934 / 898 TF/s,
    # profiles/ab/gemm16_persistent_stagger_peritem_r04.log) but still slower in the step:
    # 1,085-1,088k vs 1,095-1,098k tok/s, 3 of 3 alternating pairs
    # (profiles/ab/ab_shortk_fwd_r04.log; round 3: -0.7-0.9 %, ab_fwd_shortk_r03o.log).
    return w_kmajor


def use_hip_gemm(x: torch.Tensor, w: torch.Tensor, w_kmajor: bool) -> bool:
    if _GEMM_IMPL == "blas" and not (_FORCE_HIP or deterministic()):
        return False
    forced = _FORCE_HIP or _GEMM_IMPL == "hip" or deterministic()
    if not forced and not (_GEMM_IMPL == "auto" and _hip_wins(x, w, w_kmajor)):
        return False
    return _hip_eligible(x, w, w_kmajor)


# ORION_FWD_BLASLT=1: plain forwards through the in-tree hipBLASLt wrapper (csrc/blaslt.cpp,
# every solution timed once per shape) instead of torch's hipBLASLt call (TunableOp's tuned
# pick where a table entry exists, the library heuristic otherwise); A/B knob
_FWD_BLASLT = os.environ.get("ORION_FWD_BLASLT", "0") == "1"


def linear_fwd(x, w, b=None):
    """x W^T (+ b): csrc/gemm16.hip when selected (see above), else hipBLASLt."""
    if use_hip_gemm(x, w, False):
        return C().gemm(x, w, False, EPI_BIAS if b is not None else EPI_STORE, b, None)[0]
    _note_fallback("linear_fwd", x, w)
    if (_FWD_BLASLT and x.is_contiguous() and x.dtype == w.dtype == torch.bfloat16
            and w.is_contiguous() and not deterministic()):
        y = C().linear_residual(x.reshape(-1, x.shape[-1]), w, b, None)
        return y.view(*x.shape[:-1], w.shape[0])
    return torch.nn.functional.linear(x, w, b)


def linear_dgrad(dy, w):
    """dy W for W (N_out, N_in): the input gradient of x W^T."""
    if use_hip_gemm(dy, w, True):
        return C().gemm(dy, w, True, EPI_STORE, None, None)[0]
    _note_fallback("linear_dgrad", dy, w)
    return dy @ w

# Order of a linear layer's two backward GEMMs.  Both read dY; the input gradient dX is
# consumed by the very next backward kernel (LayerNorm / GELU / attention backward), the
# weight gradient by nothing until the optimizer.  ORION_WGRAD_FIRST=1 issues the weight
# gradient first, so dX is written right before its consumer reads it and is still in the
# 256 MB Infinity Cache (the weight gradient's operand streaming would evict it otherwise).
WGRAD_FIRST = os.environ.get("ORION_WGRAD_FIRST", "0") == "1"

_FORCE = os.environ.get("ORION_WGRAD_SPLITS")
_IMPL = os.environ.get("ORION_WGRAD", "hip")  # "hip" (csrc/gemm16.hip) | "blas" | "bmm"


def _hip_ok(dy, x):
    # x row-major (M, n2), or the transposed view of a row-major (n2, M) tensor (the NT-operand
    # kernel, M % 64 == 0)
    x_rows = x.stride(1) == 1 and x.stride(0) % 8 == 0
    x_t = x.stride(0) == 1 and x.stride(1) % 8 == 0 and dy.shape[0] % 64 == 0
    return (_IMPL == "hip" and dy.is_cuda and dy.shape[0] % 32 == 0 and dy.shape[1] % 8 == 0
            and x.shape[1] % 8 == 0 and dy.stride(1) == 1 and (x_rows or x_t)
            and dy.stride(0) % 8 == 0 and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0)


def wgrad_splits(M: int, n1: int, n2: int) -> int:
    """How many token chunks to split a (n1 x n2, K = M) weight gradient into."""
    if _FORCE is not None:
        s = int(_FORCE)
        return s if s >= 1 and M % s == 0 else 1
    tiles = -(-n1 // 256) * -(-n2 // 256)
    if tiles >= 128:
        return 1  # enough output tiles already; the fp32 slab round trip would cost more
    s = 16
    while s > 1 and (M % s or M // s < 2048 or tiles * s > 1024):
        s //= 2
    return s


def _blas_wins(n1: int, n2: int) -> bool:
    """hipBLASLt for the weight gradient only when asked (ORION_WGRAD=blas): the in-tree
    kernel beats it on every measured shape -- GPT-2 (1.3-2x) and the Llama-7B shapes at 16k
    tokens (profiles/gemm16/bench_wgrad_gemm16_vs_gemm32*.log)."""
    return _IMPL == "blas" and not deterministic() and not _FORCE_HIP


def wgrad_into(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, accumulate: bool,
               scale: torch.Tensor | None = None):
    """out (n1, n2) [+]= dy^T x [* scale]: the weight gradient written straight into its
    slice of the gradient arena (``ops/grad_sink.py``)."""
    n1, n2 = dy.shape[1], x.shape[1]
    if scale is None and _blas_wins(n1, n2):
        o2 = out.view(n1, n2)
        if o2.dtype == torch.float32:  # fp32 gradient arena: hipBLASLt with fp32 output, in place
            if accumulate:
                torch.addmm(o2, dy.t(), x, out_dtype=torch.float32, out=o2)
            else:
                torch.mm(dy.t(), x, out_dtype=torch.float32, out=o2)
        elif accumulate:
            torch.addmm(o2, dy.t(), x, out=o2)
        else:
            torch.mm(dy.t(), x, out=o2)
    elif _hip_ok(dy, x):
        C().wgrad_into(dy, x, scale, out.view(n1, n2), bool(accumulate), int(_FORCE or 0))
    else:
        _note_fallback("wgrad_into", dy, x)
        g = wgrad(dy, x, scale)
        if accumulate:
            out.view(n1, n2).add_(g)
        else:
            out.view(n1, n2).copy_(g)


def wgrad(dy: torch.Tensor, x: torch.Tensor, scale: torch.Tensor | None = None) -> torch.Tensor:
    """dy (M, n1), x (M, n2) bf16 -> dy^T x (n1, n2) bf16 [times the device scalar ``scale``]."""
    if scale is None and dy.is_cuda and _blas_wins(dy.shape[1], x.shape[1]):
        return dy.t() @ x
    if _hip_ok(dy, x):
        return C().wgrad(dy, x, scale, int(_FORCE or 0))
    _note_fallback("wgrad", dy, x)
    M, n1 = dy.shape
    n2 = x.shape[1]
    S = wgrad_splits(M, n1, n2)
    if S == 1:
        dw = dy.t() @ x
        if scale is not None:
            C().scale_(dw, scale)
        return dw
    slabs = torch.bmm(dy.contiguous().view(S, M // S, n1).transpose(1, 2),
                      x.contiguous().view(S, M // S, n2), out_dtype=torch.float32)
    return C().slab_sum(slabs, scale)
