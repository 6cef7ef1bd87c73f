#!/usr/bin/env python3
"""Co-residency of a second stream's kernel with gemm16.

In a data-parallel step RCCL's reduction kernels run on their own stream while the backward
GEMMs fill the GPU.  gemm16 is one 512-thread workgroup per CU holding all 160 KB of LDS and
~2 x 232 of the 512 VGPRs per SIMD lane, so nothing that needs LDS can share a CU with it: a
kernel on another stream gets a CU only when a gemm16 workgroup retires.  With one workgroup
per work item that happens every item (~20 us); with the persistent walk only at the end of
the whole GEMM.  This measures it on one GPU: a chain of backward-shaped GEMMs on a normal
stream, and, 1 ms into it, a memory-bound kernel (a 64 MB copy, about what one ring step of a
large bucket moves) on a HIGH-priority stream; the copy's time from its stream reaching it to
its end (events) against the same copy alone; then the same with a 64 MB sum (a reduction
kernel with an LDS stage, like RCCL's collectives).  Prints one JSON line per probe and GEMM
mode.

usage: python scripts/coresidency.py [--reps 5]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
load_ext(required=True)
ops = C()
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(torch.bfloat16)  # noqa: E731
M = 65536
dy, w = rnd(M, 768), rnd(768, 3072)       # fc input gradient shape (K = 768, N = 3072)
xf, wf = rnd(M, 768), rnd(768, 3072)      # fc forward shape for the hipBLASLt chain
src = torch.empty(32 * 1024 * 1024, device="cuda", dtype=torch.bfloat16)
dst = torch.empty_like(src)
hi = torch.cuda.Stream(priority=-1)      # the high-priority stream (RCCL's own stream is one)
lo = torch.cuda.current_stream()


acc = torch.empty((), device="cuda", dtype=torch.float32)


def probe(kind):
    """the second-stream kernel: a 64 MB copy (no LDS) or a 64 MB sum (a reduction kernel
    with an LDS stage, as RCCL's collectives have)"""
    if kind == "copy":
        dst.copy_(src)
    else:
        torch.sum(src, dim=0, dtype=torch.float32, out=acc)


def copy_alone(kind="copy"):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(hi):
        e0.record()
        probe(kind)
        e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1)


def copy_beside_gemms(kind="copy", blas=False):
    def one():
        if blas:
            torch.mm(xf, wf)
        else:
            ops.gemm(dy, w, True, 0, None, None)
    for _ in range(2):
        one()
    torch.cuda.synchronize()
    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g0.record(lo)
    for _ in range(12):                   # ~5 ms of GEMMs
        one()
    g1.record(lo)
    time.sleep(0.001)                     # the copy arrives mid-chain
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(hi):
        e0.record()
        probe(kind)
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1), g0.elapsed_time(g1)


for kind in ("copy", "sum"):
    for _ in range(3):
        copy_alone(kind)
    alone = sorted(copy_alone(kind) for _ in range(10))[5]
    for mode, flags in (("persistent", 0), ("per_item", 64), ("hipblaslt", 0)):
        ops.gemm_diag(flags)
        res = [copy_beside_gemms(kind, mode == "hipblaslt") for _ in range(a.reps)]
        ops.gemm_diag(0)
        cp = sorted(r[0] for r in res)
        gm = sorted(r[1] for r in res)
        print(json.dumps({"probe": kind, "gemm_mode": mode, "probe_alone_ms": round(alone, 4),
                          "probe_beside_gemm_ms_median": round(cp[len(cp) // 2], 4),
                          "probe_beside_gemm_ms_max": round(cp[-1], 4),
                          "gemm_chain_ms_median": round(gm[len(gm) // 2], 3)}), flush=True)
