#!/usr/bin/env python3
"""Time Llama-7B's down_proj input gradient with the SwiGLU' epilogue (gemm16 EPI_SWIGLU_BWD,
M = 16,384 tokens, K = 4,096, F = 11,008) and the same GEMM with a plain store, median of 20;
one JSON line.  usage: python scripts/time_swiglu_bwd.py [M K F]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

M, K, F = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (16384, 4096, 11008)
load_ext(required=True)
g = torch.Generator(device="cuda").manual_seed(0)
dy = (torch.randn(M, K, device="cuda", generator=g) * 0.1).bfloat16()
w = (torch.randn(K, F, device="cuda", generator=g) * 0.02).bfloat16()
gu = torch.randn(M, 2 * F, device="cuda", generator=g).bfloat16()


def med(f):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[10]


t = med(lambda: C().gemm_swiglu_bwd(dy, w, gu))
from orion_amd.ops.gemm import linear_dgrad  # noqa: E402
t0 = med(lambda: linear_dgrad(dy, w))  # the same GEMM, plain bf16 store (no epilogue operands)
print(json.dumps({"ms": round(t, 4), "PFs": round(2.0 * M * K * F / t / 1e12, 3), "plain_ms": round(t0, 4)}))
