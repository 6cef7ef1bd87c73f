#!/usr/bin/env python3
"""Time the weight-gradient GEMM (csrc/wgrad.hip via gemm16) on one shape, x row-major vs
x given as the transposed view of a (N2, M) tensor (the NT-operand kernel), and hipBLASLt
(fp32 output), interleaved.
usage: python scripts/time_wgrad.py [M N1 N2] [iters]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

M, N1, N2 = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (65536, 50304, 768)
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
load_ext(required=True)
g = torch.Generator(device="cuda").manual_seed(0)
dy = (torch.randn(M, N1, device="cuda", generator=g) * 0.02).bfloat16()
x = torch.randn(M, N2, device="cuda", generator=g).bfloat16()
xt = x.t().contiguous().t()
out = torch.zeros(N1, N2, device="cuda")
fns = {"kmajor": lambda: C().wgrad_into(dy, x, None, out, False, 0),
       "nt": lambda: C().wgrad_into(dy, xt, None, out, False, 0),
       "blas": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=out)}
ts = {k: [] for k in fns}
for f in fns.values():
    f()
torch.cuda.synchronize()
for _ in range(iters):
    for k, f in fns.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        b.synchronize()
        ts[k].append(a.elapsed_time(b))
flop = 2.0 * M * N1 * N2
rec = {"M": M, "N1": N1, "N2": N2, "splits": C().wgrad_splits(M, N1, N2)}
for k, v in ts.items():
    v.sort()
    rec[f"{k}_ms"] = round(v[len(v) // 2], 4)
    rec[f"{k}_TFs"] = round(flop / v[len(v) // 2] / 1e9, 1)
print(json.dumps(rec))
