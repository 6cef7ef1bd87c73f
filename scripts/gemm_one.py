#!/usr/bin/env python3
"""Run one csrc/gemm16.hip shape a few times (for rocprofv3 --pmc passes).
usage: python scripts/gemm_one.py M N K wkm epi [reps] [blas]
(blas = 1: the same product through torch / hipBLASLt with the committed TunableOp table)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

M, N, K, wkm, epi = (int(v) for v in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
blas = len(sys.argv) > 7 and sys.argv[7] == "1"
load_ext(required=True)
if blas:
    from orion_amd.tuning import use_tuned_gemms
    use_tuned_gemms()
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
w = (torch.randn(*((K, N) if wkm else (N, K)), device="cuda", generator=g) * 0.5).to(torch.bfloat16)
b = (torch.randn(N, device="cuda", generator=g)).to(torch.bfloat16) if epi in (1, 2) else None
pre = (torch.randn(M, N, device="cuda", generator=g)).to(torch.bfloat16) if epi == 3 else None
for _ in range(reps):
    if blas:
        _ = x @ w if wkm else torch.nn.functional.linear(x, w, b)
    else:
        C().gemm(x, w, bool(wkm), epi, b, pre)
torch.cuda.synchronize()
