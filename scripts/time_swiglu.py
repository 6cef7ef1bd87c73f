#!/usr/bin/env python3
"""Time swiglu_fwd over Llama-7B's gate|up activations (16,384 tokens x 2 x 11,008), median
of 20; prints one JSON line with the effective HBM rate (reads gate|up, writes h).
usage: python scripts/time_swiglu.py [tokens]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

load_ext(required=True)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
F = 11008
gu = torch.randn(M, 2 * F, device="cuda").bfloat16()
for _ in range(3):
    C().swiglu_fwd(gu)
torch.cuda.synchronize()
ts = []
for _ in range(20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    C().swiglu_fwd(gu)
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
t = sorted(ts)[10]
print(json.dumps({"M": M, "F": F, "ms": round(t, 4), "TBs": round(3 * 2.0 * M * F / t / 1e9, 2)}))
