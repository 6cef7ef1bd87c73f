#!/usr/bin/env python3
"""Time the fused AdamW over a flat fp32 arena of N parameters (default GPT-2-124M's padded
arena), median of 20; prints one JSON line with the effective HBM rate (30 bytes / param).
usage: python scripts/time_adamw.py [N]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 124475392
n -= n % 2048
load_ext(required=True)
dev = "cuda"
p16 = torch.zeros(n, dtype=torch.bfloat16, device=dev)
master, m, v, g = (torch.randn(n, device=dev) for _ in range(4))
v.abs_()
decay = torch.ones(n // 2048, dtype=torch.uint8, device=dev)
hyper = torch.tensor([6e-4, 0.9, 0.95, 1e-8, 0.1, 0.1, 0.05, 0.0], device=dev)
sumsq = torch.ones(1, device=dev)
for _ in range(3):
    C().adamw_flat(p16, master, m, v, g, decay, hyper, sumsq)
torch.cuda.synchronize()
ts = []
for _ in range(20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    C().adamw_flat(p16, master, m, v, g, decay, hyper, sumsq)
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
t = sorted(ts)[10]
print(json.dumps({"n": n, "ms": round(t, 4), "TBs": round(30.0 * n / t / 1e9, 2)}))
