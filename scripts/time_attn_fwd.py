#!/usr/bin/env python3
"""Time the flash-attention forward alone on one shape (median of 30), one JSON line.
usage: python scripts/time_attn_fwd.py [B T H D]   (default: GPT-2's 64 1024 12 64)"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

B, T, H, D = (int(v) for v in sys.argv[1:5]) if len(sys.argv) > 4 else (64, 1024, 12, 64)
load_ext(required=True)
torch.manual_seed(0)
qkv = torch.randn(B, T, 3 * H, D, device="cuda", dtype=torch.bfloat16)
q, k, v = qkv[:, :, :H], qkv[:, :, H:2 * H], qkv[:, :, 2 * H:]
sc = 1 / math.sqrt(D)
for _ in range(3):
    C().attn_fwd(q, k, v, True, sc)
torch.cuda.synchronize()
ts = []
for _ in range(30):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    C().attn_fwd(q, k, v, True, sc)
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
t = sorted(ts)[15]
print(json.dumps({"B": B, "T": T, "H": H, "D": D, "fwd_ms": round(t, 4),
                  "TFs": round(4 * B * H * T * T / 2 * D / t / 1e9, 1)}))
