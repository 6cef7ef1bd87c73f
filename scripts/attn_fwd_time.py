#!/usr/bin/env python3
"""Forward-attention timing on one shape (median of N launches, random data); prints one
JSON line.  Pair with ORION_ATTN_FWD=v2 for a same-box A/B of the two forward kernels.
usage: python scripts/attn_fwd_time.py B T Hq Hkv D [iters]"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

B, T, Hq, Hkv, D = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 30
load_ext(required=True)
torch.manual_seed(0)
qkv = torch.randn(B, T, Hq + 2 * Hkv, D, device="cuda", dtype=torch.bfloat16)
q, k, v = qkv[:, :, :Hq], qkv[:, :, Hq:Hq + Hkv], qkv[:, :, Hq + Hkv:]
sc = 1 / math.sqrt(D)
for _ in range(3):
    C().attn_fwd(q, k, v, True, sc)
torch.cuda.synchronize()
ts = []
for _ in range(iters):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    C().attn_fwd(q, k, v, True, sc)
    b.record()
    b.synchronize()
    ts.append(a.elapsed_time(b))
ts.sort()
ms = ts[len(ts) // 2]
flops = 2 * 2 * B * Hq * T * T * D * 0.5
print(json.dumps(dict(kernel=os.environ.get("ORION_ATTN_FWD", "v3"), B=B, T=T, Hq=Hq, Hkv=Hkv, D=D,
                      fwd_ms=round(ms, 4), TFs=round(flops / ms / 1e9, 1))))
