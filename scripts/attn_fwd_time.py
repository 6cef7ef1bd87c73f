#!/usr/bin/env python3
"""Attention timing on one shape (median of N launches, random data): forward and the
split backward; prints one JSON line.  Pair with ORION_ATTN_FWD=v2 (forward kernels) or
ORION_AMD_EXT=<variant .so> for same-box A/Bs.
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
o, lse = C().attn_fwd(q, k, v, True, sc)
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
dq, dk, dv = dqkv[:, :, :Hq], dqkv[:, :, Hq:Hq + Hkv], dqkv[:, :, Hq + Hkv:]


def med(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


fwd = med(lambda: C().attn_fwd(q, k, v, True, sc))
bwd = med(lambda: C().attn_bwd(do, q, k, v, o, lse, True, sc, dq, dk, dv, 4))
mm = 2 * B * Hq * T * T * D * 0.5  # one causal matmul
tag = os.environ.get("ORION_ATTN_FWD", "v3") + ":" + os.path.basename(os.environ.get("ORION_AMD_EXT", "_C.so"))
print(json.dumps(dict(kernel=tag, B=B, T=T, Hq=Hq, Hkv=Hkv, D=D, fwd_ms=round(fwd, 4),
                      fwd_TFs=round(2 * mm / fwd / 1e9, 1), bwd_ms=round(bwd, 4),
                      bwd_TFs=round(7 * mm / bwd / 1e9, 1))))
