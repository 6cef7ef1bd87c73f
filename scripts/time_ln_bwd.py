#!/usr/bin/env python3
"""Time the fused add+LayerNorm backward at GPT-2's shape (65,536 x 768, residual gradient
folded, branch-bias column sum), median of 30; one JSON line.  usage: python scripts/time_ln_bwd.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

load_ext(required=True)
R, Cn = 65536, 768
g = torch.Generator(device="cuda").manual_seed(0)
mk = lambda *s: torch.randn(*s, device="cuda", generator=g).bfloat16()  # noqa: E731
s, dy, dres = mk(R, Cn), mk(R, Cn), mk(R, Cn)
w, b = mk(Cn), mk(Cn)
mean = s.float().mean(1)
rstd = torch.rsqrt(s.float().var(1, unbiased=False) + 1e-5)
f = lambda: C().layernorm_bwd(dy, s, w, mean, rstd, True, dres, True)  # noqa: E731
for _ in range(3):
    f()
torch.cuda.synchronize()
ts = []
for _ in range(30):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    f()
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
t = sorted(ts)[15]
nb = os.environ.get("ORION_LN_BWD_NB", "default")
print(json.dumps({"ms": round(t, 4), "TBs": round(4 * R * Cn * 2 / t / 1e9, 2), "nb": nb}))
