#!/usr/bin/env python3
"""Time the single-input LayerNorm forward at GPT-2's shape (65,536 x 768: the residual sites'
form, reading only the new stream), median of 30; one JSON line.
usage: [ORION_LN_FWD1=0] [ORION_LN_FWD1_BLOCKS=n] python scripts/time_ln_fwd.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

load_ext(required=True)
R, Cn = 65536, 768
g = torch.Generator(device="cuda").manual_seed(0)
s = torch.randn(R, Cn, device="cuda", generator=g).bfloat16()
w = torch.randn(Cn, device="cuda", generator=g).bfloat16()
b = torch.randn(Cn, device="cuda", generator=g).bfloat16()
y, mu, rs = C().layernorm_fwd(s, w, b, 1e-5)
ref = torch.nn.functional.layer_norm(s.float(), (Cn,), w.float(), b.float(), 1e-5)
err = ((y.float() - ref).norm() / ref.norm()).item()
f = lambda: C().layernorm_fwd(s, w, b, 1e-5)  # noqa: E731
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
print(json.dumps({"ms": round(t, 4), "TBs": round(2 * R * Cn * 2 / t / 1e9, 2), "rel_err": f"{err:.2e}",
                  "fwd1": os.environ.get("ORION_LN_FWD1", "1"),
                  "blocks": os.environ.get("ORION_LN_FWD1_BLOCKS", "4096")}))
