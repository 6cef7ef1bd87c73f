#!/usr/bin/env python3
"""Run the split attention backward (and forward) a few times on one shape, for
rocprofv3 --pmc passes.  usage: python scripts/attn_one.py B T Hq Hkv D [reps]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

B, T, Hq, Hkv, D = (int(v) for v in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 3
load_ext(required=True)
g = torch.Generator(device="cuda").manual_seed(0)
mk = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)
q, k, v, do = mk(B, T, Hq, D), mk(B, T, Hkv, D), mk(B, T, Hkv, D), mk(B, T, Hq, D)
sc = 1 / math.sqrt(D)
o, lse = C().attn_fwd(q, k, v, True, sc)
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
for _ in range(reps):
    C().attn_fwd(q, k, v, True, sc)
    C().attn_bwd(do, q, k, v, o, lse, True, sc, dq, dk, dv, 4)
torch.cuda.synchronize()
