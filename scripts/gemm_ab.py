#!/usr/bin/env python3
"""Same-box A/B of extension builds on the GPT-2 GEMM shapes (scripts/ab_variants.sh runs it
once per variants/_C_*.so): times C().gemm / wgrad_into on each shape, interleaved rounds,
median; prints one JSON line {shape: TF/s}.  Works with any build that has the gemm op.
usage: python scripts/gemm_ab.py [--iters 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
load_ext(required=True)
ops = C()
M = 65536
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(torch.bfloat16)  # noqa: E731
shapes = [("qkv_fwd", "fwd", 2304, 768, 1), ("attnproj_fwd", "fwd", 768, 768, 0),
          ("fc_fwd_gelu", "fwd", 3072, 768, 2), ("mlpproj_fwd", "fwd", 768, 3072, 0),
          ("lmhead_fwd", "fwd", 50304, 768, 0), ("qkv_dgrad", "dgrad", 768, 2304, 0),
          ("fc_dgrad", "dgrad", 768, 3072, 0), ("mlpproj_dgrad_gelu", "dgrad", 3072, 768, 3),
          ("lmhead_dgrad", "dgrad", 768, 50304, 0), ("wgrad_fc", "wgrad", 3072, 768, 0),
          ("wgrad_qkv", "wgrad", 2304, 768, 0), ("wgrad_lmhead", "wgrad", 50304, 768, 0)]
fns, flops = {}, {}
for name, kind, N, K, epi in shapes:
    if kind == "wgrad":
        dy, x = rnd(M, N), rnd(M, K)
        out = torch.zeros(N, K, device="cuda")
        fns[name] = (lambda dy=dy, x=x, out=out: ops.wgrad_into(dy, x, None, out, False, 0))
    else:
        x = rnd(M, K)
        w = rnd(N, K) if kind == "fwd" else rnd(K, N)
        b = rnd(N) if epi in (1, 2) else None
        pre = rnd(M, N) if epi == 3 else None
        fns[name] = (lambda x=x, w=w, b=b, pre=pre, kind=kind, epi=epi:
                     ops.gemm(x, w, kind != "fwd", epi, b, pre))
    flops[name] = 2.0 * M * N * K
for f in fns.values():
    for _ in range(3):
        f()
torch.cuda.synchronize()
ts = {k: [] for k in fns}
for _ in range(a.iters):
    for k, f in fns.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        e1.synchronize()
        ts[k].append(e0.elapsed_time(e1))
res = {k: round(flops[k] / sorted(v)[len(v) // 2] / 1e9, 1) for k, v in ts.items()}
print(json.dumps(res))
