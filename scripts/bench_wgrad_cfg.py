#!/usr/bin/env python3
"""Weight-gradient kernels A/B in one process: ORION_WGRAD_CFG variants (7 = the phased kernel
of csrc/gemm_phased.hip, 0 = csrc/wgrad.hip's default) on the GPT-2 shapes at M = 65,536
tokens, writing an fp32 gradient slice as in training (split-K slabs + slab_sum included).
usage: python scripts/bench_wgrad_cfg.py [--cfgs 7,0] [--iters 15] [--M 65536]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfgs", default="7,0")
ap.add_argument("--iters", type=int, default=15)
ap.add_argument("--M", type=int, default=65536)
ap.add_argument("--shapes", default="768x768,2304x768,3072x768,768x3072,50304x768")
ap.add_argument("--blas", action="store_true", help="also time hipBLASLt (fp32-output mm into the slice)")
a = ap.parse_args()
load_ext(required=True)
ops = C()
g = torch.Generator(device="cuda").manual_seed(0)
tot = {}
for sh in a.shapes.split(","):
    n1, n2 = (int(v) for v in sh.split("x"))
    dy = (torch.randn(a.M, n1, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    x = (torch.randn(a.M, n2, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    out = torch.empty(n1, n2, device="cuda", dtype=torch.float32)
    ref = dy.float().t() @ x.float()
    rec = {"shape": sh}
    ts = {c: [] for c in a.cfgs.split(",") + (["blas"] if a.blas else [])}
    for it in range(a.iters + 3):
        for c in ts:
            os.environ["ORION_WGRAD_CFG"] = c if c != "blas" else "7"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if c == "blas":
                torch.mm(dy.t(), x, out_dtype=torch.float32, out=out)
            else:
                ops.wgrad_into(dy, x, None, out, False, 0)
            e1.record()
            e1.synchronize()
            if it >= 3:
                ts[c].append(e0.elapsed_time(e1))
            if it == 0:
                rec[f"cfg{c}_rel_err"] = float((out - ref).norm() / ref.norm())
    for c, v in ts.items():
        ms = sorted(v)[len(v) // 2]
        rec[f"cfg{c}_ms"] = round(ms, 4)
        rec[f"cfg{c}_TFs"] = round(2.0 * a.M * n1 * n2 / ms / 1e9, 1)
        tot[c] = tot.get(c, 0.0) + ms
    print(json.dumps(rec), flush=True)
print(json.dumps({f"total_cfg{c}_ms": round(v, 3) for c, v in tot.items()}))
