#!/usr/bin/env python3
"""Time csrc/gemm*.hip variants under diagnostic flags (ORION_GEMM_CFG x ORION_GEMM_DIAG) on
a few shapes, interleaved in one process (median of --iters).  Diagnostic runs compute wrong
products by design (skipped staging / fragment reads): timing only.
usage: python scripts/diag_gemm.py [--cfgs 7,0] [--diags 0,1,2,3] [--iters 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfgs", default="7")
ap.add_argument("--diags", default="0,1,2,3")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--shapes", default="4096x4096x4096x0,65536x768x3072x0,65536x2304x768x0,65536x768x3072x1")
a = ap.parse_args()
load_ext(required=True)
ops = C()
g = torch.Generator(device="cuda").manual_seed(0)
summary = {}
for sh in a.shapes.split(","):
    M, N, K, wkm = (int(v) for v in sh.split("x"))
    x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(*((K, N) if wkm else (N, K)), device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    variants = [(c, d) for c in a.cfgs.split(",") for d in a.diags.split(",")]
    ts = {v: [] for v in variants}
    for it in range(a.iters + 3):
        for c, d in variants:
            os.environ["ORION_GEMM_CFG"], os.environ["ORION_GEMM_DIAG"] = c, d
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.gemm(x, w, bool(wkm), 0, None, None)
            e1.record()
            e1.synchronize()
            if it >= 3:
                ts[(c, d)].append(e0.elapsed_time(e1))
    rec = {"shape": sh}
    for (c, d), v in ts.items():
        ms = sorted(v)[len(v) // 2]
        rec[f"cfg{c}_diag{d}_TFs"] = round(2.0 * M * N * K / ms / 1e9, 1)
        summary[f"{sh}_c{c}d{d}"] = rec[f"cfg{c}_diag{d}_TFs"]
    print(json.dumps(rec), flush=True)
print(json.dumps(summary))  # one line with every shape (scripts/ab.sh prints the last line)
os.environ["ORION_GEMM_DIAG"] = "0"
