#!/usr/bin/env python3
"""gemm16 work-order sweep: the m-tile group size GM (gemm_diag bits 8-15) on the K = 768
forward shapes, persistent walk, interleaved rounds; one JSON line per shape {GM: TF/s}.
usage: python scripts/gemm_gm_sweep.py [--gms 2,4,8,16] [--iters 10]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gms", default="2,4,8,16")
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
load_ext(required=True)
ops = C()
M = 65536
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(torch.bfloat16)  # noqa: E731
gms = [int(v) for v in a.gms.split(",")]
for name, N, K, epi in [("lmhead_fwd", 50304, 768, 0), ("fc_fwd_gelu", 3072, 768, 2), ("qkv_fwd", 2304, 768, 1),
                        ("lmhead_dgrad", 768, 50304, 0)]:
    x = rnd(M, K)
    kind_dgrad = name.endswith("dgrad")
    w = rnd(K, N) if kind_dgrad else rnd(N, K)
    b = rnd(N) if epi else None
    f = lambda: ops.gemm(x, w, kind_dgrad, epi, b, None)  # noqa: E731
    ts = {gm: [] for gm in gms}
    for gm in gms:
        ops.gemm_diag(gm << 8)
        f()
    torch.cuda.synchronize()
    for _ in range(a.iters):
        for gm in gms:
            ops.gemm_diag(gm << 8)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            e1.synchronize()
            ts[gm].append(e0.elapsed_time(e1))
    ops.gemm_diag(0)
    fl = 2.0 * M * N * K
    print(json.dumps({"shape": name, **{f"GM{gm}": round(fl / sorted(v)[len(v) // 2] / 1e9, 1)
                                        for gm, v in ts.items()}}), flush=True)
    del x, w
