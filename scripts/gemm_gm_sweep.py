#!/usr/bin/env python3
"""gemm16 work-order sweep: the m-tile group size GM (gemm_diag bits 8-15) on the K = 768
GPT-2 shapes (forwards, input gradients, weight gradients), persistent walk, interleaved rounds;
one JSON line per shape {GM: TF/s}.
usage: python scripts/gemm_gm_sweep.py [--gms 2,4,8,16] [--iters 10] [--backward]"""
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
ap.add_argument("--backward", action="store_true", help="input / weight gradient shapes only")
a = ap.parse_args()
load_ext(required=True)
ops = C()
M = 65536
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(torch.bfloat16)  # noqa: E731
gms = [int(v) for v in a.gms.split(",")]
SHAPES = [("lmhead_fwd", 50304, 768, 0), ("fc_fwd_gelu", 3072, 768, 2), ("qkv_fwd", 2304, 768, 1),
          ("lmhead_dgrad", 768, 50304, 0), ("qkv_dgrad", 768, 2304, 0), ("attnproj_dgrad", 768, 768, 0),
          ("fc_dgrad", 768, 3072, 0), ("mlpproj_dgrad_gelu", 3072, 768, 3),
          ("wgrad_qkv", 2304, 768, -1), ("wgrad_fc", 3072, 768, -1), ("wgrad_lmhead", 50304, 768, -1)]
if a.backward:
    SHAPES = [s for s in SHAPES if "fwd" not in s[0]]
SHAPES += [("lmhead_exp_fwd", 50304, 768, 6), ("lmhead_rowscale_dgrad", 768, 50304, 7)]
if a.backward:
    SHAPES = [s for s in SHAPES if "fwd" not in s[0]]
for name, N, K, epi in SHAPES:
    if epi == 6:  # LM head forward through the exp epilogue (+ the fold)
        x, w = rnd(M, K), rnd(N, K) * 0.1
        tg = torch.randint(0, N, (M,), device="cuda", generator=g)
        cref = torch.zeros(1, device="cuda")
        f = lambda: ops.lmhead_fwd(x, w, tg, -1, cref)  # noqa: E731
        fl_mnk = (M, N, K)
    elif epi == 7:  # LM head input gradient: row-scaled E W
        x, w = rnd(M, K), rnd(K, N)
        srow = torch.rand(M, device="cuda", generator=g)
        f = lambda: ops.gemm_rowscale(x, w, srow)  # noqa: E731
        fl_mnk = (M, N, K)
    kind_dgrad = name.endswith("dgrad") or (name.endswith("gelu") and epi == 3)
    if epi in (6, 7):
        pass
    elif epi == -1:  # weight gradient: dy (M x N) ^T x (M x K), k-major operands, split-K as chosen
        x, w = rnd(M, N), rnd(M, K)
        f = lambda: ops.wgrad(x, w, None, 0)  # noqa: E731
        fl_mnk = (N, K, M)
    else:
        x = rnd(M, K)
        w = rnd(K, N) if kind_dgrad else rnd(N, K)
        b = rnd(N) if epi in (1, 2) else None
        pre = rnd(M, N) if epi == 3 else None
        f = lambda: ops.gemm(x, w, kind_dgrad, epi, b, pre)  # noqa: E731
        fl_mnk = (M, N, K)
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
    fl = 2.0 * fl_mnk[0] * fl_mnk[1] * fl_mnk[2]
    print(json.dumps({"shape": name, **{f"GM{gm}": round(fl / sorted(v)[len(v) // 2] / 1e9, 1)
                                        for gm, v in ts.items()}}), flush=True)
    del x, w
