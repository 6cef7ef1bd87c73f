#!/usr/bin/env python3
"""Weight gradient dW = dY^T X at the Llama-7B shapes (16,384 tokens): the in-tree kernel (both
operands k-major; round 2 measured the since-removed csrc/gemm_phased.hip, now gemm16) vs
transposing dY once (HBM pass) and running the library GEMM in the dgrad (NN) layout with fp32
output.  One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

load_ext(required=True)
M = int(os.environ.get("WG_TOKENS", 16384))
shapes = [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008), (32000, 4096)]


def med(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(it):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


torch.manual_seed(0)
tot = {"phased": 0.0, "t+nn": 0.0, "transpose": 0.0}
for n1, n2 in shapes:
    dy = torch.randn(M, n1, device="cuda").bfloat16()
    x = torch.randn(M, n2, device="cuda").bfloat16()
    out = torch.empty(n1, n2, device="cuda")
    dyt = torch.empty(n1, M, device="cuda", dtype=torch.bfloat16)
    t_ph = med(lambda: C().wgrad_into(dy, x, None, out, False, 0))
    ref = out.clone()
    t_tr = med(lambda: dyt.copy_(dy.t()))
    t_nn = med(lambda: (dyt.copy_(dy.t()), torch.mm(dyt, x, out_dtype=torch.float32, out=out)))
    err = ((out - ref).norm() / ref.norm()).item()
    fl = 2.0 * M * n1 * n2
    tot["phased"] += t_ph
    tot["t+nn"] += t_nn
    tot["transpose"] += t_tr
    print(json.dumps(dict(n1=n1, n2=n2, M=M, phased_ms=round(t_ph, 3), transpose_ms=round(t_tr, 3),
                          t_plus_nn_ms=round(t_nn, 3), phased_TFs=round(fl / t_ph / 1e9),
                          nn_TFs_incl_transpose=round(fl / t_nn / 1e9), rel_err=round(err, 5))), flush=True)
print(json.dumps({k: round(v, 3) for k, v in tot.items()}))
