#!/usr/bin/env python3
"""Price folding the residual add into the branch's output GEMM (GPT-2 attn-proj / fc2):
today  o = h W^T + b (hipBLASLt), (s, y) = add_layernorm(x, o)          -- 500 MB per site
probe  s = x + h W^T (hipBLASLt beta = 1, in place), y = layernorm(s)    -- 400 MB per site
blaslt s = h W^T + b + x (C().linear_residual: csrc/blaslt.cpp, bias and residual in the epilogue)
Medians of 20 per piece, TunableOp tables as in bench.py; one JSON line per GEMM shape.
usage: python scripts/probe_residual_gemm.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

load_ext(required=True)
from orion_amd.tuning import use_tuned_gemms  # noqa: E402
use_tuned_gemms()
M, D = 65536, 768
g = torch.Generator(device="cuda").manual_seed(0)
mk = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.1).bfloat16()  # noqa: E731


def med(f):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[10]


x, o = mk(M, D), mk(M, D)
lw, lb, rb = mk(D), mk(D), mk(D)
t_addln = med(lambda: C().add_layernorm_fwd(x, o, lw, lb, 1e-5, rb))
s = x + o
t_ln = med(lambda: C().layernorm_fwd(s, lw, lb, 1e-5))
for name, K in (("attn_proj", 768), ("fc2", 3072)):
    h, w, b = mk(M, K), mk(D, K), mk(D)
    t_mm = med(lambda: torch.nn.functional.linear(h, w))
    scratch = x.clone()
    t_addmm = med(lambda: scratch.addmm_(h, w.t()))
    t_res = med(lambda: C().linear_residual(h, w, b, x))
    got = C().linear_residual(h, w, b, x).float()
    want = h.float() @ w.float().t() + b.float() + x.float()
    err = ((got - want).norm() / want.norm()).item()
    print(json.dumps({"gemm": name, "linear_ms": round(t_mm, 4), "addmm_inplace_ms": round(t_addmm, 4),
                      "linear_residual_ms": round(t_res, 4), "rel_err": f"{err:.2e}",
                      "add_layernorm_ms": round(t_addln, 4), "layernorm_ms": round(t_ln, 4),
                      "today_ms": round(t_mm + t_addln, 4), "probe_ms": round(t_addmm + t_ln, 4),
                      "blaslt_ms": round(t_res + t_ln, 4)}))
# plain forwards (no residual): TunableOp-tuned F.linear vs the wrapper's own all-solution search
for name, N, K in (("qkv+bias", 2304, 768), ("attn_proj", 768, 768), ("fc2", 768, 3072)):
    h, w, b = mk(M, K), mk(N, K), mk(N)
    t_lin = med(lambda: torch.nn.functional.linear(h, w, b))
    t_own = med(lambda: C().linear_residual(h, w, b, None))
    err = ((C().linear_residual(h, w, b, None).float() - torch.nn.functional.linear(h, w, b).float()).norm()
           / torch.nn.functional.linear(h, w, b).float().norm()).item()
    print(json.dumps({"plain": name, "linear_bias_ms": round(t_lin, 4), "wrapper_ms": round(t_own, 4),
                      "rel_diff": f"{err:.2e}"}))
# residual without the bias (beta = 1, no bias epilogue): the solutions that support it
for name, K in (("attn_proj", 768), ("fc2", 3072)):
    h, w = mk(M, K), mk(D, K)
    t_nb = med(lambda: C().linear_residual(h, w, None, x))
    print(json.dumps({"residual_no_bias": name, "ms": round(t_nb, 4)}))

