#!/usr/bin/env python3
"""Every GEMM of one GPT-2-124M training step at micro-batch 64 (M = 65536 tokens),
called exactly as the model calls it, timed standalone (median of interleaved runs).
Loads the committed TunableOp table unless --untuned."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
from bench_attn import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--untuned", action="store_true")
    a = ap.parse_args()
    n = 0
    if not a.untuned:
        from orion_amd.tuning import use_tuned_gemms
        n = use_tuned_gemms()
    from orion_amd.ops.gemm import wgrad
    M, C, V = a.M, 768, 50304
    bf = torch.bfloat16
    r = lambda *s: torch.randn(*s, device="cuda", dtype=bf)  # noqa: E731
    res = {"tuned_entries": n}
    x, h = r(M, C), r(M, 4 * C)
    for name, K, N, bias in (("qkv", C, 3 * C, True), ("attn_proj", C, C, False),
                             ("fc", C, 4 * C, False), ("mlp_proj", 4 * C, C, False)):
        inp = x if K == C else h
        W = r(N, K)
        b = r(N) if bias else None
        dy = r(M, N)
        fl = 2.0 * M * K * N
        t_f = timeit(lambda: F.linear(inp, W, b))
        t_dx = timeit(lambda: dy @ W)
        t_dw = timeit(lambda: wgrad(dy, inp))
        res[name] = {"fwd_ms": round(t_f, 4), "dx_ms": round(t_dx, 4), "dw_ms": round(t_dw, 4),
                     "fwd_PF": round(fl / t_f / 1e12, 2), "dx_PF": round(fl / t_dx / 1e12, 2),
                     "dw_PF": round(fl / t_dw / 1e12, 2)}
        del W, dy
    Wte = r(V, C)
    dl = r(M, V)
    fl = 2.0 * M * C * V
    t_f = timeit(lambda: F.linear(x, Wte), 5)
    t_dx = timeit(lambda: dl @ Wte, 5)
    t_dw = timeit(lambda: wgrad(dl, x), 5)
    res["lm_head"] = {"fwd_ms": round(t_f, 4), "dx_ms": round(t_dx, 4), "dw_ms": round(t_dw, 4),
                      "fwd_PF": round(fl / t_f / 1e12, 2), "dx_PF": round(fl / t_dx / 1e12, 2),
                      "dw_PF": round(fl / t_dw / 1e12, 2)}
    per_layer = sum(res[k][f] for k in ("qkv", "attn_proj", "fc", "mlp_proj") for f in ("fwd_ms", "dx_ms", "dw_ms"))
    res["step_gemm_ms"] = round(12 * per_layer + sum(res["lm_head"][f] for f in ("fwd_ms", "dx_ms", "dw_ms")), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
