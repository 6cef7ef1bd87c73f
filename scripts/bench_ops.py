#!/usr/bin/env python3
"""Memory-bound kernel microbenchmark at the GPT-2 bench shapes (rows = B*T).

Times the fused add+LayerNorm fwd, LayerNorm bwd (with residual grad and branch-bias
colsum), bias+GELU fwd/bwd, fused cross-entropy fwd+bwd and the flat AdamW, and prints
one JSON line with ms and achieved GB/s (bytes that must cross HBM at least once).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C  # noqa: E402
from bench_attn import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--C", type=int, default=768)
    ap.add_argument("--V", type=int, default=50304)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    R, Cc, V = a.rows, a.C, a.V
    ops = C()
    dev = "cuda"
    bf = torch.bfloat16
    torch.manual_seed(0)
    x = torch.randn(R, Cc, device=dev, dtype=bf)
    r = torch.randn(R, Cc, device=dev, dtype=bf)
    w = torch.randn(Cc, device=dev, dtype=bf)
    b = torch.randn(Cc, device=dev, dtype=bf)
    rb = torch.randn(Cc, device=dev, dtype=bf)
    dy = torch.randn(R, Cc, device=dev, dtype=bf)
    dres = torch.randn(R, Cc, device=dev, dtype=bf)
    res = {}
    E = R * Cc * 2  # bytes of one (R, C) bf16 tensor

    def rec(name, ms, nbytes):
        res[name + "_ms"] = round(ms, 4)
        res[name + "_GBs"] = round(nbytes / ms / 1e6, 1)

    s, y, mean, rstd = ops.add_layernorm_fwd(x, r, w, b, 1e-5, rb)
    rec("add_ln_fwd", timeit(lambda: ops.add_layernorm_fwd(x, r, w, b, 1e-5, rb), a.iters), 4 * E)
    rec("ln_bwd", timeit(lambda: ops.layernorm_bwd(dy, s, w, mean, rstd, True, dres, True), a.iters), 4 * E)
    rec("ln_bwd_nores", timeit(lambda: ops.layernorm_bwd(dy, s, w, mean, rstd, True, None, False), a.iters), 3 * E)
    h = torch.randn(R, 4 * Cc, device=dev, dtype=bf)
    hb = torch.randn(4 * Cc, device=dev, dtype=bf)
    dh = torch.randn(R, 4 * Cc, device=dev, dtype=bf)
    rec("bias_gelu_fwd", timeit(lambda: ops.bias_gelu_fwd(h, hb), a.iters), 2 * 4 * E)
    rec("bias_gelu_bwd", timeit(lambda: ops.bias_gelu_bwd(dh, h, hb), a.iters), 3 * 4 * E)
    del h, dh
    logits = torch.randn(R, V, device=dev, dtype=bf)
    tg = torch.randint(0, V, (R,), device=dev)
    rec("xent", timeit(lambda: ops.xent_fwd_bwd(logits, tg, -1), a.iters), 2 * R * V * 2)
    del logits
    # flat AdamW over a GPT-2-124M-sized arena (fp32 grads, master, m, v; bf16 weights)
    n = 124 * 1024 * 1024
    p16 = torch.zeros(n, device=dev, dtype=bf)
    master, mm, vv, gg = (torch.randn(n, device=dev) * 0.01 for _ in range(4))
    vv.abs_()
    decay = torch.ones(n // 2048, device=dev, dtype=torch.uint8)
    hyper = torch.tensor([6e-4, 0.9, 0.95, 1e-8, 0.1, 0.1, 0.05, 1.0], device=dev)
    ssq = torch.ones(1, device=dev)
    rec("adamw", timeit(lambda: ops.adamw_flat(p16, master, mm, vv, gg, decay, hyper, ssq), a.iters), n * 30)
    del p16, master, mm, vv, gg
    res.update(rows=R, C=Cc, V=V)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
