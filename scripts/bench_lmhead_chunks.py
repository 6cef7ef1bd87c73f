#!/usr/bin/env python3
"""LM head forward + fused cross-entropy, whole vs row-chunked (Infinity Cache reuse probe).

The whole form writes all 65,536 x 50,304 bf16 logits (6.6 GB) and the cross-entropy kernel
then reads them back from HBM.  The chunked form runs GEMM + cross-entropy per block of rows,
so a block's logits (rows x 50,304 x 2 B) may still be in the 256 MB Infinity Cache when the
cross-entropy reads them.  Timing only (a chunk's loss scaling is chunk-local here).

usage: python scripts/bench_lmhead_chunks.py [--rows 65536] [--chunks 1 8 16 32 64]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--vocab", type=int, default=50304)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--chunks", type=int, nargs="+", default=[1, 8, 16, 32, 64])
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from orion_amd.ops._ext import C, load_ext
    from orion_amd.tuning import use_tuned_gemms
    load_ext(required=True)
    use_tuned_gemms()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(a.rows, a.dim, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(a.vocab, a.dim, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    t = torch.randint(0, 50257, (a.rows,), device=dev, generator=g)
    logits = torch.empty(a.rows, a.vocab, device=dev, dtype=torch.bfloat16)
    for n in a.chunks:
        rc = a.rows // n

        def run():
            for i in range(n):
                sl = slice(i * rc, (i + 1) * rc)
                torch.mm(x[sl], w.t(), out=logits[sl])
                C().xent_fwd_bwd(logits[sl], t[sl], -1)

        def gemm_only():
            for i in range(n):
                sl = slice(i * rc, (i + 1) * rc)
                torch.mm(x[sl], w.t(), out=logits[sl])

        res = {}
        for name, fn in (("gemm+xent", run), ("gemm", gemm_only)):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name] = e0.elapsed_time(e1) / a.iters
        print(f"chunks {n:3d} ({rc} rows, {rc * a.vocab * 2 / 2**20:.0f} MiB logits): "
              f"gemm+xent {res['gemm+xent']:.3f} ms  gemm {res['gemm']:.3f} ms  "
              f"xent share {res['gemm+xent'] - res['gemm']:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
