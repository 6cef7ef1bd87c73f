#!/usr/bin/env python3
"""Weight-gradient GEMM at Llama-2-7B shapes: HIP wgrad kernel vs hipBLASLt (dy^T x).

Prints one JSON line: per (M, n1, n2) the median ms and PF/s of
  hip     csrc/wgrad.hip (C().wgrad)
  blas    dy.t() @ x              (hipBLASLt through torch)
  blas_sw (x.t() @ dy).t()
  blas_acc torch.addmm(g, dy.t(), x) accumulating into an existing bf16 buffer
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_attn import timeit  # noqa: E402
from orion_amd.ops._ext import C  # noqa: E402


def main():
    Ms = [int(m) for m in os.environ.get("WG_MS", "16384 4096").split()]
    shapes = [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008), (32000, 4096),
              (2304, 768), (3072, 768), (768, 3072), (50304, 768)]
    bf = torch.bfloat16
    out = {}
    for M in Ms:
        for n1, n2 in shapes:
            if n2 == 768 and M != 16384:
                continue
            MM = 65536 if n2 == 768 or n1 == 768 else M
            dy = torch.randn(MM, n1, device="cuda", dtype=bf)
            x = torch.randn(MM, n2, device="cuda", dtype=bf)
            g = torch.zeros(n1, n2, device="cuda", dtype=bf)
            fl = 2.0 * MM * n1 * n2
            r = {}
            r["hip"] = timeit(lambda: C().wgrad(dy, x, None, 0))
            r["blas"] = timeit(lambda: dy.t() @ x)
            r["blas_sw"] = timeit(lambda: (x.t() @ dy).t())
            r["blas_acc"] = timeit(lambda: torch.addmm(g, dy.t(), x, out=g))
            ref = (dy[:4096].float().t() @ x[:4096].float())
            err = ((C().wgrad(dy[:4096], x[:4096], None, 0).float() - ref).abs().max() / ref.abs().max()).item()
            key = f"M{MM}_{n1}x{n2}"
            out[key] = {k: round(v, 4) for k, v in r.items()}
            out[key].update({f"{k}_PF": round(fl / v / 1e12, 3) for k, v in r.items()})
            out[key]["hip_relerr"] = err
            print(key, out[key], flush=True)
            del dy, x, g, ref
            torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
