#!/usr/bin/env python3
"""Weight-gradient GEMM study: dW = dY^T X with the token dim (65536) as the reduction.

hipBLASLt's picks for these shapes run at 0.4-0.8 PF/s while the forward GEMMs of the
same layers reach 1.3-1.6 PF/s.  Compares, per GPT-2 layer shape:
  plain   dy.t() @ x
  swap    (x.t() @ dy).t()
  splitS  bmm over S token chunks with fp32 output, summed (explicit split-K)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_attn import timeit  # noqa: E402


def main():
    M = int(os.environ.get("WG_M", 65536))
    shapes = [(768, 768), (2304, 768), (3072, 768), (768, 3072), (50304, 768)]
    bf = torch.bfloat16
    out = {}
    for n1, n2 in shapes:
        dy = torch.randn(M, n1, device="cuda", dtype=bf)
        x = torch.randn(M, n2, device="cuda", dtype=bf)
        fl = 2.0 * M * n1 * n2
        r = {}
        r["plain"] = timeit(lambda: dy.t() @ x)
        r["swap"] = timeit(lambda: (x.t() @ dy).t())
        r["plain_f32"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        for S in (2, 4, 8, 16):
            d3, x3 = dy.view(S, M // S, n1), x.view(S, M // S, n2)
            def f(d3=d3, x3=x3):
                return torch.bmm(d3.transpose(1, 2), x3, out_dtype=torch.float32).sum(0).to(bf)
            try:
                r[f"split{S}"] = timeit(f)
            except Exception as e:  # pragma: no cover
                r[f"split{S}"] = str(e)[:80]
        ref = (dy.float().t() @ x.float())
        got = torch.bmm(dy.view(8, -1, n1).transpose(1, 2), x.view(8, -1, n2), out_dtype=torch.float32).sum(0)
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        out[f"{n1}x{n2}"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}
        out[f"{n1}x{n2}"]["best_PFs"] = round(fl / min(v for v in r.values() if isinstance(v, float)) / 1e12, 3)
        out[f"{n1}x{n2}"]["split8_relerr"] = err
        del dy, x, ref
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
