#!/usr/bin/env python3
"""HBM bandwidth ceiling probe: device-to-device copies and a read-only reduction of N-byte
buffers (median of 20), to price the memory-bound kernels against what the chip delivers.
usage: python scripts/hbm_copy_bw.py [MB]"""
import json
import sys

import torch

mb = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = mb * 1024 * 1024 // 4
a = torch.randn(n, device="cuda")
b = torch.empty_like(a)


def med(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


t_copy = med(lambda: b.copy_(a))
t_sum = med(lambda: a.sum())
nbytes = n * 4
print(json.dumps({"MB": mb, "copy_ms": round(t_copy, 4), "copy_TBs": round(2 * nbytes / t_copy / 1e9, 2),
                  "read_ms": round(t_sum, 4), "read_TBs": round(nbytes / t_sum / 1e9, 2)}))
