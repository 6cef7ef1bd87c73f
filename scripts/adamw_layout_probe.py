#!/usr/bin/env python3
"""Does the fused AdamW's HBM rate depend on where its five streams start?  Times
adamw_flat over N parameters with the fp32 streams (master, m, v, grad) and the bf16
parameter placed at (a) the allocator's offsets, (b) staggered base offsets (stream i
shifted by i * SHIFT bytes), for a few sizes; prints one JSON line per case.
usage: python scripts/adamw_layout_probe.py [N ...]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

load_ext(required=True)
dev = "cuda"


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


def case(n, shift):
    pad = 4 * shift // 4 + 64  # elements of slack for the largest shift (fp32)
    bufs = []
    views = []
    for i in range(4):
        b = torch.empty(n + pad * 5, device=dev)
        o = (i * shift) // 4
        views.append(b[o:o + n])
        bufs.append(b)
    pb = torch.zeros(n + pad * 10, dtype=torch.bfloat16, device=dev)
    p16 = pb[(4 * shift) // 2:(4 * shift) // 2 + n]
    master, m, v, g = views
    for t in views:
        t.normal_()
    v.abs_()
    decay = torch.ones(n // 2048, dtype=torch.uint8, device=dev)
    hyper = torch.tensor([6e-4, 0.9, 0.95, 1e-8, 0.1, 0.1, 0.05, 0.0], device=dev)
    sumsq = torch.ones(1, device=dev)
    t = med(lambda: C().adamw_flat(p16, master, m, v, g, decay, hyper, sumsq))
    addrs = [x.data_ptr() % (1 << 22) for x in (master, m, v, g, p16)]
    print(json.dumps({"n": n, "shift_B": shift, "ms": round(t, 4), "TBs": round(30.0 * n / t / 1e9, 2),
                      "base_mod_4MiB": addrs}), flush=True)
    del bufs, pb, views, master, m, v, g, p16
    torch.cuda.empty_cache()


sizes = [int(a) for a in sys.argv[1:]] or [124475392, 1 << 30]
for n in sizes:
    n -= n % 2048
    for shift in (0, 4096 + 256, 65536 + 1024, (1 << 20) + 4096):
        case(n, shift)
