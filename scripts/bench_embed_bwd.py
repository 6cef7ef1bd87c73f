#!/usr/bin/env python3
"""Token-embedding backward at the GPT-2 bench shape (65,536 ids, 50,304 x 768 table): the
fp32-atomic scatter-add into an fp32 slice (csrc/embedding.hip) vs autograd's sort-based
dense backward + fp32 fold.  Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

load_ext(required=True)
V, Cc, N = 50304, 768, 65536
torch.manual_seed(0)
idx = torch.randint(0, 50257, (N,), device="cuda")
dx = torch.randn(N, Cc, device="cuda").bfloat16()
out = torch.zeros(V, Cc, device="cuda")


def med(fn, it=20):
    for _ in range(3):
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


t_atomic = med(lambda: C().embed_scatter_add_(dx, idx, out))
t_dense = med(lambda: out.add_(torch.ops.aten.embedding_dense_backward(dx, idx, V, -1, False)))
ref = torch.zeros(V, Cc, device="cuda")
ref.add_(torch.ops.aten.embedding_dense_backward(dx, idx, V, -1, False).float())
out.zero_()
C().embed_scatter_add_(dx, idx, out)
err = ((out - ref).norm() / ref.norm()).item()
print(json.dumps(dict(atomic_ms=round(t_atomic, 4), dense_ms=round(t_dense, 4), rel_err=err)))
