#!/usr/bin/env python3
"""Does the bandwidth-bound cross-entropy pass overlap the compute-bound LM-head GEMM when the
two run on separate streams, chunked over rows?  GPT-2 LM head: x (65,536 x 768) @ W^T
(50,304 x 768) on hipBLASLt, then csrc/xent.hip's in-place loss + dlogits pass.

serial:   GEMM(all rows); xent(all rows)
chunked:  stream A: GEMM(chunk 0), GEMM(chunk 1), ...; stream B: xent(chunk i) after GEMM(i)
Prints one JSON line per configuration (median of 10 runs, ms)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

load_ext(required=True)
ops = C()
M, K, V = 65536, 768, 50304
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
w = (torch.randn(V, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
tgt = torch.randint(0, V, (M,), device="cuda", generator=g)
logits = torch.empty(M, V, device="cuda", dtype=torch.bfloat16)
sa, sb = torch.cuda.current_stream(), torch.cuda.Stream()


def serial():
    torch.matmul(x, w.t(), out=logits)
    ops.xent_fwd_bwd(logits, tgt, -1)


def chunked(n):
    rows = M // n
    evs = [torch.cuda.Event() for _ in range(n)]
    for i in range(n):
        torch.matmul(x[i * rows:(i + 1) * rows], w.t(), out=logits[i * rows:(i + 1) * rows])
        evs[i].record(sa)
    with torch.cuda.stream(sb):
        for i in range(n):
            sb.wait_event(evs[i])
            ops.xent_fwd_bwd(logits[i * rows:(i + 1) * rows], tgt[i * rows:(i + 1) * rows], -1)
    sa.wait_stream(sb)


def gemm_only(n):
    rows = M // n
    for i in range(n):
        torch.matmul(x[i * rows:(i + 1) * rows], w.t(), out=logits[i * rows:(i + 1) * rows])


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


res = {"serial_ms": timeit(serial), "gemm_only_ms": timeit(lambda: gemm_only(1)),
       "xent_only_ms": timeit(lambda: ops.xent_fwd_bwd(logits, tgt, -1))}
for n in (2, 4, 8):
    res[f"chunked{n}_ms"] = timeit(lambda: chunked(n))
    res[f"gemm_chunks{n}_ms"] = timeit(lambda: gemm_only(n))
print(json.dumps({k: round(v, 4) for k, v in res.items()}), flush=True)
