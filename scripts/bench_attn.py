#!/usr/bin/env python3
"""Attention microbenchmark on the GPT-2 training shape: orion_amd HIP flash attention
(fwd, bwd, bwd without dQ atomics) vs PyTorch SDPA on the same random data.
Prints one JSON line per measurement (median of interleaved rounds)."""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C  # noqa: E402


ITERS = 20


def timeit(fn, iters=None):
    iters = iters or ITERS
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--Hkv", type=int, default=0, help="KV heads (GQA); 0 = H")
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--causal", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    B, T, H, D, causal = a.B, a.T, a.H, a.D, bool(a.causal)
    Hkv = a.Hkv or H
    global ITERS
    ITERS = a.iters
    torch.manual_seed(0)
    qkv = torch.randn(B, T, H + 2 * Hkv, D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[:, :, :H], qkv[:, :, H:H + Hkv], qkv[:, :, H + Hkv:]
    scale = 1 / math.sqrt(D)
    ops = C()
    o, lse = ops.attn_fwd(q, k, v, causal, scale)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    flops_mm = 2 * B * H * T * T * D * (0.5 if causal else 1.0)
    res = {}
    res["fwd_ms"] = timeit(lambda: ops.attn_fwd(q, k, v, causal, scale))
    dq, dk, dv = dqkv[:, :, :H], dqkv[:, :, H:H + Hkv], dqkv[:, :, H + Hkv:]
    # flags: 8 = fused (fp32-atomic dQ), 9 = fused without the atomics, 4 = split (no atomics)
    res["bwd_fused_ms"] = timeit(lambda: ops.attn_bwd(do, q, k, v, o, lse, causal, scale, dq, dk, dv, 8))
    res["bwd_fused_noatomic_ms"] = timeit(lambda: ops.attn_bwd(do, q, k, v, o, lse, causal, scale,
                                                               dq, dk, dv, 9))
    res["bwd_split_ms"] = timeit(lambda: ops.attn_bwd(do, q, k, v, o, lse, causal, scale, dq, dk, dv, 4))
    res["bwd_ms"] = min(res["bwd_fused_ms"], res["bwd_split_ms"])
    if Hkv == H and D == 64:  # packed QKV with the bias gradient summed in the split kernels
        d5 = dqkv.view(B, T, 3, H, D)
        db = torch.empty(3 * H * D, device="cuda", dtype=torch.float32)
        res["bwd_split_bias_ms"] = timeit(lambda: ops.attn_bwd(do, q, k, v, o, lse, causal, scale, d5[:, :, 0],
                                                               d5[:, :, 1], d5[:, :, 2], 4, db))
        res["bwd_split_plus_colsum_ms"] = timeit(lambda: (ops.attn_bwd(do, q, k, v, o, lse, causal, scale, d5[:, :, 0],
                                                                       d5[:, :, 1], d5[:, :, 2], 4),
                                                          ops.colsum(dqkv.view(B * T, -1), db)))
    res["fwd_TFs"] = 2 * flops_mm / res["fwd_ms"] / 1e9
    res["bwd_TFs"] = 5 * flops_mm / res["bwd_ms"] / 1e9
    res["bwd_over_fwd"] = res["bwd_ms"] / res["fwd_ms"]
    qt, kt, vt = (t.transpose(1, 2).contiguous().requires_grad_() for t in (q, k, v))
    if Hkv != H:
        kt, vt = (t.detach().repeat_interleave(H // Hkv, 1).requires_grad_() for t in (kt, vt))
    try:
        sdpa = torch.nn.functional.scaled_dot_product_attention
        res["sdpa_fwd_ms"] = timeit(lambda: sdpa(qt, kt, vt, is_causal=causal))
        out = torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)
        g = torch.randn_like(out)
        res["sdpa_bwd_ms"] = timeit(lambda: torch.autograd.grad(out, (qt, kt, vt), g, retain_graph=True))
    except Exception as e:  # pragma: no cover
        res["sdpa_error"] = str(e)[:200]
    res.update(B=B, T=T, H=H, Hkv=Hkv, D=D, causal=causal)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
