#!/usr/bin/env python3
"""Debug aid: forward attention outputs of the current kernel vs an fp32 reference on small
shapes, with the first mismatching (batch, token, head) positions.  usage: python
scripts/attn_fwd_diff.py"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

load_ext(required=True)
torch.manual_seed(0)
for (B, T, Hq, Hkv, D, causal) in [(1, 64, 1, 1, 64, False), (1, 64, 1, 1, 64, True),
                                   (1, 128, 1, 1, 64, False), (1, 256, 1, 1, 64, False),
                                   (1, 256, 1, 1, 64, True), (2, 320, 4, 2, 64, True),
                                   (1, 256, 1, 1, 128, True)]:
    q = torch.randn(B, T, Hq, D, device="cuda").bfloat16()
    k = torch.randn(B, T, Hkv, D, device="cuda").bfloat16()
    v = torch.randn(B, T, Hkv, D, device="cuda").bfloat16()
    sc = 1 / math.sqrt(D)
    o, lse = C().attn_fwd(q, k, v, causal, sc)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    kf = kf.repeat_interleave(Hq // Hkv, 1)
    vf = vf.repeat_interleave(Hq // Hkv, 1)
    ref = torch.nn.functional.scaled_dot_product_attention(qf, kf, vf, is_causal=causal).transpose(1, 2)
    err = (o.float() - ref).abs().amax(-1)  # (B, T, H)
    bad = (err > 0.05).nonzero()
    print(f"B{B} T{T} H{Hq}/{Hkv} D{D} causal={causal}: max err {err.max().item():.4f}, "
          f"bad rows {bad.shape[0]} / {err.numel()}", flush=True)
    if bad.shape[0]:
        print("   first bad (b, t, h):", bad[:8].tolist(), " t range", bad[:, 1].min().item(),
              bad[:, 1].max().item(), flush=True)
        t0 = bad[0].tolist()
        print("   got", o[t0[0], t0[1], t0[2], :6].float().tolist(), "want",
              ref[t0[0], t0[1], t0[2], :6].tolist(), flush=True)
