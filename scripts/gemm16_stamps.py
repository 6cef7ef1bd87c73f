#!/usr/bin/env python3
"""Slot anatomy of csrc/gemm16.hip from its stamped diagnostic instantiation
(gemm_diag(4)): every wave of every workgroup stamps s_memtime at
kernel start, prologue landed, the six slot boundaries of both phases of the middle k-tile,
main-loop end and epilogue end.  Prints medians (cycles) per group and phase over all
workgroups: reads+DMA issue, vmcnt wait, barrier wait into the MMA slot, lgkmcnt wait, MFMA
issue, barrier wait out of it; plus prologue, main loop, epilogue and the k-tile time.
usage: python scripts/gemm16_stamps.py M N K wkm"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

M, N, K, wkm = (int(v) for v in sys.argv[1:5])
load_ext(required=True)
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
w = (torch.randn(*((K, N) if wkm else (N, K)), device="cuda", generator=g) * 0.5).to(torch.bfloat16)
nwg = ((M + 255) // 256) * ((N + 255) // 256)
buf = torch.zeros(nwg * 8 * 20, device="cuda", dtype=torch.int64)
C().gemm_diag(0)
for _ in range(10):
    C().gemm(x, w, bool(wkm), 0, None, None)
C().gemm_diag(4)
for _ in range(3):
    C().gemm(x, w, bool(wkm), 0, None, buf)
torch.cuda.synchronize()
C().gemm_diag(0)
st = buf.view(nwg, 8, 20)[:, :, :16].cpu()
rec = {"shape": f"{M}x{N}x{K}x{wkm}", "workgroups": nwg}
names = ["issue", "vmcnt", "bar_in", "lgkm", "mfma", "bar_out"]
for grp in (0, 1):
    s = st[:, 4 * grp: 4 * grp + 4, :].reshape(-1, 16).double()
    for H in (0, 1):
        b = 2 + 6 * H
        nxt = s[:, b + 6] if H == 0 else None
        cols = [s[:, b + k + 1] - s[:, b + k] for k in range(5)]
        if nxt is not None:
            cols.append(nxt - s[:, b + 5])
        rec[f"g{grp}H{H}"] = {n: round(float(c.median()), 0) for n, c in zip(names, cols)}
    rec[f"g{grp}_phase0_cycles"] = round(float((s[:, 8] - s[:, 2]).median()), 0)
    rec[f"g{grp}_prologue"] = round(float((s[:, 1] - s[:, 0]).median()), 0)
    rec[f"g{grp}_mainloop"] = round(float((s[:, 14] - s[:, 1]).median()), 0)
    rec[f"g{grp}_epilogue"] = round(float((s[:, 15] - s[:, 14]).median()), 0)
rec["k_tiles"] = K // 64
rec["mfma_cycles_per_phase"] = 512
print(json.dumps(rec))
