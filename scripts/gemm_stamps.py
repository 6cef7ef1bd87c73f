#!/usr/bin/env python3
"""Slot timing of the phased GEMM (csrc/gemm_phased.hip, ORION_GEMM_DIAG=4): workgroup 0's
per-wave s_memtime stamps at each READ / MMA slot boundary, summarised per phase type.
usage: python scripts/gemm_stamps.py M N K wkm [diag_extra]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

M, N, K, wkm = (int(v) for v in sys.argv[1:5])
extra = int(sys.argv[5]) if len(sys.argv) > 5 else 0
load_ext(required=True)
os.environ["ORION_GEMM_CFG"] = "7"
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
w = (torch.randn(*((K, N) if wkm else (N, K)), device="cuda", generator=g) * 0.5).to(torch.bfloat16)
os.environ["ORION_GEMM_DIAG"] = "0"
for _ in range(5):
    C().gemm(x, w, bool(wkm), 0, None, None)
os.environ["ORION_GEMM_DIAG"] = str(4 | extra)
out = C().gemm(x, w, bool(wkm), 0, None, None)[0]
torch.cuda.synchronize()
st = out.reshape(-1)[: 8 * 1024 * 4].view(torch.int64).reshape(8, 1024).cpu()
nk = K // 64
t0 = int(st[:, 0].min())
rec = {"shape": f"{M}x{N}x{K}x{wkm}", "total_cycles": int(st[:, 1023].max()) - t0}
# per phase P, wave v: R = st[v, 1+3P] (READ start), S = st[v, 2+3P] (MMA start after lds wait),
# E = st[v, 3+3P] (MFMAs issued)
import statistics as stt
for grp in (0, 1):
    waves = range(4 * grp, 4 * grp + 4)
    for q in range(4):
        read, wait, mma, gap = [], [], [], []
        for t in range(2, nk - 2):
            P = 4 * t + q
            if 3 + 3 * (P + 1) >= 1023:
                break
            for v in waves:
                R, S, E = (int(st[v, 1 + 3 * P + i]) for i in range(3))
                Rn = int(st[v, 1 + 3 * (P + 1)])
                read.append(S - R)
                mma.append(E - S)
                gap.append(Rn - E)
        if read:
            rec[f"g{grp}q{q}"] = {"read_to_mma": stt.median(read), "mma_issue": stt.median(mma),
                                  "mma_end_to_next_read": stt.median(gap)}
print(json.dumps(rec))
