#!/usr/bin/env python3
"""Slot anatomy of the phased GEMM (csrc/gemm_phased.hip, ORION_GEMM_DIAG=4 instantiation):
workgroup 0's per-wave s_memtime stamps at each slot boundary -- R (READ slot start, after
the barrier), S (fragments landed, MFMAs start), E (MFMAs issued) -- as medians per group
and quadrant over the steady-state k-tiles of the first tile.
usage: python scripts/gemm_stamps.py M N K wkm"""
import json
import os
import statistics as stt
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

M, N, K, wkm = (int(v) for v in sys.argv[1:5])
load_ext(required=True)
os.environ["ORION_GEMM_CFG"] = "7"
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
w = (torch.randn(*((K, N) if wkm else (N, K)), device="cuda", generator=g) * 0.5).to(torch.bfloat16)
buf = torch.zeros(8 * 1024, device="cuda", dtype=torch.int64)
os.environ["ORION_GEMM_DIAG"] = "0"
for _ in range(5):
    C().gemm(x, w, bool(wkm), 0, None, None)
os.environ["ORION_GEMM_DIAG"] = "4"
C().gemm(x, w, bool(wkm), 0, None, buf)
torch.cuda.synchronize()
os.environ["ORION_GEMM_DIAG"] = "0"
st = buf.view(8, 1024).cpu().tolist()
nk = K // 64
rec = {"shape": f"{M}x{N}x{K}x{wkm}"}
# per phase 3 stamps (R, S, E); first tile's phases 0 .. 4 nk - 1
per_phase = []
for grp in (0, 1):
    for q in range(4):
        rd, wt, mm, gp = [], [], [], []
        for t in range(2, nk - 2):
            P = 4 * t + q
            if 3 * (P + 2) >= 1024:
                break
            for v in range(4 * grp, 4 * grp + 4):
                R, S, E = st[v][3 * P], st[v][3 * P + 1], st[v][3 * P + 2]
                Rn = st[v][3 * (P + 1)]
                rd.append(S - R)
                mm.append(E - S)
                gp.append(Rn - E)
                per_phase.append(Rn - R)
        if rd:
            rec[f"g{grp}q{q}"] = {"R_to_S": stt.median(rd), "S_to_E": stt.median(mm), "E_to_nextR": stt.median(gp)}
rec["phase_cycles_median"] = stt.median(per_phase) if per_phase else None
print(json.dumps(rec))
