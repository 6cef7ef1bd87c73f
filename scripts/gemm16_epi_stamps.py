#!/usr/bin/env python3
"""Epilogue anatomy of csrc/gemm16.hip on the persistent walk (gemm_diag(4 | 128)): for the
middle item of every workgroup, every wave stamps s_memtime around its epilogue and at the
exits of the next item's first k-tile (phase 0 vmcnt wait, its barrier, phase 1 wait, barrier).
Prints medians (cycles) per group: the middle k-tile, the epilogue, and the four waits.
usage: python scripts/gemm16_epi_stamps.py [M N K]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (65536, 3072, 768)
load_ext(required=True)
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(M, K, device="cuda", generator=g)).to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
b = (torch.randn(N, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
buf = torch.zeros(256 * 8 * 20, device="cuda", dtype=torch.int64)
ops = C()
for epi in (0, 1, 2):
    bias = b if epi else None
    ops.gemm_diag(0)
    for _ in range(5):
        ops.gemm(x, w, False, epi, bias, None)
    ops.gemm_diag(4 | 128)
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.gemm(x, w, False, epi, bias, buf)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ops.gemm_diag(0)
    st = buf.view(256, 8, 20).cpu().double()
    rec = {"epi": epi, "shape": f"{M}x{N}x{K}", "ms_stamped": round(sorted(ts)[1], 4)}
    for grp in (0, 1):
        s = st[:, 4 * grp: 4 * grp + 4, :].reshape(-1, 20)
        s = s[(s[:, 19] > 0) & (s[:, 14] > 0)]
        med = lambda a: float(a.median())
        rec[f"g{grp}"] = {"ktile": med(s[:, 13] - s[:, 2]), "epilogue": med(s[:, 15] - s[:, 14]),
                          "next_p0_wait": med(s[:, 16] - s[:, 15]), "next_p0_bar": med(s[:, 17] - s[:, 16]),
                          "next_p1_wait": med(s[:, 18] - s[:, 17]), "next_p1_bar": med(s[:, 19] - s[:, 18]),
                          "waves": int(s.shape[0])}
    print(json.dumps(rec), flush=True)
