#!/usr/bin/env python3
"""Per-CU timeline of csrc/gemm16.hip from its stamped diagnostic instantiation
(gemm_diag(4)): for every workgroup the start, prologue-landed,
main-loop-end and epilogue-issued s_memtime stamps plus the CU it ran on (HW_ID / XCC_ID);
with --wait (DIAG 4 | 32) also when its stores were acknowledged.  Reports, per CU and then
as medians over CUs: the share of the CU's span in prologue / main loop / epilogue and the
gap between one workgroup's last epilogue instruction and the next workgroup's first
instruction on the same CU (dispatch + whatever the hardware waits for).

usage: python scripts/gemm16_timeline.py M N K [--wait]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C, load_ext  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
wait = "--wait" in sys.argv
load_ext(required=True)
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
nwg = ((M + 255) // 256) * ((N + 255) // 256)
buf = torch.zeros(nwg * 8 * 20, device="cuda", dtype=torch.int64)
C().gemm_diag(0)
for _ in range(10):
    C().gemm(x, w, False, 0, None, None)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    C().gemm(x, w, False, 0, None, None)
b.record()
b.synchronize()
plain_ms = a.elapsed_time(b) / 10
C().gemm_diag(4 | (32 if wait else 0))
a.record()
C().gemm(x, w, False, 0, None, buf)
b.record()
b.synchronize()
diag_ms = a.elapsed_time(b)
C().gemm_diag(0)
st = buf.view(nwg, 8, 20).cpu().to(torch.float64)
hw = buf.view(nwg, 8, 20)[:, 0, 16].cpu()
start = st[:, :, 0].min(1).values
landed = st[:, :, 1].max(1).values
loop_end = st[:, :, 14].max(1).values
epi = st[:, :, 15].max(1).values
ack = st[:, :, 17].max(1).values
hwid = (hw & 0xFFFFFFFF)
cu = (hwid >> 8) & 0xF
sh = (hwid >> 12) & 0x1
se = (hwid >> 13) & 0x7
xcc = (hw >> 32) & 0xF
key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
by = {}
for i in range(nwg):
    by.setdefault(int(key[i]), []).append(i)
gaps, shares, per_cu_wg = [], {"prologue": [], "main": [], "epilogue": [], "gap": []}, []
acks = []
for k, ids in by.items():
    ids.sort(key=lambda i: float(start[i]))
    per_cu_wg.append(len(ids))
    span = float(epi[ids[-1]] - start[ids[0]])
    pro = sum(float(landed[i] - start[i]) for i in ids)
    main = sum(float(loop_end[i] - landed[i]) for i in ids)
    ep = sum(float(epi[i] - loop_end[i]) for i in ids)
    gp = [float(start[j] - epi[i]) for i, j in zip(ids, ids[1:])]
    gaps += gp
    if span > 0:
        shares["prologue"].append(pro / span)
        shares["main"].append(main / span)
        shares["epilogue"].append(ep / span)
        shares["gap"].append(sum(gp) / span)
    if wait:
        acks += [float(ack[i] - epi[i]) for i in ids]


def med(v):
    v = sorted(v)
    return round(v[len(v) // 2], 3) if v else None


rec = {"shape": f"{M}x{N}x{K}", "workgroups": nwg, "cus_seen": len(by), "wg_per_cu_median": med(per_cu_wg),
       "plain_ms": round(plain_ms, 4), "diag_ms": round(diag_ms, 4), "wait_for_stores": wait,
       "cycles_median": {"prologue": med((landed - start).tolist()), "main": med((loop_end - landed).tolist()),
                         "epilogue": med((epi - loop_end).tolist()), "gap_to_next_wg": med(gaps)},
       "share_of_cu_span_median": {k: med(v) for k, v in shares.items()}}
if wait:
    rec["cycles_median"]["store_ack_after_issue"] = med(acks)
print(json.dumps(rec), flush=True)
