#!/usr/bin/env python3
"""Phase anatomy of the attention forward (csrc/attn_fwd.hip, D = 64, causal, two query blocks
per wave) from in-kernel s_memtime stamps.

usage: python scripts/attn_fwd_stamps.py [B T H]
Runs the stamped instantiation (ORION_ATTN_FWD_DIAG=1: the kernel writes per-wave phase sums
over the output O) and prints cycles per active key tile for each phase, averaged over all
waves, plus each wave's lifetime per stepped tile."""
import math
import os
import sys

os.environ["ORION_ATTN_FWD_DIAG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from orion_amd.ops._ext import C, load_ext  # noqa: E402

B, T, H = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (64, 1024, 12)
D = 64
load_ext(required=True)
g = torch.Generator(device="cuda").manual_seed(0)
mk = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)  # noqa: E731
q, k, v = mk(B, T, H, D), mk(B, T, H, D), mk(B, T, H, D)
for _ in range(3):
    o, lse = C().attn_fwd(q, k, v, True, 1 / math.sqrt(D))
torch.cuda.synchronize()
nw = ((T + 255) // 256) * B * H * 4
st = o.reshape(-1).view(torch.int64)[: nw * 8].view(nw, 8).cpu().double()
names = ["stage write + load issue", "K reads + S MFMA issue", "softmax (incl. S wait)", "V reads + PV issue",
         "barrier"]
act = st[:, 5].sum().item()
tiles = st[:, 6].sum().item()
print(f"waves {nw}, active tiles {act:.0f} of {tiles:.0f} stepped")
tot = st[:, :5].sum(0)
for n, x in zip(names, tot):
    print(f"  {n:28s} {x.item() / act:8.0f} cycles / active tile   {x.item() / tiles:8.0f} / stepped tile")
life = st[:, 7].sum().item()
print(f"  lifetime per stepped tile   {life / tiles:8.0f} cycles (all phases {tot.sum().item() / tiles:.0f})")
