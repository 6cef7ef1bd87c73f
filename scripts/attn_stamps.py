#!/usr/bin/env python3
"""Phase anatomy of the split dK/dV attention kernel (D = 64) from in-kernel s_memtime stamps.

usage: python scripts/attn_stamps.py [B T H]
Runs the stamped instantiation (ORION_ATTN_DIAG=1: the kernel writes per-wave phase sums over
the dQ buffer and the dQ kernel is skipped) and prints cycles per active query tile for
each phase, averaged over all waves, plus the lifetime split."""
import math
import os
import sys

os.environ["ORION_ATTN_DIAG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from orion_amd.ops._ext import C, load_ext  # noqa: E402

B, T, H = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (64, 1024, 12)
D = 64
load_ext(required=True)
g = torch.Generator(device="cuda").manual_seed(0)
mk = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)  # noqa: E731
q, k, v, do = mk(B, T, H, D), mk(B, T, H, D), mk(B, T, H, D), mk(B, T, H, D)
sc = 1 / math.sqrt(D)
o, lse = C().attn_fwd(q, k, v, True, sc)
dq, dk, dv = torch.zeros_like(q), torch.empty_like(k), torch.empty_like(v)
for _ in range(3):
    C().attn_bwd(do, q, k, v, o, lse, True, sc, dq, dk, dv, 4)
torch.cuda.synchronize()
nw = ((T + 127) // 128) * B * H * 4
st = dq.view(-1).view(torch.int64)[: nw * 8].view(nw, 8).cpu().double()
names = ["S/dP chain issue", "softmax (incl. MFMA wait)", "dV/dK issue", "stage write", "barrier"]
act = st[:, 5].sum().item()
tiles = st[:, 6].sum().item()
print(f"waves {nw}, active tiles {act:.0f} of {tiles:.0f} stepped")
tot = st[:, :5].sum(0)
for n, x in zip(names, tot):
    print(f"  {n:28s} {x.item() / act:8.0f} cycles / active tile")
life = st[:, 7].sum().item()
print(f"  lifetime per stepped tile   {life / tiles:8.0f} cycles (all phases {tot.sum().item() / tiles:.0f})")
