"""The one-shot launches of the fused AdamW and the elementwise kernels (csrc/adamw.hip,
csrc/activations.hip ``ew_grid``; round 5) against their grid-stride loop: the grid caps
ORION_ADAMW_GRID / ORION_EW_GRID are read once per process, so each form runs in a child
process on the same inputs and the parent compares the outputs bitwise.  A small cap makes
every thread loop many times (the path Llama-7B's 6.7 G-parameter arena takes past 2^22
workgroups)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[2])
from orion_amd.ops._ext import C, load_ext
load_ext(required=True)
g = torch.Generator(device="cuda").manual_seed(0)
n = 2048 * 301
p16 = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
master, m, v, gr = (torch.randn(n, device="cuda", generator=g) for _ in range(4))
v.abs_()
decay = (torch.arange(n // 2048, device="cuda") % 3 != 0).to(torch.uint8)
hyper = torch.tensor([6e-4, 0.9, 0.95, 1e-8, 0.1, 0.1, 0.05, 1.0], device="cuda")
sumsq = torch.full((1,), 4.0, device="cuda")
C().adamw_flat(p16, master, m, v, gr, decay, hyper, sumsq)
gu = torch.randn(257, 2 * 1032, device="cuda", generator=g).bfloat16()
h = C().swiglu_fwd(gu)
torch.save({"p16": p16.cpu(), "master": master.cpu(), "m": m.cpu(), "v": v.cpu(), "h": h.cpu()}, sys.argv[1])
"""


def _run(tmp_path, tag, env_extra):
    out = tmp_path / f"{tag}.pt"
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD, str(out), ROOT], env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    return torch.load(out, weights_only=True)


def test_one_shot_and_grid_stride_launches_agree(tmp_path):
    a = _run(tmp_path, "oneshot", {})
    b = _run(tmp_path, "loop", {"ORION_ADAMW_GRID": "3", "ORION_EW_GRID": "2"})
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert a["p16"].abs().sum() > 0 and a["h"].abs().sum() > 0
