"""The debug build (ORION_AMD_DEBUG=1 -> orion_amd/_C_debug.so: -O1 -g, device-side bounds
asserts via ORION_DASSERT) runs the hand-written kernels on ragged shapes without tripping
an assert, in a subprocess that loads it through ORION_AMD_EXT."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG_SO = os.path.join(ROOT, "orion_amd", "_C_debug.so")

SCRIPT = r"""
import math, torch
from orion_amd.ops._ext import C, load_ext, EXT_PATH
assert EXT_PATH.endswith("_C_debug.so"), EXT_PATH
load_ext(required=True)
ops = C()
g = torch.Generator(device="cuda").manual_seed(0)
r = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
x, w, b = r(300, 192), r(264, 192), r(264)
ops.gemm(x, w, False, 2, b, None)
ops.gemm(r(300, 256), r(256, 200), True, 3, None, r(300, 200))
ops.wgrad(r(320, 264), r(320, 136), None, 0)
ops.wgrad(r(8192, 264), r(8192, 136), None, 0)  # split-K work items
ops.gemm(r(777, 128), r(50304, 128), False, 0, None, None)  # persistent tile walk
q, k, v, do = r(1, 200, 4, 128), r(1, 328, 2, 128), r(1, 328, 2, 128), r(1, 200, 4, 128)
o, lse = ops.attn_fwd(q, k, v, True, 1 / math.sqrt(128))
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
ops.attn_bwd(do, q, k, v, o, lse, True, 1 / math.sqrt(128), dq, dk, dv, 4)
torch.cuda.synchronize()
print("debug build ok")
"""


@pytest.mark.skipif(not os.path.isfile(DEBUG_SO),
                    reason="debug build not present (ORION_AMD_DEBUG=1 python -m orion_amd.build)")
def test_debug_build_kernels_pass_their_bounds_asserts():
    # PYTHONPATH is prepended to, not replaced: the harness's own entries (which record the
    # native libraries a process loads) must reach this child too
    env = dict(os.environ, ORION_AMD_EXT=DEBUG_SO,
               PYTHONPATH=os.pathsep.join(p for p in (ROOT, os.environ.get("PYTHONPATH")) if p))
    out = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True,
                         timeout=180, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "debug build ok" in out.stdout
