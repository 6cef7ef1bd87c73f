#!/usr/bin/env python3
"""Run the HIP wgrad kernel on one GPT-2 shape a few times (for rocprofv3 PMC runs)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.ops._ext import C  # noqa: E402

M, n1, n2 = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (65536, 3072, 768)))
dy = torch.randn(M, n1, device="cuda", dtype=torch.bfloat16)
x = torch.randn(M, n2, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    C().wgrad(dy, x, None, 0)
torch.cuda.synchronize()
print("ok")
