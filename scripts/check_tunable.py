#!/usr/bin/env python3
"""A/B one tuned GEMM shape with TunableOp on/off to verify the committed table is applied."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n


x = torch.randn(32768, 768, device="cuda", dtype=torch.bfloat16)
w = torch.randn(50304, 768, device="cuda", dtype=torch.bfloat16)
w2 = torch.randn(3072, 768, device="cuda", dtype=torch.bfloat16)
f1 = lambda: torch.nn.functional.linear(x, w)
f2 = lambda: torch.nn.functional.linear(x, w2)
print("default  lm_head %.3f ms  c_fc %.3f ms" % (t(f1), t(f2)))
from orion_amd.tuning import use_tuned_gemms
n = use_tuned_gemms(verbose=True)
tun = torch.cuda.tunable
print("enabled", tun.is_enabled(), "tuning", tun.tuning_is_enabled(), "file", tun.get_filename())
print("tuned    lm_head %.3f ms  c_fc %.3f ms" % (t(f1), t(f2)))
res = tun.get_results()
print(len(res), res[:3])
