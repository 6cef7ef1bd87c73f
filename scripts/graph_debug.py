#!/usr/bin/env python3
"""Per-step loss of eager vs graph-captured Trainer steps, built exactly like bench.py."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.models import build_model  # noqa: E402
from orion_amd.train.engine import Trainer, OptimConfig  # noqa: E402

B, T = int(os.environ.get("GD_B", 8)), int(os.environ.get("GD_T", 256))
name = os.environ.get("GD_MODEL", "gpt2-tiny")
dev = torch.device("cuda", 0)
if os.environ.get("GD_SETDEV") == "1":
    torch.cuda.set_device(0)
if os.environ.get("GD_LOADEXT") == "1":
    from orion_amd import ops
    ops.load_ext(required=True)
res = {}
order = [g == "1" for g in os.environ.get("GD_ORDER", "0,1").split(",")]
for graph in order:
    torch.manual_seed(1337)
    with torch.device(dev):
        m = build_model(name, block_size=max(1024, T))
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    pool = [(torch.randint(0, 50257, (B, T), device=dev, generator=g),
             torch.randint(0, 50257, (B, T), device=dev, generator=g)) for _ in range(4)]
    tr = Trainer(m, OptimConfig(warmup_iters=10, lr_decay_iters=10000), graph=graph)
    res[graph] = []
    for i in range(25):
        if os.environ.get("GD_SYNC5") == "1" and i == 5:
            torch.cuda.synchronize()
        loss = tr.step([pool[i % 4]])
        res[graph].append(round(float(loss), 4))
    print("graph" if graph else "eager", res[graph], flush=True)
print("max abs diff", max(abs(a - b) for a, b in zip(res[False], res[True])))
