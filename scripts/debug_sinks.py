"""Per-slot comparison: direct-to-arena gradients vs the AccumulateGrad path (GPU)."""
import torch
from orion_amd import ops
from orion_amd.models import build_model
from orion_amd.train.flat import FlatArena

ops.load_ext(required=True)
torch.manual_seed(0)
m1 = build_model("gpt2-tiny").cuda()
m2 = build_model("gpt2-tiny").cuda()
m2.load_state_dict(m1.state_dict())
a1, a2 = FlatArena(m1), FlatArena(m2)
a2.detach_sinks()
g = torch.Generator().manual_seed(100)
data = [(torch.randint(0, 50257, (2, 64), generator=g).cuda(), torch.randint(0, 50257, (2, 64), generator=g).cuda())
        for _ in range(2)]
for nmb in (1, 2):
    for m, a in ((m1, a1), (m2, a2)):
        a.zero_grad()
        for x, y in data[:nmb]:
            _, loss = m(x, y)
            (loss / nmb).backward()
    torch.cuda.synchronize()
    print("micro-batches", nmb)
    for s in a1.slots:
        g1 = a1.grads[s.offset:s.offset + s.numel].float()
        g2 = a2.grads[s.offset:s.offset + s.numel].float()
        e = ((g1 - g2).norm() / (g2.norm() + 1e-12)).item()
        if e > 1e-3:
            print(f"  {s.name:40s} err {e:.4f} |g1| {g1.norm().item():.4e} |g2| {g2.norm().item():.4e}")
