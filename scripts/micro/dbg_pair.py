import torch, sys
sys.path.insert(0, "/root/repo")
from orion_amd.ops._ext import C, load_ext
load_ext(required=True)
c = C()
for (M, N, K) in [(300, 264, 128), (256, 264, 128), (300, 256, 128), (256, 256, 128), (512, 512, 64)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).bfloat16()
    w = (torch.randn(K, N, device="cuda", generator=g) * 0.5).bfloat16()
    c.gemm_diag(0x2000)
    out, _ = c.gemm(x, w, True, 0, None, None)
    torch.cuda.synchronize()
    want = x.float() @ w.float()
    err = (out.float() - want).abs()
    bad = (err > 0.05 * want.abs().max()) | ~torch.isfinite(out.float())
    print(M, N, K, "bad", int(bad.sum()), "of", bad.numel())
    if bad.any():
        idx = bad.nonzero()
        print("  rows", idx[:, 0].min().item(), idx[:, 0].max().item(), "cols", idx[:, 1].min().item(), idx[:, 1].max().item())
        rows = sorted(set(idx[:, 0].tolist()))
        cols = sorted(set(idx[:, 1].tolist()))
        print("  nrows", len(rows), rows[:20], "ncols", len(cols), cols[:40])
