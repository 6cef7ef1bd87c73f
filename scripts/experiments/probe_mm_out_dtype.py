import torch
a = torch.randn(512, 256, device="cuda").bfloat16()
b = torch.randn(512, 384, device="cuda").bfloat16()
ref = a.float().t() @ b.float()
o = torch.zeros(256, 384, device="cuda")
for name, fn in [
    ("mm_out_dtype_out", lambda: torch.mm(a.t(), b, out_dtype=torch.float32, out=o)),
    ("addmm_out_dtype_out", lambda: torch.addmm(o, a.t(), b, out_dtype=torch.float32, out=o)),
    ("addmm_out_dtype", lambda: o.copy_(torch.addmm(o, a.t(), b, out_dtype=torch.float32))),
]:
    try:
        o.zero_(); fn(); fn() if name.startswith("addmm") else None
        want = ref * (2 if name.startswith("addmm") else 1)
        print(name, "ok", float((o - want).abs().max()))
    except Exception as e:
        print(name, "ERR", str(e)[:150])
