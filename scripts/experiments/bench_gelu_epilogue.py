"""A/B: GPT-2 MLP GEMM + separate GELU kernels vs hipBLASLt GELU-epilogue GEMMs
(csrc/gemm_epilogue.hip), at 65,536 tokens x 768 -> 3072; numerics vs fp32."""
import torch
import torch.nn.functional as F
from orion_amd import ops
from orion_amd.tuning import use_tuned_gemms

use_tuned_gemms(None, verbose=True)
ops.load_ext(required=True)
C = torch.ops.orion_amd
M, K, N = 65536, 768, 3072
dev = "cuda"
torch.manual_seed(0)
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
wfc = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
bfc = (torch.randn(N, device=dev) * 0.1).bfloat16()
wpr = (torch.randn(K, N, device=dev) * 0.02).bfloat16()
dy = torch.randn(M, K, device=dev, dtype=torch.bfloat16) * 0.01


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def fwd_base():
    h = F.linear(x, wfc)
    return C.bias_gelu_fwd(h, bfc), h


def fwd_epi():
    return C.gemm_gelu_aux(x, wfc, bfc)


hnob = F.linear(x, wfc)
hfull = (hnob.float() + bfc.float()).bfloat16()
db = torch.empty(N, device=dev, dtype=torch.bfloat16)


def bwd_base():
    da = dy @ wpr
    return C.bias_gelu_bwd(da, hnob, bfc)


def bwd_epi():
    return C.gemm_dgelu_bgrad(dy, wpr, hfull, db)


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm()).item()


# numerics
import sys
try:
    a2, h2 = fwd_epi()
except RuntimeError as e:
    print("fwd epilogue unavailable:", e, flush=True)
    fwd_epi = None
    a2, h2 = fwd_base()
try:
    bwd_epi()
except RuntimeError as e:
    print("bwd epilogue unavailable:", e, flush=True)
    sys.exit(0)
href = x.float() @ wfc.float().t() + bfc.float()
aref = F.gelu(href, approximate="tanh")
print(f"fwd: rel(h) {rel(h2, href):.2e} rel(a) {rel(a2, aref):.2e}  "
      f"base rel(a) {rel(fwd_base()[0], aref):.2e}", flush=True)
dh2 = bwd_epi()
daref = dy.float() @ wpr.float()
hr = hfull.float().requires_grad_()
g = F.gelu(hr, approximate="tanh")
dhref, = torch.autograd.grad(g, hr, daref)
dbref = dhref.sum(0)
dhb, dbb = bwd_base()
print(f"bwd: rel(dh) {rel(dh2, dhref):.2e} rel(db) {rel(db, dbref):.2e}  "
      f"base rel(dh) {rel(dhb, dhref):.2e} rel(db) {rel(dbb, dbref):.2e}", flush=True)
tb, te = timeit(fwd_base), (timeit(fwd_epi) if fwd_epi else float("nan"))
print(f"fwd ms: base {tb:.3f}  epilogue {te:.3f}", flush=True)
tb, te = timeit(bwd_base), timeit(bwd_epi)
print(f"bwd ms: base {tb:.3f}  epilogue {te:.3f}", flush=True)
t_lin, t_dg = timeit(lambda: F.linear(x, wfc)), timeit(lambda: dy @ wpr)
print(f"plain F.linear fwd ms {t_lin:.3f}  dy@wpr ms {t_dg:.3f}", flush=True)
