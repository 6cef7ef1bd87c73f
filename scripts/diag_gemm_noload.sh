cd $GRAFT_REPO_ROOT
for cfg in 1 2 3; do for d in 0 2; do
ORION_GEMM_CFG=$cfg ORION_GEMM_DIAG=$d timeout 120 python - <<'PY'
import torch, os, sys
sys.path.insert(0, '.')
from orion_amd.ops._ext import C, load_ext
load_ext(required=True)
M,N,K=65536,768,3072
x=torch.randn(M,K,device='cuda').bfloat16(); w=torch.randn(N,K,device='cuda').bfloat16()
for _ in range(3): C().gemm(x,w,False,0,None,None)
torch.cuda.synchronize()
a,b=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20): C().gemm(x,w,False,0,None,None)
b.record(); b.synchronize()
ms=a.elapsed_time(b)/20
print(os.environ['ORION_GEMM_CFG'], os.environ['ORION_GEMM_DIAG'], round(ms,4), round(2*M*N*K/ms/1e9,1), 'TF/s')
PY
done; done
