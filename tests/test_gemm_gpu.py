"""The linear-layer GEMMs (csrc/gemm_phased.hip by default, csrc/gemm.hip's 2-stage kernel
under ORION_GEMM_CFG=0; forward NT / input-gradient NN with fused epilogues) against an fp32
PyTorch reference, including ragged M and N (partial 256 x 256 tiles), more tiles than CUs
(the persistent tile walk: 777 x 50304) and the epilogues (bias, bias + GELU with the
pre-activation output, GELU backward)."""
import pytest
import torch

from orion_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _C():
    from orion_amd.ops._ext import C, load_ext
    load_ext(required=True)
    return C()


def _rnd(g, *s):
    return (torch.randn(*s, device=DEV, generator=g) * 0.5).to(torch.bfloat16)


def _gelu_grad(z):
    return torch.func.vmap(torch.func.grad(lambda t: ref.gelu_tanh(t)))(z.reshape(-1)).view_as(z)


SHAPES = [(256, 256, 64), (300, 264, 128), (1000, 768, 768), (513, 1000, 192), (64, 8, 64),
          (4096, 2304, 768), (2048, 3072, 768), (1024, 768, 3072), (777, 50304, 128)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("wkm", [False, True])
def test_gemm_store(M, N, K, wkm):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x = _rnd(g, M, K)
    w = _rnd(g, K, N) if wkm else _rnd(g, N, K)
    out, _ = _C().gemm(x, w, wkm, 0, None, None)
    want = x.float() @ (w.float() if wkm else w.float().t())
    assert out.shape == (M, N)
    assert rel_err(out, want) < 1e-2


@pytest.mark.parametrize("M,N,K", SHAPES[:6])
def test_gemm_bias_and_bias_gelu(M, N, K):
    g = torch.Generator(device=DEV).manual_seed(7 + M)
    x, w, b = _rnd(g, M, K), _rnd(g, N, K), _rnd(g, N)
    a = x.float() @ w.float().t() + b.float()
    out, none = _C().gemm(x, w, False, 1, b, None)
    assert rel_err(out, a) < 1e-2
    pre, h = _C().gemm(x, w, False, 2, b, None)
    assert rel_err(pre, a) < 1e-2
    assert rel_err(h, ref.gelu_tanh(a)) < 1e-2


@pytest.mark.parametrize("M,N,K", SHAPES[:6])
def test_gemm_gelu_backward_epilogue(M, N, K):
    g = torch.Generator(device=DEV).manual_seed(11 + N)
    dy, w, pre = _rnd(g, M, K), _rnd(g, K, N), _rnd(g, M, N)
    out, _ = _C().gemm(dy, w, True, 3, None, pre)
    want = (dy.float() @ w.float()) * _gelu_grad(pre.float())
    assert rel_err(out, want) < 1e-2


def test_gemm_batched_input_shape_and_strided_rows():
    g = torch.Generator(device=DEV).manual_seed(3)
    x = _rnd(g, 4, 96, 256)
    w = _rnd(g, 512, 256)
    out, _ = _C().gemm(x, w, False, 0, None, None)
    assert out.shape == (4, 96, 512)
    assert rel_err(out, x.float() @ w.float().t()) < 1e-2
    big = _rnd(g, 300, 2304)           # a column slice of a wider buffer (row stride 2304)
    xs = big[:, 768:1536]
    out2, _ = _C().gemm(xs, w[:, :256].contiguous().repeat(1, 3), False, 0, None, None)
    assert rel_err(out2, xs.float() @ w[:, :256].float().repeat(1, 3).t()) < 1e-2


@pytest.mark.parametrize("M,N,K", [(300, 264, 128), (1000, 768, 768), (777, 50304, 128)])
@pytest.mark.parametrize("wkm", [False, True])
@pytest.mark.parametrize("cfg", ["0", "8"])
def test_gemm_other_schedules(M, N, K, wkm, cfg, monkeypatch):
    """csrc/gemm.hip's 2-stage kernel (ORION_GEMM_CFG=0) and the phased kernel's 4-quadrant
    schedule (8); the variable is read per call."""
    monkeypatch.setenv("ORION_GEMM_CFG", cfg)
    g = torch.Generator(device=DEV).manual_seed(M + 3 * N + K)
    x = _rnd(g, M, K)
    w = _rnd(g, K, N) if wkm else _rnd(g, N, K)
    out, _ = _C().gemm(x, w, wkm, 0, None, None)
    assert rel_err(out, x.float() @ (w.float() if wkm else w.float().t())) < 1e-2


@pytest.mark.parametrize("M,N1,N2", [(8192, 264, 136), (65536, 768, 768), (4096, 3072, 768), (8224, 200, 264)])
@pytest.mark.parametrize("cfg", ["7", "8", "0"])
@pytest.mark.parametrize("acc", [False, True])
def test_wgrad_phased_and_two_stage_into_fp32(M, N1, N2, cfg, acc, monkeypatch):
    """Weight gradients on the phased kernel (split-K work items, fp32 slabs) and on
    csrc/wgrad.hip (ORION_WGRAD_CFG=0) into an fp32 arena slice, overwrite and accumulate
    (8224 tokens: not a multiple of 64, so the phased default hands over to csrc/wgrad.hip)."""
    monkeypatch.setenv("ORION_WGRAD_CFG", cfg)
    g = torch.Generator(device=DEV).manual_seed(M + N1)
    dy, x = _rnd(g, M, N1), _rnd(g, M, N2)
    out = torch.randn(N1, N2, device=DEV, generator=g)
    base = out.clone()
    _C().wgrad_into(dy, x, None, out, acc, 0)
    want = dy.float().t() @ x.float() + (base if acc else 0)
    assert rel_err(out, want) < 1e-4
