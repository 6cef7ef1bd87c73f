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


@pytest.fixture(params=["7", "9"], ids=["mfma32", "mfma16"])
def gemm_cfg(request, monkeypatch):
    """The phased kernel on v_mfma_f32_32x32x16 (csrc/gemm_phased.hip, 7) and on
    v_mfma_f32_16x16x32 (csrc/gemm16.hip, 9)."""
    monkeypatch.setenv("ORION_GEMM_CFG", request.param)
    return request.param


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("wkm", [False, True])
def test_gemm_store(M, N, K, wkm, gemm_cfg):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x = _rnd(g, M, K)
    w = _rnd(g, K, N) if wkm else _rnd(g, N, K)
    out, _ = _C().gemm(x, w, wkm, 0, None, None)
    want = x.float() @ (w.float() if wkm else w.float().t())
    assert out.shape == (M, N)
    assert rel_err(out, want) < 1e-2


@pytest.mark.parametrize("M,N,K", SHAPES[:6])
def test_gemm_bias_and_bias_gelu(M, N, K, gemm_cfg):
    g = torch.Generator(device=DEV).manual_seed(7 + M)
    x, w, b = _rnd(g, M, K), _rnd(g, N, K), _rnd(g, N)
    a = x.float() @ w.float().t() + b.float()
    out, none = _C().gemm(x, w, False, 1, b, None)
    assert rel_err(out, a) < 1e-2
    pre, h = _C().gemm(x, w, False, 2, b, None)
    assert rel_err(pre, a) < 1e-2
    assert rel_err(h, ref.gelu_tanh(a)) < 1e-2


@pytest.mark.parametrize("M,N,K", SHAPES[:6])
def test_gemm_gelu_backward_epilogue(M, N, K, gemm_cfg):
    g = torch.Generator(device=DEV).manual_seed(11 + N)
    dy, w, pre = _rnd(g, M, K), _rnd(g, K, N), _rnd(g, M, N)
    out, _ = _C().gemm(dy, w, True, 3, None, pre)
    want = (dy.float() @ w.float()) * _gelu_grad(pre.float())
    assert rel_err(out, want) < 1e-2


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (1000, 768, 768), (4096, 3072, 768), (777, 264, 128)])
@pytest.mark.parametrize("cfg", ["9", "7", "8", "0"])
@pytest.mark.parametrize("arena", [None, torch.float32, torch.bfloat16])
def test_gemm_gelu_bwd_with_bias_grad(M, N, K, cfg, arena, monkeypatch):
    """gemm_gelu_bwd: da = (dy w) * GELU'(pre + b) and db = colsum(da) (per-64-row partials
    from the phased kernel's epilogue, cfg 7/8; a column-sum pass after csrc/gemm.hip's
    kernel, cfg 0), db returned or written into a gradient-arena slice."""
    monkeypatch.setenv("ORION_GEMM_CFG", cfg)
    g = torch.Generator(device=DEV).manual_seed(M + N + 5 * K)
    dy, w, pre, b = _rnd(g, M, K), _rnd(g, K, N), _rnd(g, M, N), _rnd(g, N)
    want = (dy.float() @ w.float()) * _gelu_grad(pre.float() + b.float())
    out = None if arena is None else torch.full((N,), 7.0, device=DEV, dtype=arena)
    da, db = _C().gemm_gelu_bwd(dy, w, pre, b, out)
    assert rel_err(da, want) < 1e-2
    got = db if arena is None else out
    assert (db is None or db.numel() == 0) if arena is not None else db.shape == (N,)
    assert rel_err(got, want.sum(0)) < 1e-2


def test_gemm_gelu_bwd_without_bias():
    g = torch.Generator(device=DEV).manual_seed(21)
    dy, w, pre = _rnd(g, 640, 256), _rnd(g, 256, 512), _rnd(g, 640, 512)
    da, db = _C().gemm_gelu_bwd(dy, w, pre, None, None)
    want = (dy.float() @ w.float()) * _gelu_grad(pre.float())
    assert rel_err(da, want) < 1e-2
    assert rel_err(db, want.sum(0)) < 1e-2


@pytest.mark.parametrize("fuse_out_bias", [False, True])
def test_fused_mlp_tail_matches_two_node_path(fuse_out_bias, monkeypatch):
    """ops.gelu_linear (one autograd node, backward = one GEMM with GELU' and the fc-bias
    gradient in its epilogue) against bias_gelu -> linear: output and every gradient."""
    from orion_amd import ops
    from orion_amd.ops import activations
    g = torch.Generator(device=DEV).manual_seed(4)
    a = _rnd(g, 2, 384, 3072)
    bfc, w, b = _rnd(g, 3072), _rnd(g, 768, 3072) * 0.05, _rnd(g, 768)
    dy = _rnd(g, 2, 384, 768)
    res = []
    for fused in (True, False):
        monkeypatch.setattr(activations, "_FUSED_MLP", fused)
        ts = [t.clone().requires_grad_() for t in (a, bfc, w, b)]
        y = ops.gelu_linear(ts[0], ts[1], ts[2], None if fuse_out_bias else ts[3])
        y.backward(dy)
        res.append([y] + [t.grad for t in ts[:3]] + ([] if fuse_out_bias else [ts[3].grad]))
    for name, x, y in zip(("y", "da", "dbfc", "dw", "db"), *res):
        assert rel_err(x, y) < 1e-2, (name, rel_err(x, y))


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
@pytest.mark.parametrize("cfg", ["0", "8", "7", "9"])
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
@pytest.mark.parametrize("cfg", ["9", "7", "8", "0"])
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
