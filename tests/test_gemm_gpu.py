"""The linear-layer GEMMs of csrc/gemm16.hip (forward NT / input-gradient NN with fused
epilogues, weight gradients with split-K) against an fp32 PyTorch reference, including ragged
M and N (partial 256 x 256 tiles), more work items than CUs (the persistent walk: 777 x 50304
has 4 x 197 items for 256 workgroups, i.e. items of different lengths meet inside one
workgroup's continuous DMA stream) and the epilogues (bias, bias + GELU with the
pre-activation output, GELU backward with column sums).  Every shape runs on the persistent
walk (the default) and with one workgroup per work item (gemm_diag(64)).  Error budgets: the
in-tree result may be at most 2x as far from fp32 as the same product in stock PyTorch bf16
(tests/tolerance.py)."""
import pytest
import torch

from orion_amd.ops import reference as ref
from tolerance import rel_err, within_bf16_budget

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _C():
    from orion_amd.ops._ext import C, load_ext
    load_ext(required=True)
    return C()


def _rnd(g, *s):
    return (torch.randn(*s, device=DEV, generator=g) * 0.5).to(torch.bfloat16)


def _gelu_grad(z):
    return torch.func.vmap(torch.func.grad(lambda t: ref.gelu_tanh(t)))(z.reshape(-1)).view_as(z)


SHAPES = [(256, 256, 64), (300, 264, 128), (1000, 768, 768), (513, 1000, 192), (64, 8, 64),
          (4096, 2304, 768), (2048, 3072, 768), (1024, 768, 3072), (777, 50304, 128),
          (65536, 768, 768)]


@pytest.fixture(params=["persistent", "per_item"])
def gemm_cfg(request):
    """gemm16's persistent walk (one workgroup per CU, continuous DMA stream across items)
    and the one-workgroup-per-item launch (diagnostic flag 64)."""
    C = _C()
    old = C.gemm_diag(64 if request.param == "per_item" else 0)
    yield request.param
    C.gemm_diag(old)


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("wkm", [False, True])
def test_gemm_store(M, N, K, wkm, gemm_cfg):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x = _rnd(g, M, K)
    w = _rnd(g, K, N) if wkm else _rnd(g, N, K)
    out, _ = _C().gemm(x, w, wkm, 0, None, None)
    want = x.float() @ (w.float() if wkm else w.float().t())
    assert out.shape == (M, N)
    within_bf16_budget("out", out, want, x @ (w if wkm else w.t()))


@pytest.mark.parametrize("M,N,K", SHAPES[:6])
def test_gemm_bias_and_bias_gelu(M, N, K, gemm_cfg):
    g = torch.Generator(device=DEV).manual_seed(7 + M)
    x, w, b = _rnd(g, M, K), _rnd(g, N, K), _rnd(g, N)
    a = x.float() @ w.float().t() + b.float()
    ab = torch.nn.functional.linear(x, w, b)
    out, none = _C().gemm(x, w, False, 1, b, None)
    within_bf16_budget("bias", out, a, ab)
    pre, h = _C().gemm(x, w, False, 2, b, None)
    within_bf16_budget("pre", pre, a, ab)
    within_bf16_budget("gelu", h, ref.gelu_tanh(a), torch.nn.functional.gelu(ab, approximate="tanh"))


@pytest.mark.parametrize("M,N,K", SHAPES[:6])
def test_gemm_gelu_backward_epilogue(M, N, K, gemm_cfg):
    g = torch.Generator(device=DEV).manual_seed(11 + N)
    dy, w, pre = _rnd(g, M, K), _rnd(g, K, N), _rnd(g, M, N)
    out, _ = _C().gemm(dy, w, True, 3, None, pre)
    want = (dy.float() @ w.float()) * _gelu_grad(pre.float())
    within_bf16_budget("da", out, want, (dy @ w) * _gelu_grad(pre.float()).bfloat16())


@pytest.mark.parametrize("M,N,K", SHAPES[:6])
def test_gemm_gelu_derivative_forms(M, N, K, gemm_cfg):
    """The derivative form of the fused MLP (ORION_GELU_DERIV): the forward epilogue returns
    (GELU'(a), gelu(a)) for a = x w^T + b (epi 2 | 0x100), and gemm_gelu_bwd with
    pre_is_deriv multiplies by that stored derivative -- against fp32, and the backward equal
    to the pre-activation form within the bf16 budget."""
    g = torch.Generator(device=DEV).manual_seed(13 + M + N)
    x, w, b = _rnd(g, M, K), _rnd(g, N, K), _rnd(g, N)
    a = x.float() @ w.float().t() + b.float()
    ab = torch.nn.functional.linear(x, w, b)
    d, h = _C().gemm(x, w, False, 0x102, b, None)
    within_bf16_budget("gelu'", d, _gelu_grad(a), _gelu_grad(ab.float()).bfloat16())
    within_bf16_budget("gelu", h, ref.gelu_tanh(a), torch.nn.functional.gelu(ab, approximate="tanh"))
    dy, w2 = _rnd(g, M, 384), _rnd(g, 384, N)
    da, db = _C().gemm_gelu_bwd(dy, w2, d, None, None, True)
    want = (dy.float() @ w2.float()) * _gelu_grad(a)
    base = (dy @ w2) * _gelu_grad(ab.float()).bfloat16()
    within_bf16_budget("da", da, want, base)
    within_bf16_budget("db", db, want.sum(0), base.float().sum(0).bfloat16())
    with pytest.raises(RuntimeError):  # the bias is inside the stored derivative
        _C().gemm_gelu_bwd(dy, w2, d, b, None, True)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (1000, 768, 768), (4096, 3072, 768), (777, 264, 128)])
@pytest.mark.parametrize("arena", [None, torch.float32, torch.bfloat16])
def test_gemm_gelu_bwd_with_bias_grad(M, N, K, arena, gemm_cfg):
    """gemm_gelu_bwd: da = (dy w) * GELU'(pre + b) and db = colsum(da) (per-64-row partials
    from gemm16's epilogue, folded by a second pass), db returned or written into a
    gradient-arena slice."""
    g = torch.Generator(device=DEV).manual_seed(M + N + 5 * K)
    dy, w, pre, b = _rnd(g, M, K), _rnd(g, K, N), _rnd(g, M, N), _rnd(g, N)
    gp = _gelu_grad(pre.float() + b.float())
    want = (dy.float() @ w.float()) * gp
    base = (dy @ w) * gp.bfloat16()
    out = None if arena is None else torch.full((N,), 7.0, device=DEV, dtype=arena)
    da, db = _C().gemm_gelu_bwd(dy, w, pre, b, out)
    within_bf16_budget("da", da, want, base)
    got = db if arena is None else out
    assert (db is None or db.numel() == 0) if arena is not None else db.shape == (N,)
    within_bf16_budget("db", got, want.sum(0), base.float().sum(0).to(arena or torch.bfloat16))


def test_gemm_gelu_bwd_without_bias():
    g = torch.Generator(device=DEV).manual_seed(21)
    dy, w, pre = _rnd(g, 640, 256), _rnd(g, 256, 512), _rnd(g, 640, 512)
    da, db = _C().gemm_gelu_bwd(dy, w, pre, None, None)
    gp = _gelu_grad(pre.float())
    want = (dy.float() @ w.float()) * gp
    base = (dy @ w) * gp.bfloat16()
    within_bf16_budget("da", da, want, base)
    within_bf16_budget("db", db, want.sum(0), base.float().sum(0).bfloat16())


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


@pytest.mark.parametrize("proj_bias", [False, True])
@pytest.mark.parametrize("fc_bias", [True, False])
def test_fused_mlp_matches_reference(proj_bias, fc_bias, monkeypatch):
    """ops.mlp on the GPU path with ORION_FUSED_MLP (bias + GELU in the fc GEMM's epilogue,
    GELU' + fc-bias column sums in the projection's input-gradient GEMM) against fp32 autograd
    of linear -> GELU-tanh -> linear: output and every gradient, ragged token count."""
    from orion_amd import ops
    from orion_amd.ops import activations
    monkeypatch.setattr(activations, "_FUSED_MLP", True)
    g = torch.Generator(device=DEV).manual_seed(5)
    x = _rnd(g, 3, 333, 256)
    wfc, bfc = _rnd(g, 1024, 256) * 0.1, _rnd(g, 1024)
    wp, bp = _rnd(g, 256, 1024) * 0.05, _rnd(g, 256)
    dy = _rnd(g, 3, 333, 256)
    ts = [t.clone().requires_grad_() for t in (x, wfc, bfc, wp, bp)]
    y = ops.mlp(ts[0], ts[1], ts[2] if fc_bias else None, ts[3], ts[4] if proj_bias else None)
    y.backward(dy)
    fs = [t.detach().float().requires_grad_() for t in (x, wfc, bfc, wp, bp)]
    a = fs[0] @ fs[1].t() + (fs[2] if fc_bias else 0)
    yr = ref.gelu_tanh(a) @ fs[3].t() + (fs[4] if proj_bias else 0)
    yr.backward(dy.float())
    bs = [t.detach().clone().requires_grad_() for t in (x, wfc, bfc, wp, bp)]
    F = torch.nn.functional
    yb = F.linear(F.gelu(F.linear(bs[0], bs[1], bs[2] if fc_bias else None), approximate="tanh"),
                  bs[3], bs[4] if proj_bias else None)
    yb.backward(dy)
    within_bf16_budget("y", y, yr, yb)
    names = ["dx", "dwfc", "dbfc", "dwproj", "dbproj"]
    for i, (n, t, f, bb) in enumerate(zip(names, ts, fs, bs)):
        if (i == 2 and not fc_bias) or (i == 4 and not proj_bias):
            assert t.grad is None
            continue
        within_bf16_budget(n, t.grad, f.grad, bb.grad)


def test_gemm_batched_input_shape_and_strided_rows():
    g = torch.Generator(device=DEV).manual_seed(3)
    x = _rnd(g, 4, 96, 256)
    w = _rnd(g, 512, 256)
    out, _ = _C().gemm(x, w, False, 0, None, None)
    assert out.shape == (4, 96, 512)
    within_bf16_budget("out", out, x.float() @ w.float().t(), x @ w.t())
    big = _rnd(g, 300, 2304)           # a column slice of a wider buffer (row stride 2304)
    xs = big[:, 768:1536]
    w3 = w[:, :256].contiguous().repeat(1, 3)
    out2, _ = _C().gemm(xs, w3, False, 0, None, None)
    within_bf16_budget("strided", out2, xs.float() @ w3.float().t(), xs @ w3.t())


@pytest.mark.parametrize("M,N1,N2", [(8192, 264, 136), (65536, 768, 768), (4096, 3072, 768), (8224, 200, 264),
                                     (16384, 50304, 768), (2048, 22016, 4096)])
@pytest.mark.parametrize("acc", [False, True])
def test_wgrad_into_fp32(M, N1, N2, acc, gemm_cfg):
    """Weight gradients on gemm16 (split-K work items into fp32 slabs, or straight into the
    arena) into an fp32 arena slice, overwrite and accumulate; 8224 tokens (not a multiple of
    64) take csrc/wgrad.hip's 32-row kernel; 50,304 x 768 is the LM head; 22,016 x 4,096 (Llama
    gate_up) takes the tail split (80 tile rows unsplit, 6 rows split-K into slabs)."""
    g = torch.Generator(device=DEV).manual_seed(M + N1)
    dy, x = _rnd(g, M, N1), _rnd(g, M, N2)
    out = torch.randn(N1, N2, device=DEV, generator=g)
    base = out.clone()
    _C().wgrad_into(dy, x, None, out, acc, 0)
    want = dy.float().t() @ x.float() + (base if acc else 0)
    # fp32 output, fp32 accumulation: far below any bf16 budget
    assert rel_err(out, want) < 1e-4


@pytest.mark.parametrize("M,N1,N2,R1", [(2048, 22016, 4096, 20480), (4096, 50304, 768, 43520)])
def test_wgrad_tail_split_bf16_scaled(M, N1, N2, R1):
    """The tail-split weight gradient into a bf16 output with a device scale: head rows and
    tail rows both scaled once (the head in its epilogue, the tail in the slab sum).  Llama's
    gate_up (whole tile rows), GPT-2's LM head (591 tiles: 170 rows unsplit, the last 26.5
    rows -- a partial row of tiles among them -- split-K over 3 chunks)."""
    g = torch.Generator(device=DEV).manual_seed(7)
    assert _C().wgrad_splits(M, N1, N2) == 1
    assert _C().wgrad_tail_rows(M, N1, N2)[0] == R1
    dy, x = _rnd(g, M, N1), _rnd(g, M, N2)
    sc = torch.tensor([0.25], device=DEV)
    out = _C().wgrad(dy, x, sc, 0)
    want = (dy.float().t() @ x.float()) * 0.25
    within_bf16_budget("dw", out, want, ((dy.t() @ x).float() * 0.25).bfloat16())
    assert rel_err(out[:R1], want[:R1]) < 5e-3 and rel_err(out[R1:], want[R1:]) < 5e-3


@pytest.mark.parametrize("M,N1,N2", [(4096, 768, 768), (8192, 2304, 768), (4096, 50304, 768), (1024, 1000, 264)])
def test_wgrad_transposed_x_matches(M, N1, N2, gemm_cfg):
    """x given as the transposed view of a row-major (N2, M) tensor takes the NT-operand
    weight-gradient kernel (the LM head's scaled activations, csrc/lmhead.hip): fp32 arena
    output against fp32 (split-K, tail split and ragged shapes), and bitwise equal to the
    k-major form on the same data (same fragments, same MFMA order)."""
    g = torch.Generator(device=DEV).manual_seed(M + N1 + N2)
    dy, x = _rnd(g, M, N1), _rnd(g, M, N2)
    xt = x.t().contiguous().t()  # (M, N2) view, stride (1, M)
    assert xt.stride(0) == 1
    out_t = torch.zeros(N1, N2, device=DEV)
    out_k = torch.zeros(N1, N2, device=DEV)
    _C().wgrad_into(dy, xt, None, out_t, False, 0)
    _C().wgrad_into(dy, x, None, out_k, False, 0)
    want = dy.float().t() @ x.float()
    assert rel_err(out_t, want) < 1e-4
    assert torch.equal(out_t, out_k)


@pytest.mark.parametrize("wkm", [False, True])
def test_gemm16_operands_past_4gb(wkm, monkeypatch):
    """csrc/gemm16.hip bases its buffer resources at the work item's tile, so a > 4 GB
    operand (the LM head's logits: 65,536 x 50,304 bf16 = 6.6 GB) stays on the kernel: the
    forward writes a 4.4 GB output, the input gradient reads a 4.4 GB operand.  Rows at both
    ends checked against fp32."""
    g = torch.Generator(device=DEV).manual_seed(7)
    M, V = 43776, 50304
    if not wkm:  # out (M, V) = x (M, 64) W (V, 64)^T
        x, w = _rnd(g, M, 64), _rnd(g, V, 64)
        out, _ = _C().gemm(x, w, False, 0, None, None)
        for rows in (slice(0, 256), slice(M - 300, M)):
            within_bf16_budget("fwd rows", out[rows], x[rows].float() @ w.float().t(), x[rows] @ w.t())
    else:  # out (M, 128) = dl (M, V) W (V, 128)
        dl, w = _rnd(g, M, V), _rnd(g, V, 128)
        out, _ = _C().gemm(dl, w, True, 0, None, None)
        for rows in (slice(0, 256), slice(M - 300, M)):
            within_bf16_budget("dgrad rows", out[rows], dl[rows].float() @ w.float(), dl[rows] @ w)


@pytest.mark.parametrize("M,C_,F_", [(333, 256, 512), (4096, 1024, 2752), (1000, 512, 1376)])
def test_gemm_swiglu_bwd_epilogue(M, C_, F_, gemm_cfg):
    """gemm_swiglu_bwd: dh = dy W_down (W_down (C, F) read k-major) with the SwiGLU backward in
    the epilogue: dgate = dh up silu'(gate), dup = dh silu(gate) into the packed (M, 2F)."""
    g = torch.Generator(device=DEV).manual_seed(M + F_)
    dy, w, gu = _rnd(g, M, C_), _rnd(g, C_, F_), _rnd(g, M, 2 * F_)
    got = _C().gemm_swiglu_bwd(dy, w, gu)
    gr = gu.float().requires_grad_()
    ga, ua = gr.chunk(2, -1)
    (torch.nn.functional.silu(ga) * ua).backward(dy.float() @ w.float())
    gb = gu.clone().requires_grad_()
    a_, b_ = gb.chunk(2, -1)
    (torch.nn.functional.silu(a_) * b_).backward(dy @ w)
    assert got.shape == (M, 2 * F_)
    within_bf16_budget("dgate", got[:, :F_], gr.grad[:, :F_], gb.grad[:, :F_])
    within_bf16_budget("dup", got[:, F_:], gr.grad[:, F_:], gb.grad[:, F_:])


@pytest.mark.parametrize("F_", [1376, 1408])
def test_swiglu_mlp_matches_reference(F_):
    """ops.swiglu_mlp (Llama feed-forward, SwiGLU backward fused into the down_proj input
    gradient GEMM; F = 1408 also the SwiGLU forward in the gate_up GEMM's epilogue, 1376 the
    swiglu pass) against fp32 autograd: output and every gradient, ragged token count."""
    from orion_amd import ops
    g = torch.Generator(device=DEV).manual_seed(9)
    x = _rnd(g, 3, 111, 512)
    wgu, wd = _rnd(g, 2 * F_, 512) * 0.1, _rnd(g, 512, F_) * 0.05
    dy = _rnd(g, 3, 111, 512)
    ts = [t.clone().requires_grad_() for t in (x, wgu, wd)]
    y = ops.swiglu_mlp(*ts)
    y.backward(dy)
    fs = [t.detach().float().requires_grad_() for t in (x, wgu, wd)]
    ga, ua = (fs[0] @ fs[1].t()).chunk(2, -1)
    yr = (torch.nn.functional.silu(ga) * ua) @ fs[2].t()
    yr.backward(dy.float())
    bs = [t.detach().clone().requires_grad_() for t in (x, wgu, wd)]
    gb_, ub_ = (bs[0] @ bs[1].t()).chunk(2, -1)
    yb = (torch.nn.functional.silu(gb_) * ub_) @ bs[2].t()
    yb.backward(dy)
    within_bf16_budget("y", y, yr, yb)
    for n, t, f, b in zip(("dx", "dwgu", "dwdown"), ts, fs, bs):
        within_bf16_budget(n, t.grad, f.grad, b.grad)


def test_per_item_walk_is_bitwise_identical():
    """ops.gemm.set_per_item_walk (what the trainer selects under multi-rank data parallelism,
    so RCCL's kernels get CUs between work items) changes only which workgroup runs an item:
    input gradients, fused epilogues and split-K weight gradients are bitwise identical."""
    from orion_amd.ops import gemm as G
    g = torch.Generator(device=DEV).manual_seed(3)
    x, w = _rnd(g, 4096, 768), _rnd(g, 768, 3072)
    dy, xa = _rnd(g, 8192, 768), _rnd(g, 8192, 2304)
    outs = []
    for per_item in (False, True):
        G.set_per_item_walk(per_item)
        try:
            assert G.per_item_walk() is per_item
            outs.append((_C().gemm(x, w, True, 0, None, None)[0], G.wgrad(dy, xa)))
        finally:
            G.set_per_item_walk(False)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_per_item_walk_requests_are_reference_counted():
    """overlapping DDP trainers each request the per-item walk; releasing the older
    one must not switch the walk back while the newer one is alive."""
    from orion_amd.ops import gemm as G
    G.set_per_item_walk(False)
    r1 = G.request_per_item_walk()
    r2 = G.request_per_item_walk()
    try:
        assert G.per_item_walk() and (_C().gemm_diag(-1) & 64)
        r1()
        r1()  # idempotent
        assert G.per_item_walk() and (_C().gemm_diag(-1) & 64)
        r2()
        assert not G.per_item_walk() and not (_C().gemm_diag(-1) & 64)
    finally:
        r1()
        r2()
        G.set_per_item_walk(False)


@pytest.mark.parametrize("M,K,F_", [(300, 256, 128), (513, 512, 384), (2048, 128, 640), (4096, 768, 1408)])
def test_gemm_swiglu_epilogue(M, K, F_, gemm_cfg):
    """EPI_SWIGLU (Llama's gate_up projection): the W stream reads gate rows f and up rows F + f
    into one wave's tile, the epilogue writes gu in its natural (M, 2F) layout and h = silu(gate)
    up -- against the fp32 GEMM + SwiGLU and the bf16 GEMM + the swiglu pass, ragged M."""
    g = torch.Generator(device=DEV).manual_seed(M + K + F_)
    x = _rnd(g, M, K)
    w = _rnd(g, 2 * F_, K)
    gu, h = _C().gemm_swiglu(x, w)
    want = x.float() @ w.float().t()
    base = x @ w.t()
    within_bf16_budget("gu", gu, want, base)
    assert gu.shape == (M, 2 * F_) and h.shape == (M, F_)
    ga, ua = want.chunk(2, -1)
    within_bf16_budget("h", h, torch.nn.functional.silu(ga) * ua, _C().swiglu_fwd(base))


def _rope_ref(y, T, nrot, D, cos, sin, pos0):
    """Rotate-half RoPE of the first nrot columns (heads of D) of y (M, N): row m at position
    (m % T) + pos0 -- the fp32 reference of gemm16's EPI_ROPE."""
    M, N = y.shape
    y = y.clone()
    pos = torch.arange(M, device=y.device) % T + pos0
    c, s = cos[pos].unsqueeze(1), sin[pos].unsqueeze(1)      # (M, 1, D / 2)
    h = y[:, :nrot].view(M, nrot // D, D)
    x1, x2 = h[..., :D // 2].clone(), h[..., D // 2:].clone()
    h[..., :D // 2] = x1 * c - x2 * s
    h[..., D // 2:] = x2 * c + x1 * s
    return y


@pytest.mark.parametrize("B,T,K,Hq,Hkv,pos0", [(3, 100, 256, 2, 1, 5), (2, 256, 512, 4, 2, 0),
                                               (1, 1000, 128, 3, 3, 17)])
def test_gemm_rope_epilogue(B, T, K, Hq, Hkv, pos0, gemm_cfg):
    """EPI_ROPE (Llama's packed QKV projection): q | k heads rotated in the epilogue at
    position (row % T) + pos0, v heads stored as computed, ragged rows (B T not a multiple of
    256) -- against the fp32 GEMM + rotation and the bf16 GEMM + the rope pass."""
    from orion_amd.ops.reference import rope_tables
    D = 128
    g = torch.Generator(device=DEV).manual_seed(B * T + K)
    x = _rnd(g, B * T, K)
    w = _rnd(g, (Hq + 2 * Hkv) * D, K)
    cos, sin = (t.to(DEV).float().contiguous() for t in rope_tables(T + pos0 + 8, D, 10000.0))
    out = _C().gemm_rope(x, w, cos, sin, pos0, T, (Hq + Hkv) * D, D)
    want = _rope_ref(x.float() @ w.float().t(), T, (Hq + Hkv) * D, D, cos, sin, pos0)
    base = _rope_ref((x @ w.t()).float(), T, (Hq + Hkv) * D, D, cos, sin, pos0).bfloat16()
    within_bf16_budget("qkv", out, want, base)
    v0 = (Hq + Hkv) * D  # the v heads are the plain product
    within_bf16_budget("v", out[:, v0:], want[:, v0:], (x @ w.t())[:, v0:])
