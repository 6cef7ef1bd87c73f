"""Trainer on CPU (BASELINE.json config 1: GPT-2 tiny, 10 steps, synthetic tokens)."""
import math

import torch

from orion_amd.models.gpt2 import build_gpt2
from orion_amd.ops import reference as ref
from orion_amd.train.engine import OptimConfig, Trainer, cosine_lr
from orion_amd.train.flat import ALIGN, FlatArena


def test_gpt2_tiny_trains_10_steps():
    torch.manual_seed(0)
    model = build_gpt2("gpt2-tiny")
    tr = Trainer(model, OptimConfig(learning_rate=3e-3, warmup_iters=2, lr_decay_iters=10, min_lr=3e-4))
    x = torch.randint(0, 256, (4, 64))
    y = torch.roll(x, -1, dims=1)
    losses = [float(tr.step([(x, y)])) for _ in range(10)]
    assert losses[-1] < losses[0] - 0.5, losses


def test_arena_layout_and_views():
    model = build_gpt2("gpt2-tiny")
    arena = FlatArena(model, dtype=torch.float32)
    names = [s.name for s in arena.slots]
    assert names[-1] == "transformer.wte.weight"  # tied with lm_head, counted once, last
    for s in arena.slots:
        assert s.offset % ALIGN == 0
        assert s.param.data_ptr() == arena.params[s.offset:].data_ptr()
        assert s.param.grad.data_ptr() == arena.grads[s.offset:].data_ptr()
        assert s.decay == (s.param.dim() >= 2)


def test_flat_adamw_reference_matches_torch():
    torch.manual_seed(0)
    model = build_gpt2("gpt2-tiny")
    ref_model = build_gpt2("gpt2-tiny")
    ref_model.load_state_dict(model.state_dict())
    tr = Trainer(model, OptimConfig(learning_rate=1e-3, warmup_iters=0, decay_lr=False, grad_clip=0.0))
    # eps well above the ~1e-10 rounding noise of gradients that are zero in exact
    # arithmetic (the key bias: softmax is invariant to it), which Adam would otherwise
    # amplify to +-lr differently in any two implementations
    tr.opt.eps = 1e-6
    decay = [p for n, p in ref_model.named_parameters() if p.dim() >= 2]
    nodecay = [p for n, p in ref_model.named_parameters() if p.dim() < 2]
    opt = torch.optim.AdamW([{"params": decay, "weight_decay": 0.1}, {"params": nodecay, "weight_decay": 0.0}],
                            lr=1e-3, betas=(0.9, 0.95), eps=1e-6)
    x = torch.randint(0, 256, (2, 32))
    y = torch.randint(0, 256, (2, 32))
    for _ in range(3):
        tr.step([(x, y)])
        opt.zero_grad()
        _, loss = ref_model(x, y)
        loss.backward()
        opt.step()
    got = dict(model.named_parameters())
    for n, p in ref_model.named_parameters():
        assert torch.allclose(got[n], p, atol=1e-5), n


def test_cosine_lr():
    cfg = OptimConfig(learning_rate=1.0, warmup_iters=10, lr_decay_iters=110, min_lr=0.1)
    assert math.isclose(cosine_lr(0, cfg), 1 / 11)
    assert math.isclose(cosine_lr(60, cfg), 0.55)
    assert cosine_lr(200, cfg) == 0.1


def test_reference_attention_matches_sdpa():
    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 16, 4, 8) for _ in range(3))
    o = ref.attention(q, k, v, causal=True)
    o2 = torch.nn.functional.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2),
                                                          v.transpose(1, 2), is_causal=True).transpose(1, 2)
    assert torch.allclose(o, o2, atol=1e-5)


def test_reference_gqa_and_rope_inverse():
    torch.manual_seed(0)
    q = torch.randn(1, 8, 4, 16)
    k = torch.randn(1, 8, 2, 16)
    o = ref.attention(q, k, k, causal=True)
    assert o.shape == q.shape
    cos, sin = ref.rope_tables(8, 16)
    r = ref.rope(q, cos, sin)
    back = ref.rope(r, cos, -sin)
    assert torch.allclose(back, q, atol=1e-5)


def test_fp32_grad_arena_for_bf16_params_folds_accumulate_grad():
    """bf16 weights with an fp32 gradient arena: p.grad stays unbound, AccumulateGrad results
    are folded into the fp32 slices, so A micro-batches sum in fp32 (here on the CPU, where
    every gradient takes the AccumulateGrad path)."""
    torch.manual_seed(0)
    m1 = build_gpt2("gpt2-tiny", block_size=32).to(torch.bfloat16)
    m2 = build_gpt2("gpt2-tiny", block_size=32).to(torch.bfloat16)
    m2.load_state_dict(m1.state_dict())
    arena = FlatArena(m1, dtype=torch.bfloat16, grad_dtype=torch.float32)
    assert not arena.bound and arena.grads.dtype == torch.float32
    batches = [(torch.randint(0, 50257, (2, 32)), torch.randint(0, 50257, (2, 32))) for _ in range(6)]
    arena.zero_grad()
    ref_acc = {n: torch.zeros(p.shape) for n, p in m2.named_parameters()}
    for x, y in batches:
        _, loss = m1(x, y)
        (loss / len(batches)).backward()
        m2.zero_grad(set_to_none=True)
        _, l2 = m2(x, y)
        (l2 / len(batches)).backward()
        for n, p in m2.named_parameters():
            ref_acc[n] += p.grad.float()
    for s in arena.slots:
        assert s.param.grad is None, s.name
        got = arena.grads[s.offset:s.offset + s.numel].view(s.param.shape)
        assert torch.allclose(got, ref_acc[s.name], atol=1e-6, rtol=1e-5), s.name


def test_embed_layer_norm_cpu_path_matches_unfused():
    """ops.embed_layer_norm on the CPU (the reference path the GPU kernel is tested against):
    x = wte[idx] + wpe[:T], h = LayerNorm(x), gradients through both outputs."""
    import torch
    from orion_amd import ops
    torch.manual_seed(0)
    V, Tm, C, B, T = 50, 16, 32, 2, 12
    wte, wpe = torch.randn(V, C, requires_grad=True), torch.randn(Tm, C, requires_grad=True)
    w, b = torch.randn(C, requires_grad=True), torch.randn(C, requires_grad=True)
    idx = torch.randint(0, V, (B, T))
    x, h = ops.embed_layer_norm(idx, wte, wpe, w, b)
    (x.sum() + (h * h).sum()).backward()
    g = [t.grad.clone() for t in (wte, wpe, w, b)]
    for t in (wte, wpe, w, b):
        t.grad = None
    x2 = wte[idx] + wpe[:T]
    h2 = torch.nn.functional.layer_norm(x2, (C,), w, b, 1e-5)
    (x2.sum() + (h2 * h2).sum()).backward()
    assert torch.allclose(x, x2) and torch.allclose(h, h2, atol=1e-5)
    for a, t in zip(g, (wte, wpe, w, b)):
        assert torch.allclose(a, t.grad, atol=1e-4)
    assert float(g[1][T:].abs().max()) == 0.0


def test_gemms_forced_in_tree_record_library_fallbacks():
    """Inside ``hip_gemms()`` (HIP-graph capture) a GEMM that is not eligible for the in-tree
    kernels falls back to a library call; that fallback is recorded so the trainer can keep the
    step eager instead of capturing a library GEMM (ops/gemm.py)."""
    from orion_amd.ops import gemm
    gemm.forced_fallbacks(clear=True)
    x, w = torch.randn(4, 8), torch.randn(6, 8)
    gemm.linear_fwd(x, w)  # outside the block: nothing recorded
    assert gemm.forced_fallbacks() == []
    with gemm.hip_gemms():
        y = gemm.linear_fwd(x, w)
        gemm.linear_dgrad(torch.randn(4, 6), w)
    assert torch.allclose(y, x @ w.t())
    fb = gemm.forced_fallbacks(clear=True)
    assert [k for k, _ in fb] == ["linear_fwd", "linear_dgrad"] and fb[0][1] == ((4, 8), (6, 8))
    assert gemm.forced_fallbacks() == []
