"""Data-parallel reducer on CPU with gloo, world_size 2 (SURVEY.md §7.6 tests/dist):
bucketed, hook-driven all-reduce of the flat gradient arena must equal the
single-process gradient of the concatenated batch, and the full Trainer must
keep ranks bit-identical."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

from orion_amd.models.gpt2 import build_gpt2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, bucket_mb, accum, out, bf16_params=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    from orion_amd.train.engine import Trainer, OptimConfig
    model = build_gpt2("gpt2-tiny", block_size=32)
    kw = {}
    if bf16_params:  # the GPU layout: bf16 weights, unbound fp32 gradient arena (fold hooks)
        model = model.to(torch.bfloat16)
        kw = dict(arena_dtype=torch.bfloat16, grad_dtype=torch.float32)
    tr = Trainer(model, OptimConfig(learning_rate=1e-3, warmup_iters=0, decay_lr=False,
                                    grad_clip=0.0), bucket_mb=bucket_mb, **kw)
    g = torch.Generator().manual_seed(100)
    data = [(torch.randint(0, 50257, (4, 32), generator=g), torch.randint(0, 50257, (4, 32), generator=g))
            for _ in range(world * accum)]
    mine = [data[rank * accum + j] for j in range(accum)]
    # capture the reduced gradient before the optimizer by stepping with lr 0 first
    tr.opt.lr = 0.0
    tr.arena.zero_grad()
    for j, (x, y) in enumerate(mine):
        tr.reducer.set_sync(j == accum - 1)
        _, loss = model(x, y)
        (loss / accum).backward()
    tr.reducer.finish()
    grads = tr.arena.grads.clone()
    # then a few real steps; parameters must stay identical across ranks
    for _ in range(2):
        tr.step(mine)
    out.put((rank, grads.numpy(), tr.arena.params.float().numpy(), len(tr.reducer.buckets)))
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb,accum,bf16_params", [(0.5, 1, False), (100.0, 2, False),
                                                         (0.5, 2, True)])
def test_ddp_matches_single_process(bucket_mb, accum, bf16_params):
    world = 2
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, accum, q, bf16_params))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    (_, g0, p0, nb), (_, g1, p1, _) = res
    g0, g1, p0, p1 = (torch.from_numpy(a) for a in (g0, g1, p0, p1))
    assert nb >= (2 if bucket_mb < 1 else 1)
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)
    # single-process reference gradient over all micro-batches
    torch.manual_seed(0)
    from orion_amd.train.flat import FlatArena
    model = build_gpt2("gpt2-tiny", block_size=32)
    if bf16_params:
        model = model.to(torch.bfloat16)
        arena = FlatArena(model, dtype=torch.bfloat16, grad_dtype=torch.float32)
    else:
        arena = FlatArena(model, dtype=torch.float32)
    g = torch.Generator().manual_seed(100)
    data = [(torch.randint(0, 50257, (4, 32), generator=g), torch.randint(0, 50257, (4, 32), generator=g))
            for _ in range(world * accum)]
    arena.zero_grad()
    for x, y in data:
        _, loss = model(x, y)
        (loss / (world * accum)).backward()
    tol = dict(atol=1e-4, rtol=2e-2) if bf16_params else dict(atol=1e-6, rtol=1e-4)
    assert torch.allclose(g0, arena.grads, **tol)


def test_tied_parameter_gets_its_own_bucket():
    """GPT-2's wte (= LM head) completes only after the embedding backward: it must not hold
    back the layers laid out next to it, so it starts a bucket of its own."""
    from orion_amd.parallel.ddp import GradBucketReducer
    from orion_amd.train.flat import FlatArena
    port = _free_port()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        arena = FlatArena(build_gpt2("gpt2-tiny", block_size=32))
        red = GradBucketReducer(arena, bucket_mb=1000.0)  # one bucket but for the split
        names = [[s.name for s in sl] for _, _, sl in red.buckets]
        assert names[-1] == ["transformer.wte.weight"], names[-1]
        assert len(red.buckets) == 2
        covered = [b1 - b0 for b0, b1, _ in red.buckets]
        assert sum(covered) == arena.numel and red.buckets[0][0] == 0
        red.remove()
    finally:
        dist.destroy_process_group()


def test_collectives_launch_in_bucket_order():
    """RCCL matches collectives by issue order: a bucket whose gradients land early must
    wait until every bucket before it has launched (arrivals fed in reverse order)."""
    from orion_amd.parallel.ddp import GradBucketReducer
    from orion_amd.train.flat import FlatArena
    port = _free_port()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        model = build_gpt2("gpt2-tiny", block_size=32)
        arena = FlatArena(model, dtype=torch.float32)
        red = GradBucketReducer(arena, bucket_mb=0.05)
        nb = len(red.buckets)
        assert nb >= 4
        red.launch_log = []
        red.set_sync(True)
        # every parameter of the LAST bucket first, then backwards through the buckets
        for bi in reversed(range(nb)):
            for s in red.buckets[bi][2]:
                red._on_grad(s.param)
            if bi > 0:
                assert red.launch_log == [], "launched ahead of an unfinished earlier bucket"
        assert red.launch_log == list(range(nb))
        red.finish()
        # an interleaved order: bucket 1 completes before bucket 0, then 0 releases both
        red.launch_log = []
        for s in red.buckets[1][2]:
            red._on_grad(s.param)
        assert red.launch_log == []
        for s in red.buckets[0][2]:
            red._on_grad(s.param)
        assert red.launch_log == [0, 1]
        red.finish()  # stragglers (buckets 2..) still go out in order
        assert red.launch_log == list(range(nb))
        red.remove()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("zero1", [False, True])
def test_bench_spawns_its_own_ranks_on_cpu(zero1):
    """``python bench.py --gpus 2`` with no launcher around it starts both ranks itself (also
    with the ZeRO-1 optimizer: half the optimizer state per rank)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in
           ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--model", "gpt2-tiny",
                          "--device", "cpu", "--dist-backend", "gloo", "--seq-len", "64",
                          "--micro-batch", "2", "--steps", "2", "--warmup", "1"]
                         + (["--zero1"] if zero1 else []),
                         cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["steps"] == 2 and rec["warmup"] == 1
    # both rounded to 0.1 tok/s: at CPU rates (tens of tok/s) that alone is ~1e-3 relative
    assert abs(rec["per_gpu"] * 2 - rec["value"]) <= 0.1 * 2 + 1e-3 * rec["value"]
    assert rec["allreduce_busbw_gbps"] is not None
    # bucket timeline of the last step: every bucket ready before it completed
    ddp = rec["ddp_buckets"]
    assert ddp is not None and ddp["exposed_tail_ms"] >= 0
    assert all(done >= ready for _, _, ready, done in ddp["buckets"])
    assert rec["zero1"] == zero1


@pytest.mark.parametrize("model", ["gpt2-tiny", "llama-tiny"])
@pytest.mark.parametrize("zero1", ["off", "on"])
def test_bench_eight_ranks_on_cpu(model, zero1):
    """The driver's N = 8 job rehearsed on the CPU: ``bench.py --gpus 8``
    self-spawns 8 gloo ranks; every gradient bucket of the last step is launched in order and
    completes after it was ready, and after the timed steps every rank holds bit-identical
    weights and fp32 master (replicated: all-reduce; ZeRO-1: reduce-scatter + all-gather)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in
           ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--model", model,
                          "--device", "cpu", "--dist-backend", "gloo", "--seq-len", "64",
                          "--micro-batch", "2", "--steps", "2", "--warmup", "1", "--bucket-mb", "0.25",
                          "--zero1", zero1, "--check-replicas", "--no-busbw"],
                         cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["config"]["parallelism"] == "dp8"
    assert rec["zero1"] == (zero1 == "on")
    ddp = rec["ddp_buckets"]
    assert ddp is not None and len(ddp["buckets"]) > 2
    assert [b[0] for b in ddp["buckets"]] == list(range(len(ddp["buckets"])))
    assert all(done >= ready for _, _, ready, done in ddp["buckets"])
    assert ddp["exposed_tail_ms_max_over_ranks"] >= ddp["exposed_tail_ms"] >= 0
    assert rec["replicas"]["identical"], rec["replicas"]


def test_default_bucket_size_by_model_size():
    from orion_amd.parallel.ddp import default_bucket_mb
    assert default_bucket_mb(124_000_000) == 64.0
    assert default_bucket_mb(6_740_000_000) == 256.0


def _divergent_worker(rank, world, port, out):
    """Ranks see their gradients arrive in DIFFERENT orders and each rank has a different
    parameter that never gets a gradient (launched only by finish)."""
    import random
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from orion_amd.parallel.launch import init_process_group
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world))
    init_process_group("gloo")
    from orion_amd.parallel.ddp import GradBucketReducer
    from orion_amd.train.flat import FlatArena
    torch.manual_seed(0)
    arena = FlatArena(build_gpt2("gpt2-tiny", block_size=32), dtype=torch.float32)
    red = GradBucketReducer(arena, bucket_mb=0.05, timing=True, watchdog_s=60.0)
    red.launch_log = []
    logs = []
    for step in range(2):
        arena.grads.fill_(float(rank + 1))
        red.set_sync(True)
        slots = [s for _, _, sl in red.buckets for s in sl]
        order = list(range(len(slots)))
        random.Random(1000 * rank + step).shuffle(order)
        unused = slots[(7 * rank + step) % len(slots)].param
        for i in order:
            if slots[i].param is not unused:
                red._on_grad(slots[i].param)
        red.finish()
        logs.append(list(red.launch_log))
        red.launch_log = []
    rep = red.timing_report()
    out.put((rank, logs, arena.grads.clone().numpy(), len(red.buckets), rep is not None))
    red.remove()
    dist.destroy_process_group()


def test_divergent_arrival_orders_and_unused_params_four_ranks():
    """SURVEY §7.6 tests/dist: 4 gloo ranks whose gradient arrival orders differ and each
    with a rank-dependent unused parameter: no hang, every rank issues the collectives in the
    same (bucket) order, and the reduced gradient is the average over ranks."""
    world = 4
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_divergent_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    nb = res[0][3]
    assert nb >= 4
    for rank, logs, grads, _, timed in res:
        assert logs == [list(range(nb))] * 2, (rank, logs)
        assert timed
        assert torch.allclose(torch.from_numpy(grads), torch.full_like(torch.from_numpy(grads), 2.5))


# ------------------------------------------------------------- split tied bucket (VERDICT r5 #5a)
def _tied_worker(rank, world, port, zero1, out):
    """One rank: GPT-2-tiny's arena (fp32 gradients) with a CPU-constructed sink on the tied
    wte (the GPU path's sinks are CUDA-only), gradients written the way the GPU backward
    writes them -- LM-head part through the sink first, every other parameter, then the
    embedding's part as the tied parameter's last use -- reduced fp32-joint and split."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from orion_amd.ops.grad_sink import GradSink
    from orion_amd.parallel.ddp import GradBucketReducer, ShardedGradReducer, zero1_pad_names
    from orion_amd.train.flat import FlatArena
    torch.manual_seed(0)
    model = build_gpt2("gpt2-tiny", block_size=32)
    res = {}
    for split in (False, True):
        kw = {}
        if zero1:
            names, pad_to = zero1_pad_names(model, 0.05, torch.float32, world)
            kw = dict(pad_after=names, pad_to=pad_to)
        arena = FlatArena(model, dtype=torch.float32, grad_dtype=torch.float32, **kw)
        wte = model.transformer.wte.weight
        slot = next(s_ for s_ in arena.slots if s_.param is wte)
        sink = GradSink(wte, arena.grad_view(slot).view_as(wte), arena.grad_listeners, expect=2)
        wte._orion_sink = sink
        cls = ShardedGradReducer if zero1 else GradBucketReducer
        red = cls(arena, bucket_mb=0.05, timing=True, watchdog_s=60.0, tied_bf16=split)
        assert len(red.tails) == (1 if split else 0)
        red.launch_log = []
        g = torch.Generator().manual_seed(1000 + rank)
        lm = torch.randn(wte.shape, generator=g)
        emb = torch.zeros(wte.shape)
        rows = torch.randint(0, wte.shape[0], (64,), generator=g)
        emb.index_add_(0, rows, torch.randn(64, wte.shape[1], generator=g))
        others = {s_.name: torch.randn(s_.numel, generator=g) for s_ in arena.slots if s_.param is not wte}
        arena.zero_grad()
        red.set_sync(True)
        assert sink.take() is False
        sink.view.copy_(lm)
        sink.notify()                     # the LM head, first kernel of the backward
        for s_ in arena.slots:
            if s_.param is not wte:
                arena.grad_view(s_).copy_(others[s_.name])
                red._on_grad(s_.param)
                time.sleep(0.002)         # a backward's worth of spacing for the timeline
        view, acc = sink.last_use_target()
        assert acc is (not split) and (view is not sink.view) is split
        if acc:
            view.add_(emb)
        else:
            view.copy_(emb)
        sink.notify(last=True)            # the embedding, last kernel of the backward
        red.finish()
        rep = red.timing_report()
        if zero1:
            full = red.gather_full(red.grad_shard)
        else:
            full = arena.grads.clone()
        res[split] = (full[slot.offset:slot.offset + slot.numel].numpy().copy(),
                      full.numpy().copy(), rep, list(red.launch_log), slot.offset, slot.numel)
        red.remove()
        del wte._orion_sink
    out.put((rank, res))
    dist.destroy_process_group()


@pytest.mark.parametrize("zero1", [False, True])
def test_tied_bucket_split_bf16_tail_eight_ranks(zero1):
    """8 gloo ranks: with ``tied_bf16`` the tied bucket launches right after the LM head's
    write (first, under the rest of the 'backward'), the embedding's part follows as a bf16
    tail after every bucket, and the result equals the fp32 joint reduction within the bf16
    budget of the tail alone (the other parameters bit-identical); the tail's wire bytes
    are half the tied bucket's fp32 bytes."""
    world = 8
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tied_worker, args=(r, world, port, zero1, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    joint_w, joint_all, rep0, log0, off, n = got[0][False]
    split_w, split_all, rep1, log1, _, _ = got[0][True]
    joint_w, joint_all, split_w, split_all = map(torch.from_numpy, (joint_w, joint_all, split_w, split_all))
    for r in range(world):  # replicas agree
        assert torch.equal(torch.from_numpy(got[r][True][1]), split_all)
    # untouched parameters: identical; the tied one within bf16 rounding of the embedding part
    mask = torch.ones_like(joint_all, dtype=torch.bool)
    mask[off:off + n] = False
    assert torch.equal(joint_all[mask], split_all[mask])
    err = (split_w - joint_w).abs().max().item()
    assert 0 < err <= 2e-2 * joint_w.abs().max().item(), err
    # launch order: joint -- bucket index order, the tied bucket (the table's arena position
    # is last) held until the embedding; split -- the tied bucket FIRST (right after the LM
    # head's write), the others in index order, the bf16 tail after everything
    tied_b = rep1["tied_tails"][0][0]
    assert log0 == list(range(len(log0))) and log0[-1] == tied_b
    assert log1 == [tied_b] + log0[:-1] + [("tail", tied_b)], log1
    fp32_mb = rep0["buckets"][tied_b][1]
    assert abs(rep1["tied_tails"][0][1] - fp32_mb / 2) < 0.02, (rep1["tied_tails"], fp32_mb)
    # the timeline: split -- the tied bucket was ready before every other bucket; joint -- after
    others = [r[2] for r in rep1["buckets"] if r[0] != tied_b]
    assert rep1["buckets"][tied_b][2] <= min(others)
    assert rep0["buckets"][tied_b][2] >= max(r[2] for r in rep0["buckets"] if r[0] != tied_b)
