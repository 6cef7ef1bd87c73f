#!/usr/bin/env python3
"""Headline benchmark: GPT-2-124M bf16 training throughput (seq 1024) on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
launched by ``torch.distributed.run`` with one rank per GPU (RCCL over xGMI).
W untimed warm-up optimizer steps, then exactly K timed optimizer steps
bracketed by barrier + device synchronize; the elapsed time is the MAX over
ranks; rank 0 prints one JSON line whose ``value`` is the whole-job token
throughput (tokens/s summed over all GPUs); ``per_gpu`` is value / n_gpus, the
tokens/sec/GPU of BASELINE.json's metric, and ``vs_baseline`` compares that per-GPU
rate with the baseline's per-GPU figure.

Every timed step is a complete training step: ``grad_accum`` micro-batches of
forward + backward through the full 12-layer model, gradient all-reduce (N>1)
and the fused AdamW update with global-norm clipping.  Data is synthetic
(random token ids, fixed pool resident on the GPU), weights random-init.

``--gpus N`` without ``WORLD_SIZE`` in the environment starts the N ranks itself
(``orion_amd/parallel/launch.py``: one process per GPU, spawned before anything
touches HIP), so ``python bench.py --gpus 8`` and the driver's
``torch.distributed.run ... bench.py --gpus 8`` run the same RCCL job.  For N>1 the
JSON also carries the RCCL all-reduce bus bandwidth of one gradient-arena-sized
buffer, measured after the timed region.

``--impl torch`` runs the same model on stock PyTorch ops (SDPA, F.layer_norm,
fp32 master params under bf16 autocast, fused torch AdamW) -- the nanoGPT
recipe minus torch.compile -- for a same-box comparison.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TOK_S_PER_GPU = 1.07e5  # nanoGPT GPT-2-124M, 8xA100-40GB, derived


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--seq-len", type=int, default=1024)
    # 64 x 1024 tokens per GPU per step: at dp8 that is 524,288 tokens per optimizer step,
    # the same global batch as nanoGPT's GPT-2-124M recipe (12 x 1024 x 40 = 491,520).
    ap.add_argument("--micro-batch", type=int, default=None,
                    help="sequences per micro-batch (default: 64 for GPT-2 presets; 16,384 tokens "
                         "per micro-batch for Llama presets, i.e. 4 at seq 4096)")
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--impl", choices=["native", "torch"], default="native")
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="DDP gradient bucket size (default: 64 MB, 256 MB from 1B parameters up)")
    ap.add_argument("--no-tuned-gemms", action="store_true",
                    help="do not load the committed TunableOp GEMM table (orion_amd/tuning/)")
    ap.add_argument("--gemm-table", default=None, help="TunableOp table to load instead of the committed one")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI, the real run) or gloo (rehearsing N>1 on one GPU)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: plumbing rehearsal (reference ops, gloo) -- not a measurement")
    ap.add_argument("--no-busbw", action="store_true", help="skip the post-run all-reduce probe")
    ap.add_argument("--grad-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="gradient arena dtype (fp32: accumulation and all-reduce in fp32)")
    ap.add_argument("--hip-graph", action="store_true",
                    help="capture the whole training step in a HIP graph (single GPU)")
    ap.add_argument("--zero1", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                    help="ZeRO-1: reduce-scatter gradients, AdamW on this rank's 1/N shard of the "
                         "fp32 master / Adam state, all-gather the bf16 weights (overlapped with the "
                         "next forward).  auto (default): on for models of >= 1B parameters at "
                         "N > 1 GPUs; a bare --zero1 = on (with one GPU: a world-1 rehearsal of "
                         "the sharded path)")
    ap.add_argument("--tied-bf16", action="store_true",
                    help="N > 1: reduce GPT-2's tied wte bucket split -- the LM head's part in fp32 under "
                         "the backward, the embedding's part in bf16 after it (parallel/ddp.py)")
    ap.add_argument("--per-item-walk", action="store_true",
                    help="force gemm16's one-workgroup-per-item walk (what multi-rank training selects "
                         "so RCCL kernels get CUs) also at N = 1: separates that walk's cost from the "
                         "communication cost on a scaling curve")
    ap.add_argument("--check-replicas", action="store_true",
                    help="after the timed region, compare a checksum of every rank's full weights "
                         "(and fp32 master) across ranks; reported as replicas_identical")
    return ap.parse_args()


def _replica_checksums(trainer, dev):
    """(bf16 compute weights, fp32 master) checksums of this rank's FULL model state: float64
    sums of the values and of the values times a position ramp, so a permutation differs."""
    if trainer.zero1:
        trainer.reducer.wait_params()
        master = trainer.full_master()
    else:
        master = trainer.opt.master
    out = []
    for t in (trainer.arena.params, master):
        v = t.detach().double()
        ramp = torch.arange(v.numel(), device=v.device, dtype=torch.float64) / max(1, v.numel())
        out += [float(v.sum()), float((v * ramp).sum())]
    return torch.tensor(out, device=dev, dtype=torch.float64)


def _per_item_walk() -> bool:
    from orion_amd.ops.gemm import per_item_walk
    return per_item_walk()


def main():
    args = parse()
    from orion_amd.parallel import launch
    if args.gpus > 1 and not launch.in_launched_job():
        # spawn the ranks before this process touches the GPU; exit with the job's status
        sys.exit(launch.spawn_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    world, rank, local_rank = launch.check_world(args.gpus)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if args.device == "cpu":
        if args.dist_backend == "nccl":
            args.dist_backend = "gloo"
        dev = torch.device("cpu")
    else:
        dev = launch.device_for(local_rank, local_world, args.dist_backend)
        torch.cuda.set_device(dev)
    rccl_log = None
    if world == 1 and args.zero1 == "on":
        # a one-rank process group so the sharded optimizer path runs as it would at N > 1
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(launch.free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        launch.init_process_group(args.dist_backend if dev.type == "cuda" else "gloo",
                                  dev if dev.type == "cuda" and args.dist_backend == "nccl" else None)
    if world > 1:
        if args.dist_backend == "nccl":
            # RCCL's topology / channel INFO log of this rank goes to a file, summarised below
            rccl_log = launch.rccl_debug_env(
                os.environ.get("ORION_BENCH_LOGDIR", os.path.join(ROOT, "gpurun_out", "bench_logs")),
                rank)
        launch.init_process_group(args.dist_backend, dev if args.dist_backend == "nccl" else None)
    n_tuned = 0
    # TunableOp's table is not applied under HIP-graph capture (solutions chosen by index
    # went wrong on replay in testing); graph runs use hipBLASLt's default heuristics
    if dev.type == "cuda" and not args.no_tuned_gemms and not args.hip_graph:
        from orion_amd.tuning import use_tuned_gemms
        n_tuned = use_tuned_gemms(args.gemm_table, verbose=(rank == 0))
    torch.manual_seed(1337 + rank)

    from orion_amd import ops
    from orion_amd.models import build_model, GPT2_PRESETS
    from orion_amd.train.engine import Trainer, OptimConfig

    if args.impl == "torch":
        ops.set_backend("torch")
    elif dev.type == "cuda":
        ops.load_ext(required=True)

    is_gpt2 = args.model in GPT2_PRESETS
    ctx_kw = dict(block_size=max(1024, args.seq_len)) if is_gpt2 else dict(max_seq_len=args.seq_len)
    with torch.device(dev):  # parameters are created (and initialised) on the GPU: 7B shapes included
        model = build_model(args.model, **ctx_kw)
    n_params = model.num_params()
    if args.micro_batch is None:
        args.micro_batch = 64 if is_gpt2 else max(1, 16384 // args.seq_len)
    B, T, A = args.micro_batch, args.seq_len, args.grad_accum
    # token ids below GPT-2's real vocabulary (50257); the padded embedding rows stay unused
    vocab = 50257 if is_gpt2 else model.config.vocab_size
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    pool = [(torch.randint(0, vocab, (B, T), device=dev, generator=g),
             torch.randint(0, vocab, (B, T), device=dev, generator=g)) for _ in range(4)]

    ocfg = OptimConfig(warmup_iters=10, lr_decay_iters=10000)
    if args.impl == "native":
        trainer = Trainer(model, ocfg, bucket_mb=args.bucket_mb, graph=args.hip_graph and world == 1,
                          grad_dtype=torch.float32 if args.grad_dtype == "fp32" else torch.bfloat16,
                          ddp_timing=False, zero1={"auto": None, "on": True, "off": False}[args.zero1],
                          tied_bf16=args.tied_bf16)
        step_fn = lambda i: trainer.step([pool[(i * A + j) % 4] for j in range(A)])
        if args.per_item_walk and dev.type == "cuda":
            from orion_amd.ops.gemm import set_per_item_walk
            set_per_item_walk(True)
    else:
        ddp_model = model
        if world > 1:
            ddp_model = torch.nn.parallel.DistributedDataParallel(
                model, device_ids=[dev.index] if dev.type == "cuda" else None,
                                                                  bucket_cap_mb=args.bucket_mb or 64.0)
        opt = torch.optim.AdamW(model.parameters(), lr=ocfg.learning_rate, betas=(0.9, 0.95),
                                weight_decay=0.1, fused=True)

        def step_fn(i):
            opt.zero_grad(set_to_none=True)
            tot = 0.0
            for j in range(A):
                x, y = pool[(i * A + j) % 4]
                ctx = ddp_model.no_sync() if (world > 1 and j < A - 1) else _null()
                with ctx, torch.autocast(dev.type, dtype=torch.bfloat16):
                    _, loss = ddp_model(x, y)
                (loss / A).backward()
                tot = tot + loss.detach()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
            return tot / A

    def barrier():
        if world > 1:
            dist.barrier()

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    loss = None
    trace = os.environ.get("ORION_BENCH_TRACE_LOSS") == "1"  # debugging: per-step loss (syncs)
    for i in range(args.warmup):
        loss = step_fn(i)
        if trace:
            print(f"warmup {i} loss {float(loss):.4f}", file=sys.stderr, flush=True)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step_fn(args.warmup + i)
        if trace:
            print(f"step {i} loss {float(loss):.4f}", file=sys.stderr, flush=True)
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    final_loss = float(loss)
    busbw = ddp = rccl = replicas = None
    if world > 1 and args.impl == "native" and trainer.reducer is not None:
        # the bucket timeline comes from ONE extra step after the timed region: the timed steps
        # run without the per-bucket events and the side-stream waits they need
        trainer.reducer.timing = True
        step_fn(args.warmup + args.steps)
        sync()
    if args.check_replicas and args.impl == "native":
        mine = _replica_checksums(trainer, dev)
        if world > 1:
            allc = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(allc, mine)
        else:
            allc = [mine]
        replicas = {"identical": all(torch.equal(c, allc[0]) for c in allc),
                    "checksums": [round(float(x), 6) for x in allc[0].tolist()]}
    if world > 1 and args.impl == "native":
        # bucket timeline of the extra step: launch -> complete per bucket, exposed tail
        ddp = trainer.reducer.timing_report()
        if ddp is not None:
            t = torch.tensor([ddp["exposed_tail_ms"], ddp["comm_ms"]], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ddp["exposed_tail_ms_max_over_ranks"] = round(float(t[0]), 3)
            ddp["comm_ms_max_over_ranks"] = round(float(t[1]), 3)
        if not args.no_busbw:
            from orion_amd.parallel.busbw import allreduce_busbw
            busbw = allreduce_busbw(trainer.arena.grads, iters=5)
        if rccl_log is not None:
            from orion_amd.parallel.busbw import rccl_summary
            rccl = rccl_summary(rccl_log)

    tokens = world * B * T * A * args.steps
    tok_s = tokens / elapsed
    flops_tok = model.flops_per_token(T)
    mfu = tok_s / world * flops_tok / 2.5e15
    headline = args.model == "gpt2" and T == 1024 and dev.type == "cuda"
    if rank == 0:
        out = {
            # BASELINE.json's metric is tokens/sec/GPU at 1/2/4/8 GPUs: ``value`` is the whole
            # job's rate (the driver's contract), ``per_gpu`` = value / n_gpus is that metric
            "metric": ("tokens/sec (whole job; per_gpu = tokens/sec/GPU), GPT-2-124M bf16 seq=1024, "
                       "at 1/2/4/8 MI355X" if headline else
                       f"tokens/sec (whole job), {args.model} bf16 seq={T} on {dev.type} (secondary config)"),
            "value": round(tok_s, 1),
            "unit": "tokens/s (whole job, summed over n_gpus)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(tok_s / world / BASELINE_TOK_S_PER_GPU, 3) if headline else None,
            "baseline": "1.07e5 tokens/s per GPU (BASELINE.md, nanoGPT 8xA100 derived); "
                        "vs_baseline = per_gpu / 1.07e5",
            "per_gpu": round(tok_s / world, 1),
            "dtype": "bf16",
            "data": "synthetic (random token ids), random-init weights",
            "impl": args.impl,
            "tuned_gemm_entries": n_tuned,
            "hip_graph": bool(args.impl == "native" and trainer.graph_enabled),
            "grad_dtype": str(trainer.arena.grads.dtype).replace("torch.", "") if args.impl == "native" else None,
            "mfu_vs_2.5PF_dense_bf16": round(mfu, 4),
            "loss": round(final_loss, 4),
            "max_mem_gb": (round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)
                           if dev.type == "cuda" else None),
            "dist_backend": args.dist_backend if world > 1 or args.zero1 == "on" else None,
            "zero1": bool(args.impl == "native" and trainer.zero1),
            "zero1_mode": args.zero1,
            "tied_bf16": bool(args.tied_bf16 and args.impl == "native" and world > 1
                              and trainer.reducer is not None and bool(trainer.reducer.tails)),
            "gemm16_walk": ("per_item" if args.impl == "native" and dev.type == "cuda" and _per_item_walk()
                            else "persistent"),
            "optimizer_state_gb_per_rank": (round(3 * 4 * trainer.opt.master.numel() / 2**30, 2)
                                            if args.impl == "native" else None),
            "allreduce_busbw_gbps": busbw,
            "ddp_buckets": ddp,
            "rccl": rccl,
            "replicas": replicas,
            "config": {"model": f"{args.model} ({n_params / 1e6:.1f}M params)",
                       "global_batch": B * A * world, "micro_batch": B, "grad_accum": A,
                       "seq_len": T, "tokens_per_step": B * T * A * world,
                       "parallelism": f"dp{world}"},
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


if __name__ == "__main__":
    main()
