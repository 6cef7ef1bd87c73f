#!/usr/bin/env python3
"""nanoGPT-compatible training script on the orion_amd MI355X engine.

    python train.py [config.py|config.yaml|config.json] [--key=value ...]
    torchrun --standalone --nproc-per-node 8 train.py config/train_gpt2.py

Configuration keys and defaults follow nanoGPT's ``train.py`` (out_dir,
eval_interval, log_interval, eval_iters, eval_only, always_save_checkpoint,
init_from, dataset, gradient_accumulation_steps, batch_size, block_size,
n_layer, n_head, n_embd, dropout, bias, learning_rate, max_iters,
weight_decay, beta1, beta2, grad_clip, decay_lr, warmup_iters,
lr_decay_iters, min_lr) plus ``model`` (a preset: gpt2, gpt2-medium,
llama2-7b, llama-tiny ...) and ``bucket_mb``
(0 = by model size, ``parallel.ddp.default_bucket_mb``).  Python config files are read
for literal ``key = value`` assignments only (parsed with ``ast``; nothing is
executed).  ``dataset`` names ``data/<dataset>/{train,val}.bin`` (uint16 token
shards); if absent, synthetic tokens are used.

Under an ``orion`` worker (``METAOPT_RESULTS_PATH`` set) the final validation
loss is reported as the trial objective, so hyper-parameters of this script
can be searched with e.g. ``--learning_rate~'loguniform(1e-4, 1e-3)'``.
"""
from __future__ import annotations

import ast
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

DEFAULTS = dict(
    out_dir="out", eval_interval=2000, log_interval=1, eval_iters=200, eval_only=False,
    always_save_checkpoint=True, init_from="scratch", dataset="openwebtext",
    gradient_accumulation_steps=5 * 8, batch_size=12, block_size=1024,
    model="gpt2", n_layer=12, n_head=12, n_embd=768, dropout=0.0, bias=True,
    learning_rate=6e-4, max_iters=600000, weight_decay=1e-1, beta1=0.9, beta2=0.95,
    grad_clip=1.0, decay_lr=True, warmup_iters=2000, lr_decay_iters=600000, min_lr=6e-5,
    backend="nccl", device="cuda", dtype="bfloat16", seed=1337, bucket_mb=0.0,
    # zero1: shard the fp32 master / Adam state over the data-parallel ranks (ZeRO-1:
    # reduce-scatter gradients, all-gather weights; parallel/ddp.py ShardedGradReducer)
    zero1=None,  # None: auto (sharded optimizer from 1B parameters at more than one rank)
    data_root="data",
    # tracing: profile_steps > 0 records that many steps, starting at
    # profile_start, with torch.profiler and writes a Chrome trace to out_dir
    profile_start=10, profile_steps=0, peak_flops=2.5e15,
)


def _literal_assignments(path):
    tree = ast.parse(open(path).read(), path)
    out = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            try:
                out[node.targets[0].id] = ast.literal_eval(node.value)
            except ValueError:
                pass  # non-literal expression (nanoGPT configs are literal in practice)
    return out


def parse_config(argv):
    cfg = dict(DEFAULTS)
    for arg in argv:
        if not arg.startswith("--"):
            if arg.endswith(".py"):
                cfg.update(_literal_assignments(arg))
            elif arg.endswith((".yaml", ".yml")):
                import yaml
                cfg.update(yaml.safe_load(open(arg)) or {})
            elif arg.endswith(".json"):
                cfg.update(json.load(open(arg)))
            else:
                raise ValueError(f"unknown config file type: {arg}")
            continue
        key, _, val = arg[2:].partition("=")
        if key not in cfg:
            raise ValueError(f"Unknown config key: {key}")
        try:
            v = ast.literal_eval(val)
        except (ValueError, SyntaxError):
            v = val
        if isinstance(cfg[key], float) and isinstance(v, int):
            v = float(v)
        cfg[key] = v
    return cfg


def main(argv=None):
    cfg = parse_config(sys.argv[1:] if argv is None else argv)
    from orion_amd import ops
    from orion_amd.models import build_model
    from orion_amd.train.ckpt import build_model_from_checkpoint, load_checkpoint, restore_trainer, save_checkpoint
    from orion_amd.train.data import get_batch_source
    from orion_amd.train.engine import OptimConfig, Trainer

    ddp = int(os.environ.get("RANK", -1)) != -1
    rank, local_rank, world = 0, 0, 1
    if ddp:
        rank, local_rank, world = (int(os.environ[k]) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"))
        if cfg["device"].startswith("cuda"):
            torch.cuda.set_device(local_rank)
            from orion_amd.parallel.launch import init_process_group
            init_process_group(cfg["backend"], torch.device("cuda", local_rank))
        else:
            from orion_amd.parallel.launch import init_process_group
            init_process_group("gloo")
    master = rank == 0
    device = torch.device(cfg["device"] if not cfg["device"].startswith("cuda") else f"cuda:{local_rank}")
    if device.type == "cuda":
        from orion_amd.tuning import use_tuned_gemms
        use_tuned_gemms()
        ops.load_ext(required=True)
    torch.manual_seed(cfg["seed"] + rank)
    tokens_per_iter = cfg["gradient_accumulation_steps"] * world * cfg["batch_size"] * cfg["block_size"]
    if master:
        os.makedirs(cfg["out_dir"], exist_ok=True)
        print(f"tokens per iteration will be: {tokens_per_iter:,}")

    ckpt = None
    if cfg["init_from"] == "resume":
        ckpt = load_checkpoint(os.path.join(cfg["out_dir"], "ckpt.pt"))
        model = build_model_from_checkpoint(ckpt)
    else:
        name = cfg["model"]
        over = {}
        if name.startswith("gpt2"):
            over = dict(n_layer=cfg["n_layer"], n_head=cfg["n_head"], n_embd=cfg["n_embd"],
                        block_size=cfg["block_size"], dropout=cfg["dropout"], bias=cfg["bias"])
            if name != "gpt2":
                over = dict(block_size=cfg["block_size"], dropout=cfg["dropout"])
        else:
            over = dict(max_seq_len=cfg["block_size"])
        model = build_model(name, **over)
    model.to(device)
    ocfg = OptimConfig(learning_rate=cfg["learning_rate"], weight_decay=cfg["weight_decay"],
                       beta1=cfg["beta1"], beta2=cfg["beta2"], grad_clip=cfg["grad_clip"],
                       warmup_iters=cfg["warmup_iters"], lr_decay_iters=cfg["lr_decay_iters"],
                       min_lr=cfg["min_lr"], decay_lr=cfg["decay_lr"])
    trainer = Trainer(model, ocfg, ddp=ddp and world > 1, bucket_mb=cfg["bucket_mb"],
                      zero1=None if cfg["zero1"] is None else bool(cfg["zero1"]) and ddp)
    best_val = 1e9
    if ckpt is not None:
        restore_trainer(trainer, ckpt)
        best_val = ckpt.get("best_val_loss") or 1e9
        del ckpt

    vocab = model.config.vocab_size
    data_dir = os.path.join(cfg["data_root"], cfg["dataset"]) if cfg["dataset"] else None
    B, T, A = cfg["batch_size"], cfg["block_size"], cfg["gradient_accumulation_steps"]
    if ddp:
        assert A % world == 0, "gradient_accumulation_steps must be divisible by the world size"
        A //= world
    train_src = get_batch_source(data_dir, "train", B, T, device, min(vocab, 50257), seed=cfg["seed"] + rank)
    val_src = get_batch_source(data_dir, "val", B, T, device, min(vocab, 50257), seed=cfg["seed"] + 7919 + rank)

    @torch.no_grad()
    def estimate_loss():
        out = {}
        model.eval()
        for split, src in (("train", train_src), ("val", val_src)):
            tot = torch.zeros((), device=device)
            for _ in range(cfg["eval_iters"]):
                x, y = src.next()
                _, loss = model(x, y)
                tot += loss.float()
            v = tot / cfg["eval_iters"]
            if ddp:
                dist.all_reduce(v)
                v /= world
            out[split] = float(v)
        model.train()
        return out

    flops_per_tok = model.flops_per_token(T) if hasattr(model, "flops_per_token") else 0.0
    prof = None
    if cfg["profile_steps"] > 0 and master:
        acts = [torch.profiler.ProfilerActivity.CPU]
        if device.type == "cuda":
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        prof = torch.profiler.profile(
            activities=acts,
            schedule=torch.profiler.schedule(wait=max(0, cfg["profile_start"] - 1), warmup=1,
                                             active=cfg["profile_steps"], repeat=1),
            on_trace_ready=lambda p: p.export_chrome_trace(
                os.path.join(cfg["out_dir"], f"trace_rank{rank}.json")))
        prof.start()
    t0 = time.time()
    last_losses = {}
    while True:
        it = trainer.iter_num
        if it % cfg["eval_interval"] == 0 and (it > 0 or cfg["eval_only"]) or it >= cfg["max_iters"]:
            last_losses = estimate_loss()
            if master:
                print(f"step {it}: train loss {last_losses['train']:.4f}, val loss {last_losses['val']:.4f}")
            if last_losses["val"] < best_val or cfg["always_save_checkpoint"]:
                best_val = min(best_val, last_losses["val"])
                # under ZeRO-1 every rank takes part in gathering the sharded state
                if it > 0 and (master or trainer.zero1):
                    save_checkpoint(os.path.join(cfg["out_dir"], "ckpt.pt"), trainer, best_val, cfg,
                                    write=master)
            if cfg["eval_only"] or it >= cfg["max_iters"]:
                break
        batches = [train_src.next() for _ in range(A)]
        loss = trainer.step(batches)
        if prof is not None:
            prof.step()
        if it % cfg["log_interval"] == 0:
            trainer.check_token_ids()  # raises on out-of-range token data (one sync per log)
        if it % cfg["log_interval"] == 0 and master:
            lossf = float(loss)
            dt = time.time() - t0
            t0 = time.time()
            tps = tokens_per_iter / dt if it > 0 else 0.0
            mfu = tps / world * flops_per_tok / cfg["peak_flops"]
            mem = (f", mem {torch.cuda.max_memory_allocated(device) / 2**30:.1f} GiB"
                   if device.type == "cuda" else "")
            print(f"iter {it}: loss {lossf:.4f}, time {dt * 1000:.2f}ms, lr {trainer.opt.lr:.2e}, "
                  f"tok/s {tps:,.0f}, mfu {100 * mfu:.1f}%{mem}", flush=True)

    if prof is not None:
        prof.stop()
    if master and os.environ.get("METAOPT_RESULTS_PATH"):
        from orion_amd.client import report_results
        report_results([dict(name="val_loss", type="objective", value=float(last_losses.get("val", best_val)))])
    if ddp:
        dist.destroy_process_group()
    return last_losses


if __name__ == "__main__":
    main()
