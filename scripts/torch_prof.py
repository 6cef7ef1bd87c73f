#!/usr/bin/env python3
"""Attribute the non-GEMM / non-kernel-library device time of one training step to the aten
ops that launch it (torch.profiler with shapes): copies, fills and elementwise adds that a
rocprofv3 kernel summary only shows as `__amd_rocclr_copyBuffer` / `FillFunctor` rows.

usage: python scripts/torch_prof.py [--model llama2-7b] [--layers 2] [--seq-len 4096] [--micro-batch 4]
Prints the top aten ops by self device time (one profiled step after two warm-up steps)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=4)
    ap.add_argument("--rows", type=int, default=30)
    a = ap.parse_args()
    from orion_amd import ops
    from orion_amd.models import GPT2_PRESETS, build_model
    from orion_amd.train.engine import OptimConfig, Trainer
    ops.load_ext(required=True)
    dev = torch.device("cuda")
    is_gpt2 = a.model in GPT2_PRESETS
    kw = dict(block_size=a.seq_len, n_layer=a.layers) if is_gpt2 else dict(max_seq_len=a.seq_len, n_layers=a.layers)
    with torch.device(dev):
        model = build_model(a.model, **kw)
    vocab = 50257 if is_gpt2 else model.config.vocab_size
    g = torch.Generator(device=dev).manual_seed(0)
    batch = [(torch.randint(0, vocab, (a.micro_batch, a.seq_len), device=dev, generator=g),
              torch.randint(0, vocab, (a.micro_batch, a.seq_len), device=dev, generator=g))]
    tr = Trainer(model, OptimConfig(warmup_iters=10, lr_decay_iters=1000))
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        tr.step(batch)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total",
                                                               row_limit=a.rows, max_name_column_width=40,
                                                               max_shapes_column_width=60))


if __name__ == "__main__":
    main()
