#!/usr/bin/env python3
"""Sample from a trained checkpoint (nanoGPT ``sample.py`` interface).

    python sample.py --out_dir=out --start="Hello" --num_samples=3 --max_new_tokens=100

``--start`` may be text (encoded with the GPT-2 BPE when ``tiktoken`` is
available), ``FILE:<path>``, or a comma-separated list of token ids
(``--start=ids:50256,464``).  Without a tokenizer the token ids are printed.
"""
from __future__ import annotations

import ast
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

DEFAULTS = dict(out_dir="out", start="\n", num_samples=10, max_new_tokens=500, temperature=0.8,
                top_k=200, seed=1337, device="cuda", ckpt="ckpt.pt")


def main(argv=None):
    cfg = dict(DEFAULTS)
    for arg in (sys.argv[1:] if argv is None else argv):
        k, _, v = arg.lstrip("-").partition("=")
        if k not in cfg:
            raise ValueError(f"Unknown config key: {k}")
        try:
            cfg[k] = ast.literal_eval(v)
        except (ValueError, SyntaxError):
            cfg[k] = v
    from orion_amd.train.ckpt import build_model_from_checkpoint, load_checkpoint
    torch.manual_seed(cfg["seed"])
    dev = torch.device(cfg["device"] if torch.cuda.is_available() or cfg["device"] == "cpu" else "cpu")
    ckpt = load_checkpoint(os.path.join(cfg["out_dir"], cfg["ckpt"]))
    model = build_model_from_checkpoint(ckpt).to(dev)
    if dev.type == "cuda":
        model = model.to(torch.bfloat16)
        for name, buf in model.named_buffers():
            if name.startswith("rope_"):
                buf.data = buf.data.float()
    model.eval()
    try:
        import tiktoken
        enc = tiktoken.get_encoding("gpt2")
        encode, decode = (lambda s: enc.encode(s, allowed_special={"<|endoftext|>"})), enc.decode
    except Exception:
        encode, decode = None, None
    start = cfg["start"]
    if isinstance(start, str) and start.startswith("FILE:"):
        start = open(start[5:]).read()
    if isinstance(start, str) and start.startswith("ids:"):
        ids = [int(t) for t in start[4:].split(",") if t]
    elif encode is not None:
        ids = encode(start)
    else:
        ids = [50256 if model.config.vocab_size > 50256 else 0]
    x = torch.tensor(ids, dtype=torch.long, device=dev)[None]
    with torch.no_grad():
        for _ in range(cfg["num_samples"]):
            y = model.generate(x, cfg["max_new_tokens"], temperature=cfg["temperature"], top_k=cfg["top_k"])
            toks = y[0].tolist()
            print(decode(toks) if decode else toks)
            print("---------------")


if __name__ == "__main__":
    main()
