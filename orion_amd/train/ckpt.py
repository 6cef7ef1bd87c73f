"""nanoGPT-compatible checkpoints (SURVEY.md §5 checkpoint/resume, north star).

``ckpt.pt`` layout (``torch.save`` of a dict, loadable with ``weights_only=True``):

* ``model``      -- fp32 state dict with the model's parameter names (taken from
                    the optimizer's fp32 master weights, not the bf16 compute copy);
* ``optimizer``  -- ``{"step", "lr", "betas", "eps", "weight_decay", "grad_clip",
                    "exp_avg", "exp_avg_sq"}`` as flat fp32 tensors (arena order);
* ``model_args`` -- the model config dict (``GPTConfig``/``LlamaConfig`` fields);
* ``model_type`` -- ``"gpt2"`` or ``"llama"``;
* ``iter_num``, ``best_val_loss``, ``config`` -- as in nanoGPT's train.py.

Writes are atomic (temp file + rename) so an interrupted trial never leaves a
truncated checkpoint; only rank 0 writes in data-parallel runs.
"""
from __future__ import annotations

import os

import torch


def model_type_of(model):
    from ..models.llama import Llama
    return "llama" if isinstance(model, Llama) else "gpt2"


def save_checkpoint(path, trainer, best_val_loss=None, config=None, write=True):
    """nanoGPT layout.  Under ZeRO-1 the master weights and Adam moments are gathered from
    the shards (a collective: every rank calls this, ``write`` only on one).  A rank that does
    not write joins the gathers and keeps nothing: no host copy of the state is built there
    (84 GB of host RAM per rank for Llama-7B)."""
    model = trainer.model
    opt = trainer.opt
    zero1 = getattr(trainer, "zero1", False)
    if not write and not zero1:
        return path  # nothing to join
    osd = opt.state_dict()
    if zero1:
        # per-bucket gathers, the full tensors assembled on the host of the writer only
        master = trainer.reducer.gather_full_host(opt.master, keep=write)
        fulls = {k: trainer.reducer.gather_full_host(osd[k], keep=write) for k in ("exp_avg", "exp_avg_sq")}
    else:
        master = opt.master
        fulls = {k: osd[k] for k in ("exp_avg", "exp_avg_sq")}
    if not write:
        return path
    sd = {}
    for s in trainer.arena.slots:
        sd[s.name] = master[s.offset:s.offset + s.numel].view(s.param.shape).detach().float().cpu().clone()
    # tied weights appear once in the arena; restore every alias name
    for name, p in model.named_parameters(remove_duplicate=False):
        if name not in sd:
            for s in trainer.arena.slots:
                if s.param is p:
                    sd[name] = sd[s.name]
    # per parameter name, so a checkpoint restores into any arena layout (ZeRO-1 padding,
    # another world size)
    for k, full in fulls.items():
        osd[k] = {s.name: full[s.offset:s.offset + s.numel].detach().cpu().clone() for s in trainer.arena.slots}
    ckpt = {
        "model": sd,
        "optimizer": {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in osd.items()
                      if k != "master"},
        "model_args": model.config.to_dict(),
        "model_type": model_type_of(model),
        "iter_num": trainer.iter_num,
        "best_val_loss": best_val_loss,
        "config": dict(config or {}),
    }
    tmp = f"{path}.tmp{os.getpid()}"
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    torch.save(ckpt, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path, map_location="cpu"):
    return torch.load(path, map_location=map_location, weights_only=True)


def build_model_from_checkpoint(ckpt):
    from ..models.gpt2 import GPT, GPTConfig
    from ..models.llama import Llama, LlamaConfig
    if ckpt.get("model_type", "gpt2") == "llama":
        model = Llama(LlamaConfig(**ckpt["model_args"]))
    else:
        model = GPT(GPTConfig(**ckpt["model_args"]))
    sd = ckpt["model"]
    # nanoGPT checkpoints from torch.compile carry an '_orig_mod.' prefix
    sd = {k[len("_orig_mod."):] if k.startswith("_orig_mod.") else k: v for k, v in sd.items()}
    model.load_state_dict(sd, strict=False)
    return model


def restore_trainer(trainer, ckpt):
    """Load master weights + Adam state into an existing Trainer (resume); under ZeRO-1 each
    rank keeps its shard of them."""
    opt = trainer.opt
    sd = ckpt["model"]
    zero1 = getattr(trainer, "zero1", False)
    with torch.no_grad():
        full = torch.zeros(trainer.arena.numel, dtype=torch.float32, device=opt.master.device) \
            if zero1 else opt.master
        for s in trainer.arena.slots:
            full[s.offset:s.offset + s.numel].copy_(sd[s.name].reshape(-1))
        o = dict(ckpt["optimizer"])
        for k in ("exp_avg", "exp_avg_sq"):
            if isinstance(o[k], dict):  # per-name moments -> this trainer's arena layout
                flat = torch.zeros(trainer.arena.numel, dtype=torch.float32, device=full.device)
                for s in trainer.arena.slots:
                    flat[s.offset:s.offset + s.numel].copy_(o[k][s.name].reshape(-1))
                o[k] = flat
        if zero1:
            shard = trainer.reducer.shard_of
            o["exp_avg"] = shard(o["exp_avg"].to(full.device))
            o["exp_avg_sq"] = shard(o["exp_avg_sq"].to(full.device))
            o["master"] = shard(full)
            opt.load_state_dict(o)
            trainer.reducer.gather_params()
        else:
            o["master"] = opt.master
            opt.load_state_dict(o)
    trainer.iter_num = int(ckpt.get("iter_num", 0))
    return trainer
