"""Training-step engine: flat bf16 weight arena + fp32 gradient arena + fused AdamW +
optional RCCL DDP.

``Trainer.step(batches)`` runs ``len(batches)`` micro-steps of forward and
backward (gradient accumulation into the flat arena), reduces gradients across
data-parallel ranks with backward overlap on the last micro-step, then applies
one fused AdamW step.  Nothing in the step synchronises with the host; the loss
is returned as a device tensor.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from ..ops.gemm import forced_fallbacks, hip_gemms
from .flat import FlatArena
from .optim import FlatAdamW


@dataclass
class OptimConfig:
    learning_rate: float = 6e-4
    weight_decay: float = 0.1
    beta1: float = 0.9
    beta2: float = 0.95
    grad_clip: float = 1.0
    warmup_iters: int = 2000
    lr_decay_iters: int = 600000
    min_lr: float = 6e-5
    decay_lr: bool = True


_GRAPH_SYNC = os.environ.get("ORION_GRAPH_SYNC") == "1"  # debugging aid


ZERO1_AUTO_PARAMS = int(float(os.environ.get("ORION_ZERO1_AUTO_PARAMS", "1e9")))


def cosine_lr(it: int, cfg: OptimConfig) -> float:
    """nanoGPT's schedule: linear warmup, cosine decay to min_lr."""
    if not cfg.decay_lr:
        return cfg.learning_rate
    if it < cfg.warmup_iters:
        return cfg.learning_rate * (it + 1) / (cfg.warmup_iters + 1)
    if it > cfg.lr_decay_iters:
        return cfg.min_lr
    ratio = (it - cfg.warmup_iters) / max(1, cfg.lr_decay_iters - cfg.warmup_iters)
    coeff = 0.5 * (1.0 + math.cos(math.pi * ratio))
    return cfg.min_lr + coeff * (cfg.learning_rate - cfg.min_lr)


class Trainer:
    """``graph=True`` (single GPU) captures the whole optimizer step -- zero-grad, every
    micro-batch's forward/backward, the fused AdamW -- in one HIP graph after two eager
    warm-up steps, and replays it with fresh batches (copied into static buffers) and
    fresh learning-rate / bias-correction scalars (written to the optimizer's device
    hyper vector before each replay).  It removes the per-kernel launch cost, which is
    what bounds small models and small micro-batches."""

    GRAPH_WARMUP = 2
    # The warm-up and the capture run every linear-layer GEMM on the in-tree gemm16 kernel
    # (ops.gemm.hip_gemms; csrc/gemm.hip dispatches to csrc/gemm16.hip, the same kernel the
    # eager step uses for dgrad / wgrad): in round 1 the captured hipBLASLt GEMMs faulted (memory-aperture
    # violation) on the third replay at 65,536 tokens per micro-batch and rocBLAS gave NaNs,
    # which is why capture used to be capped at 8,192 tokens.  With the in-tree GEMM every
    # kernel of the step takes its arguments by value, so a replay depends on no host-side
    # library state.  ORION_GRAPH_MAX_TOKENS still caps the captured micro-batch (0 = none).
    GRAPH_MAX_TOKENS = int(os.environ.get("ORION_GRAPH_MAX_TOKENS", 0))

    def __init__(self, model: torch.nn.Module, optim: OptimConfig | None = None,
                 ddp: bool | None = None, bucket_mb: float | None = None, arena_dtype=None,
                 graph: bool = False, grad_dtype=None, ddp_timing: bool = False,
                 zero1: bool | None = None, tied_bf16: bool | None = None):
        self.model = model
        self.cfg = optim or OptimConfig()
        dev = next(model.parameters()).device
        if arena_dtype is None:
            arena_dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
        if grad_dtype is None:
            # fp32 gradients: micro-batch accumulation and the all-reduce keep fp32
            # precision; ORION_GRAD_DTYPE=bf16 opts into the all-bf16 arena
            grad_dtype = (torch.bfloat16 if os.environ.get("ORION_GRAD_DTYPE") == "bf16"
                          else torch.float32)
        if ddp is None:
            ddp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        # ZeRO-1 (parallel/ddp.py ShardedGradReducer): reduce-scatter the gradient buckets, AdamW
        # on this rank's 1/N shard of master / m / v, all-gather the bf16 weights.  Also valid
        # with one rank (a rehearsal of the sharded code path).
        # zero1=None (auto): sharded from ZERO1_AUTO_PARAMS parameters up when there is more
        # than one rank -- a 7B model's replicated fp32 master + Adam state is 81 GB per GPU and
        # its all-reduce moves 2 (N-1)/N x 27 GB of fp32 gradients per step
        # split tied gradient with a bf16 tail on the wire (parallel/ddp.py; opt-in,
        # ORION_DDP_TIED_BF16=1): halves the exposed bytes of GPT-2's tied wte bucket
        if tied_bf16 is None:
            tied_bf16 = os.environ.get("ORION_DDP_TIED_BF16") == "1"
        dist_on = dist.is_available() and dist.is_initialized()
        if zero1 is None:
            zero1 = (dist_on and dist.get_world_size() > 1
                     and sum(p.numel() for p in model.parameters()) >= ZERO1_AUTO_PARAMS)
        self.zero1 = bool(zero1) and dist_on
        self.reducer = None
        if self.zero1:
            from ..parallel.ddp import ShardedGradReducer, zero1_pad_names
            names, pad_to = zero1_pad_names(model, bucket_mb, grad_dtype, dist.get_world_size())
            self.arena = FlatArena(model, dtype=arena_dtype, grad_dtype=grad_dtype,
                                   pad_after=names, pad_to=pad_to)
            # R1: every rank starts from rank 0's exact fp32 weights
            dist.broadcast(self.arena.init_fp32, 0)
            with torch.no_grad():
                self.arena.params.copy_(self.arena.init_fp32)
            self.reducer = ShardedGradReducer(self.arena, bucket_mb=bucket_mb, timing=ddp_timing,
                                              tied_bf16=tied_bf16)
            self.reducer.install_gather_hooks(model)
            self.reducer.init_fp32 = self.reducer.shard_of(self.arena.init_fp32)
            self.arena.init_fp32 = None
            self.opt = FlatAdamW(self.reducer, lr=self.cfg.learning_rate,
                                 betas=(self.cfg.beta1, self.cfg.beta2),
                                 weight_decay=self.cfg.weight_decay, grad_clip=self.cfg.grad_clip)
            self.opt.sumsq_hook = self.reducer.reduce_sumsq
        else:
            self.arena = FlatArena(model, dtype=arena_dtype, grad_dtype=grad_dtype)
            self.opt = FlatAdamW(self.arena, lr=self.cfg.learning_rate,
                                 betas=(self.cfg.beta1, self.cfg.beta2),
                                 weight_decay=self.cfg.weight_decay, grad_clip=self.cfg.grad_clip)
            if ddp:
                from ..parallel.ddp import GradBucketReducer
                self.reducer = GradBucketReducer(self.arena, bucket_mb=bucket_mb, timing=ddp_timing,
                                                 tied_bf16=tied_bf16)
                # R1: every rank starts from rank 0's exact fp32 weights
                dist.broadcast(self.opt.master, 0)
                with torch.no_grad():
                    self.arena.params.copy_(self.opt.master)
        self.iter_num = 0
        # communication kernels beside the backward GEMMs need CUs (ops/gemm.py set_per_item_walk)
        if (self.reducer is not None and dev.type == "cuda" and dist.get_world_size() > 1
                and os.environ.get("ORION_GEMM_DDP_PERSISTENT") != "1"):
            import weakref
            from ..ops.gemm import request_per_item_walk
            # scoped to this trainer (reference counted across trainers): the explicit walk
            # comes back when the last requesting trainer is collected
            weakref.finalize(self, request_per_item_walk())
        self.graph_enabled = bool(graph) and dev.type == "cuda" and self.reducer is None
        self._graph = None
        self._static = None
        self._static_loss = None
        self._side = None

    def step(self, batches):
        """batches: sequence of (idx, targets) micro-batches.  Returns mean loss (device)."""
        if (self.graph_enabled and self._graph is None and self.GRAPH_MAX_TOKENS
                and batches[0][0].numel() > self.GRAPH_MAX_TOKENS):
            print(f"[orion_amd] HIP-graph capture is validated up to {self.GRAPH_MAX_TOKENS} tokens "
                  f"per micro-batch; running {batches[0][0].numel()} eagerly", flush=True)
            self.graph_enabled = False
        if self.graph_enabled:
            return self._step_graph(batches)
        return self._step_eager(batches)

    def _step_eager(self, batches):
        self.opt.set_lr(cosine_lr(self.iter_num, self.cfg))
        self.arena.zero_grad()
        n = len(batches)
        losses = []
        for i, (x, y) in enumerate(batches):
            if self.reducer is not None:
                self.reducer.set_sync(i == n - 1)
            _, loss = self.model(x, y)
            (loss / n).backward()
            losses.append(loss.detach())
        self.arena.finish_grads()
        if self.reducer is not None:
            self.reducer.finish()
        self.opt.step()
        if self.zero1:
            self.reducer.gather_params()
        self.iter_num += 1
        return torch.stack(losses).mean()

    # ------------------------------------------------------------------ HIP graph
    def _body(self, batches):
        self.arena.zero_grad()
        n = len(batches)
        losses = []
        for x, y in batches:
            _, loss = self.model(x, y)
            (loss / n).backward()
            losses.append(loss.detach())
        self.arena.finish_grads()
        self.opt.step(hyper_prefilled=True)
        return torch.stack(losses).mean()

    def _step_graph(self, batches):
        self.opt.set_lr(cosine_lr(self.iter_num, self.cfg))
        if self._graph is None and self.iter_num < self.GRAPH_WARMUP:
            # eager warm-up on a side stream: lazy inits (kernel attributes, TunableOp
            # lookups, allocator pools) must not happen inside the capture
            if self._side is None:
                self._side = torch.cuda.Stream()
            self._side.wait_stream(torch.cuda.current_stream())
            forced_fallbacks(clear=True)
            with torch.cuda.stream(self._side), hip_gemms():
                self.opt.hyper_tensor()
                loss = self._body(batches)
            torch.cuda.current_stream().wait_stream(self._side)
            self.iter_num += 1
            fb = forced_fallbacks(clear=True)
            if fb:
                # a library GEMM must not be captured (ops/gemm.py _FORCED_FALLBACKS): eager
                print(f"[orion_amd] HIP-graph capture disabled: {len(fb)} GEMM(s) not eligible for "
                      f"the in-tree kernels, e.g. {fb[0]}; the step runs eagerly", flush=True)
                self.graph_enabled = False
            return loss
        if self._graph is None:
            self._static = [(x.clone(), y.clone()) for x, y in batches]
            self.opt.hyper_tensor()
            self._graph = torch.cuda.CUDAGraph()
            torch.cuda.synchronize()
            with torch.cuda.graph(self._graph), hip_gemms():
                self._static_loss = self._body(self._static)
            self.opt.step_count -= 1  # the capture ran nothing; the replay below is the step
        else:
            if len(batches) != len(self._static):
                raise ValueError("a captured step needs the same number of micro-batches")
            for (sx, sy), (x, y) in zip(self._static, batches):
                sx.copy_(x, non_blocking=True)
                sy.copy_(y, non_blocking=True)
            self.opt.hyper_tensor()
        self._graph.replay()
        if _GRAPH_SYNC:
            torch.cuda.synchronize()
        self.opt.step_count += 1
        self.iter_num += 1
        return self._static_loss

    def sync_params(self):
        """Wait for ZeRO-1's overlapped weight all-gathers (a no-op otherwise): for code that
        reads ``arena.params`` directly instead of through a module forward."""
        if self.zero1:
            self.reducer.wait_params()

    def check_token_ids(self):
        """Raise IndexError if an embedding kernel saw a token id outside the table since the
        last check (the kernels clamp / skip such ids and raise a device flag rather than
        fault; ops/embedding.py).  Synchronises: call it where the loop syncs anyway (log and
        eval intervals)."""
        dev = next(self.model.parameters()).device
        if dev.type != "cuda":
            return
        from ..ops import embedding
        from ..ops._ext import ext_loaded
        if ext_loaded() and embedding.id_error(dev):
            raise IndexError("token id out of range for the embedding table (device flag set by the "
                             "embedding kernels; the batch was trained with those ids clamped)")

    def full_master(self):
        """fp32 master weights in arena layout (gathered from the shards under ZeRO-1)."""
        return self.reducer.gather_full(self.opt.master) if self.zero1 else self.opt.master

    def state_dict(self):
        return dict(model=self.arena.state_dict_fp32(self.full_master()),
                    optimizer=self.opt.state_dict(), iter_num=self.iter_num)
