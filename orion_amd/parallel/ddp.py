"""Data-parallel gradient reduction over RCCL (xGMI) with backward overlap.

Design (MI355X-first, not a translation of any NCCL call pattern):

* gradients live in ONE flat arena (``train/flat.py``) laid out in reverse
  module order, so a bucket is a contiguous slice of it: an all-reduce runs
  in place on the arena, no copy-in/copy-out and no per-parameter launches;
* buckets default to 64 MB (256 MB from 1B parameters up, ``default_bucket_mb``):
  a ring all-reduce on an 8-GPU xGMI node is bound
  by per-link bandwidth (7 point-to-point links, ~153 GB/s each), and RCCL
  needs tens of MB per call to spread its channels over all links; fewer,
  larger collectives also mean fewer launches competing with backward;
* a ``register_post_accumulate_grad_hook`` per parameter counts arrivals per
  bucket; once a bucket's last gradient lands its ``all_reduce`` is issued
  asynchronously (RCCL runs on its own HIP stream, ordered after the producing
  kernels by an event), so communication overlaps the rest of backward;
* collectives are issued strictly in bucket order: bucket i launches only after
  buckets 0..i-1 have.  RCCL matches collectives by issue order on every rank,
  and gradient ARRIVAL order is not guaranteed to agree across ranks (sink
  notifications vs AccumulateGrad hooks, unused parameters, data-dependent
  graphs); a ready bucket behind a not-yet-ready one waits in ``_ready`` and is
  flushed the moment the cursor reaches it;
* a tied parameter (GPT-2's ``wte`` = LM head) starts a bucket of its own: its
  gradient is complete only after the embedding backward, the last kernel of the
  pass, and would otherwise hold back every layer sharing its bucket;
* split tied gradient (``tied_bf16``, opt-in): the tied bucket is reduced as soon as the
  LM head has written its part (under the whole backward), and only the embedding's part --
  written by the last kernel into a separate fp32 tail -- is reduced after the backward, in
  bf16 on the wire: the exposed bytes of GPT-2-124M's 154.5 MB tied bucket halve, and the
  LM head's (larger, denser) contribution keeps fp32 precision;
* gradient accumulation: reduction is only armed on the last micro-step
  (``set_sync``), the same contract as DDP's ``no_sync``;
* observability (``timing=True``): per bucket, the moment its gradients were ready on the
  compute stream and the moment its collective completed (HIP events: the completion
  event is recorded on a side stream made to wait for the collective), plus the end of the
  backward, so ``timing_report()`` gives each bucket's launch->complete time and the
  exposed communication tail (last completion minus backward end) of the last step;
* fail-fast: a watchdog thread (``ORION_DDP_WATCHDOG_S``, default 180 s, 0 = off) checks
  the launched collectives; one that has not completed in time makes the rank print which
  bucket of which step it was stuck on and exit 124, instead of the job hanging inside RCCL
  until the driver's own limit.

Works with any ``torch.distributed`` backend: ``nccl`` (= RCCL on ROCm) on
GPUs, ``gloo`` on CPU for the multi-process tests.
"""
from __future__ import annotations

import os
import sys
import threading
import time

import torch
import torch.distributed as dist

from ..train.flat import FlatArena


def default_bucket_mb(n_params: int) -> float:
    """Bucket size for a model of ``n_params`` parameters.  64 MB for GPT-2-class models
    (~8 buckets of the 0.5 GB fp32 arena: the first launches a few layers into backward);
    256 MB from 1B parameters up (Llama-7B's 27 GB fp32 arena: ~105 collectives per step
    instead of ~420, three per decoder layer), where per-call latency and RCCL's channel
    ramp-up would otherwise eat into the xGMI link bandwidth."""
    return 256.0 if n_params >= 1_000_000_000 else 64.0


def plan_buckets(slots, bucket_mb: float, esize: int) -> list[list[int]]:
    """Greedy bucket plan over arena-ordered slots ``(name, numel, tied)``: a bucket closes
    once it holds ``bucket_mb`` of (ALIGN-padded) gradients; a tied parameter (GPT-2's wte =
    LM head) starts a bucket of its own -- its gradient completes only after the embedding
    backward, the last kernel of the pass, and would hold back every layer sharing its
    bucket.  A pure function of the slot sizes, so the arena can be laid out with per-bucket
    padding (ZeRO-1) before the reducer exists.  Returns slot indices per bucket."""
    from ..train.flat import ALIGN
    cap = max(1, int(bucket_mb * 1024 * 1024 / esize))
    buckets, cur, size = [], [], 0
    for i, (_, numel, tied) in enumerate(slots):
        if tied and cur:
            buckets.append(cur)
            cur, size = [], 0
        cur.append(i)
        size += (numel + ALIGN - 1) // ALIGN * ALIGN
        if size >= cap:
            buckets.append(cur)
            cur, size = [], 0
    if cur:
        buckets.append(cur)
    return buckets


class _Watchdog(threading.Thread):
    """Polls the reducer's launched collectives; a bucket pending longer than ``limit``
    seconds ends the process with a message naming it (exit 124)."""

    def __init__(self, limit: float, rank: int):
        super().__init__(name="orion-ddp-watchdog", daemon=True)
        self.limit = limit
        self.rank = rank
        self.pending: list = []          # (step, bucket, t_launch, work, numel)
        self.lock = threading.Lock()
        self.stop = threading.Event()

    def add(self, step, bucket, work, numel):
        with self.lock:
            self.pending.append((step, bucket, time.monotonic(), work, numel))

    def run(self):
        while not self.stop.wait(1.0):
            with self.lock:
                live = []
                for rec in self.pending:
                    try:
                        done = rec[3].is_completed()
                    except Exception:  # noqa: BLE001 -- a failed collective is reported below
                        done = False
                    if not done:
                        live.append(rec)
                self.pending = live
                late = [r for r in live if time.monotonic() - r[2] > self.limit]
            if late:
                step, bi, t0, _, numel = late[0]
                print(f"[orion_amd.ddp] rank {self.rank}: all-reduce of bucket {bi} "
                      f"({numel} elements) of step {step} not complete after "
                      f"{time.monotonic() - t0:.0f} s ({len(live)} collective(s) pending); "
                      f"aborting", file=sys.stderr, flush=True)
                os._exit(124)


class _TiedTail:
    """The split last-use contribution of one tied parameter (``tied_bf16``): ``buf`` spans the
    parameter's whole bucket (fp32, zero outside the parameter, so a ZeRO-1 reduce-scatter of
    it shards like the bucket), ``view`` is the parameter-shaped slice the embedding backward
    writes, ``wire`` the bf16 copy that is reduced."""

    def __init__(self, bucket, b0, b1, slot, sink, device):
        self.bucket, self.b0, self.b1, self.slot, self.sink = bucket, b0, b1, slot, sink
        self.buf = torch.zeros(b1 - b0, dtype=torch.float32, device=device)
        self.view = self.buf[slot.offset - b0: slot.offset - b0 + slot.numel].view_as(slot.param)
        self.wire = torch.zeros(b1 - b0, dtype=torch.bfloat16, device=device)
        self.out = None          # ZeRO-1: this rank's reduced piece
        self.ready = False
        self.handle = None
        self.t_ready = self.t_done = None


class GradBucketReducer:
    def __init__(self, arena: FlatArena, bucket_mb: float | None = None, group=None,
                 average: bool = True, timing: bool = False, watchdog_s: float | None = None,
                 tied_bf16: bool = False):
        if bucket_mb is None or bucket_mb <= 0:
            bucket_mb = default_bucket_mb(arena.numel)
        self.arena = arena
        self.group = group
        self.world = dist.get_world_size(group)
        self.average = average
        esize = arena.grads.element_size()
        plan = plan_buckets([(s.name, s.numel, id(s.param) in getattr(arena, "shared", set()))
                             for s in arena.slots], bucket_mb, esize)
        # bucket i spans from its first slot's offset to the next bucket's (padding covered
        # exactly once; with ZeRO-1 padding every span is a multiple of world x ALIGN)
        starts = [0] + [arena.slots[idx[0]].offset for idx in plan[1:]]
        self.buckets = []
        for i, idx in enumerate(plan):
            b1 = starts[i + 1] if i + 1 < len(plan) else arena.numel
            self.buckets.append((starts[i], b1, [arena.slots[j] for j in idx]))
        self._slot_bucket = {}
        for bi, (_, _, slots) in enumerate(self.buckets):
            for s in slots:
                self._slot_bucket[id(s.param)] = bi
        self._need = [len(sl) for (_, _, sl) in self.buckets]
        self._names = {id(s.param): s.name for s in arena.slots}
        self._debug = None  # list -> (bucket, param, count, need) per arrival (tests)
        self._arrived = [set() for _ in self.buckets]
        self._handles = [None] * len(self.buckets)
        self._ready = [False] * len(self.buckets)
        self._cursor = 0                 # position in self._order of the next bucket to launch
        self.launch_log: list[int] | None = None  # tests: bucket indices in launch order
        self._sync = True
        self._hooks = [s.param.register_post_accumulate_grad_hook(self._on_grad)
                       for s in arena.slots]
        # weights whose gradient the GEMM writes straight into the arena (ops/grad_sink.py)
        # never run AccumulateGrad: their sinks report through the arena's listener list
        arena.grad_listeners.append(self._on_grad)
        avg = getattr(dist.ReduceOp, "AVG", None)
        self._use_avg_op = average and avg is not None and dist.get_backend(group) == "nccl"
        self.step = 0
        # per-bucket timing of the last armed step (events on the GPU, host clock on the CPU)
        self.timing = timing
        self._cuda = arena.grads.is_cuda
        self._tstream = None
        self._t0 = self._bwd_end = None
        self._t_ready = [None] * len(self.buckets)
        self._t_done = [None] * len(self.buckets)
        if watchdog_s is None:
            watchdog_s = float(os.environ.get("ORION_DDP_WATCHDOG_S", "180"))
        self._watchdog = None
        if watchdog_s > 0 and self.world > 1:
            self._watchdog = _Watchdog(watchdog_s, dist.get_rank(group))
            self._watchdog.start()
        # split tied gradients (module docstring): one tail per tied parameter whose gradient
        # goes through an fp32 arena sink (the GPU path; see ops/grad_sink.py)
        self.tails: list[_TiedTail] = []
        if tied_bf16:
            for bi, (b0, b1, slots) in enumerate(self.buckets):
                for sl in slots:
                    sk = getattr(sl.param, "_orion_sink", None)
                    if (id(sl.param) in getattr(arena, "shared", set()) and sk is not None
                            and sk.view.dtype == torch.float32 and sk.expect > 1):
                        self.tails.append(_TiedTail(bi, b0, b1, sl, sk, arena.grads.device))
        self._tail_cursor = 0
        # launch order: bucket index order, except that a split tied bucket goes FIRST -- the
        # LM head, which completes it, is the first kernel of the backward, while its arena
        # position (the table is the model's first module) is last.  Any fixed permutation
        # keeps every rank's collective sequence identical.
        tied = [t.bucket for t in self.tails]
        self._order = tied + [bi for bi in range(len(self.buckets)) if bi not in tied]

    # ------------------------------------------------------------------ timing
    def _mark(self):
        if self._cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    def timing_report(self):
        """Bucket timeline of the last armed step in ms from the step's first ready bucket:
        ``buckets`` = [(index, MB, ready, done)], ``bwd_end``, ``exposed_tail_ms`` = last
        completion - backward end (> 0: communication the backward did not hide).  Syncs."""
        if not self.timing or self._bwd_end is None or any(t is None for t in self._t_done):
            return None
        if self._cuda:
            torch.cuda.synchronize()
            ref = self._t_ready[0]
            rel = lambda ev: ref.elapsed_time(ev)  # noqa: E731
        else:
            ref = self._t_ready[0]
            rel = lambda t: (t - ref) * 1e3  # noqa: E731
        esize = self.arena.grads.element_size()
        rows = []
        for bi, (b0, b1, _) in enumerate(self.buckets):
            rows.append((bi, round((b1 - b0) * esize / 2**20, 2), round(rel(self._t_ready[bi]), 3),
                         round(rel(self._t_done[bi]), 3)))
        tails = [(t.bucket, round(t.wire.numel() * t.wire.element_size() / 2**20, 2),
                  round(rel(t.t_ready), 3), round(rel(t.t_done), 3))
                 for t in self.tails if t.t_ready is not None and t.t_done is not None]
        bwd = rel(self._bwd_end)
        last = max(r[3] for r in rows + tails)
        return {"buckets": rows, "tied_tails": tails, "bwd_end_ms": round(bwd, 3),
                "exposed_tail_ms": round(max(0.0, last - bwd), 3),
                "comm_ms": round(sum(r[3] - r[2] for r in rows + tails), 3)}

    # ------------------------------------------------------------------ control
    def set_sync(self, flag: bool):
        """Arm (True) or disarm (False) reduction for the coming backward.  Armed, a tied
        parameter's last use writes into its split tail (``tied_bf16``)."""
        self._sync = flag
        for t in self.tails:
            t.sink.tail = t.view if flag else None
            t.sink.tail_cb = self._on_tail if flag else None

    def _on_tail(self, p):
        """The last use of tied parameter ``p`` wrote its tail (on the compute stream): make
        the bf16 wire copy and launch it once every bucket has launched."""
        for t in self.tails:
            if t.slot.param is p:
                t.wire.copy_(t.buf)
                t.ready = True
        self._flush()

    def broadcast_params(self, src=0):
        """R1: make every rank start from rank ``src``'s weights."""
        dist.broadcast(self.arena.params, src, group=self.group)

    def _on_grad(self, p):
        if not self._sync:
            return
        bi = self._slot_bucket[id(p)]
        # a parameter counts once per step: a weight whose GEMM wrote its gradient straight
        # into the arena reports through its sink, and torch 2.10 still runs the (no-op)
        # post-accumulate hook of that parameter afterwards
        arrived = self._arrived[bi]
        if id(p) in arrived:
            return
        arrived.add(id(p))
        if self._debug is not None:
            self._debug.append((bi, self._names[id(p)], len(arrived), self._need[bi]))
        if len(arrived) == self._need[bi]:
            self._ready[bi] = True
            self._flush()

    def _flush(self):
        """Launch every ready bucket at the cursor, in launch order (``_order``); the tied tails
        go last, so every rank issues the same sequence of collectives."""
        while self._cursor < len(self.buckets) and self._ready[self._order[self._cursor]]:
            self._launch(self._order[self._cursor])
            self._cursor += 1
        if self._cursor == len(self.buckets):
            while self._tail_cursor < len(self.tails) and self.tails[self._tail_cursor].ready:
                self._launch_tail(self.tails[self._tail_cursor])
                self._tail_cursor += 1

    def _tail_collective(self, t, op):
        return dist.all_reduce(t.wire, op=op, group=self.group, async_op=True)

    def _launch_tail(self, t):
        if self.launch_log is not None:
            self.launch_log.append(("tail", t.bucket))
        op = dist.ReduceOp.AVG if self._use_avg_op else dist.ReduceOp.SUM
        if self.timing:
            t.t_ready = self._mark()
        t.handle = self._tail_collective(t, op)
        if self.timing and self._cuda:
            if self._tstream is None:
                self._tstream = torch.cuda.Stream()
            with torch.cuda.stream(self._tstream):
                t.handle.wait()
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(self._tstream)
            t.t_done = ev
        if self._watchdog is not None:
            self._watchdog.add(self.step, f"tied tail of bucket {t.bucket}", t.handle, t.wire.numel())

    def _finish_tails(self, add_into):
        """Wait for the tails and add each (averaged) into ``add_into(t)`` (the fp32 gradient
        the tail belongs to); a tied parameter whose last use wrote around its sink while the
        split was armed is an error (its bucket was being reduced while it was written)."""
        for t in self.tails:
            if not t.ready:
                if t.sink.notes:
                    raise RuntimeError(
                        f"tied_bf16: {t.slot.name}'s last use did not write through its gradient "
                        "sink (an AccumulateGrad path?) -- run without ORION_DDP_TIED_BF16")
                continue
            t.handle.wait()
            if self.timing and not self._cuda:
                t.t_done = time.perf_counter()
            src = t.out if t.out is not None else t.wire
            add_into(t).add_(src, alpha=1.0 if self._use_avg_op else 1.0 / self.world)
            t.ready, t.handle = False, None
        self._tail_cursor = 0

    def _launch(self, bi):
        if self._handles[bi] is not None:
            return
        if self.launch_log is not None:
            self.launch_log.append(bi)
        b0, b1, _ = self.buckets[bi]
        view = self.arena.grads[b0:b1]
        op = dist.ReduceOp.AVG if self._use_avg_op else dist.ReduceOp.SUM
        if self.timing:
            self._t_ready[bi] = self._mark()
        h = dist.all_reduce(view, op=op, group=self.group, async_op=True)
        self._handles[bi] = h
        if self.timing and self._cuda:
            # completion: a side stream waits for the collective, then records
            if self._tstream is None:
                self._tstream = torch.cuda.Stream()
            with torch.cuda.stream(self._tstream):
                h.wait()
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(self._tstream)
            self._t_done[bi] = ev
        if self._watchdog is not None:
            self._watchdog.add(self.step, bi, h, b1 - b0)

    def finish(self):
        """Launch stragglers (unused params), wait for every bucket, reset counters."""
        if not self._sync:
            return
        if self.timing:
            self._bwd_end = self._mark()
        self._ready = [True] * len(self.buckets)
        self._flush()
        for bi, h in enumerate(self._handles):
            h.wait()
            if self.timing and not self._cuda:
                self._t_done[bi] = time.perf_counter()
            if self.average and not self._use_avg_op:
                b0, b1, _ = self.buckets[bi]
                self.arena.grads[b0:b1].div_(self.world)
        self._finish_tails(lambda t: self.arena.grads[t.b0:t.b1])
        self._handles = [None] * len(self.buckets)
        self._arrived = [set() for _ in self.buckets]
        self._ready = [False] * len(self.buckets)
        self._cursor = 0
        self.step += 1

    def remove(self):
        for t in self.tails:
            t.sink.tail = t.sink.tail_cb = None
        if self._watchdog is not None:
            self._watchdog.stop.set()
            self._watchdog = None
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self._on_grad in self.arena.grad_listeners:
            self.arena.grad_listeners.remove(self._on_grad)


class ShardedGradReducer(GradBucketReducer):
    """ZeRO-1 over the same buckets: each bucket is REDUCE-SCATTERED (rank r receives the
    averaged r-th 1/N of it) instead of all-reduced, the optimizer updates only the rank's
    shard of fp32 master / m / v, and the new bf16 weights are ALL-GATHERED bucket by bucket.

    Per step and rank that moves (N-1)/N x (fp32 gradients + bf16 weights) = 0.75x the ring
    all-reduce's 2 (N-1)/N x fp32 gradients, keeps 12/N instead of 12 bytes of optimizer state
    per parameter (Llama-7B at N = 8: 10 GB instead of 81 GB) and runs AdamW over 1/N of the
    parameters.  The arena must be laid out with ``pad_after=zero1_pad_names(...)`` and
    ``pad_to = world x ALIGN`` so that every bucket splits into N equal ALIGN-aligned shards.

    Shard layout: the rank's pieces of all buckets, concatenated in bucket order
    (``shard_ranges``), so the gradient / parameter shards and the optimizer state are each one
    flat buffer and the fused AdamW kernel runs over them unchanged."""

    def __init__(self, arena: FlatArena, bucket_mb: float | None = None, group=None,
                 timing: bool = False, watchdog_s: float | None = None, tied_bf16: bool = False):
        super().__init__(arena, bucket_mb=bucket_mb, group=group, average=True, timing=timing,
                         watchdog_s=watchdog_s, tied_bf16=tied_bf16)
        from ..train.flat import ALIGN
        self.rank = dist.get_rank(group)
        n = self.world
        self.shard_ranges = []  # (bucket, arena offset of this rank's piece, shard offset, length)
        off = 0
        for bi, (b0, b1, _) in enumerate(self.buckets):
            span = b1 - b0
            if span % (n * ALIGN):
                raise ValueError(f"bucket {bi} spans {span} elements, not a multiple of "
                                 f"{n} x {ALIGN}: lay the arena out with zero1_pad_names()")
            piece = span // n
            self.shard_ranges.append((bi, b0 + self.rank * piece, off, piece))
            off += piece
        self.shard_numel = off
        for t in self.tails:
            t.out = torch.zeros((t.b1 - t.b0) // n, dtype=torch.bfloat16, device=arena.grads.device)
        dev = arena.grads.device
        self.grad_shard = torch.zeros(off, dtype=arena.grads.dtype, device=dev)
        self.param_shard = torch.zeros(off, dtype=arena.params.dtype, device=dev)
        flags = [arena.decay_flags[a // ALIGN:(a + ln) // ALIGN] for _, a, _, ln in self.shard_ranges]
        self.decay_shard = torch.cat(flags) if flags else arena.decay_flags[:0]
        # weight all-gathers in flight (per bucket) and whether gather_params returns before
        # they complete (the forward pre-hooks of install_gather_hooks wait per bucket)
        self._pgather = [None] * len(self.buckets)
        self.overlap_gather = os.environ.get("ORION_ZERO1_OVERLAP", "1") != "0"
        self._hooks = []
        # ORION_ZERO1_CHECK=1 (debug): the first gradient of a step asserts that the forward
        # waited for every overlapped weight gather -- an op that read weights outside the
        # module pre-hooks and the ops param guard would otherwise read last step's weights
        self.check_gathers = os.environ.get("ORION_ZERO1_CHECK") == "1"

    # the fused AdamW (train/optim.py) takes this object as its "arena": flat params (the
    # bf16 shard it writes), grads (the reduced fp32 shard), decay flags and the initial fp32
    # master (set by the trainer before the optimizer is built)
    @property
    def params(self):
        return self.param_shard

    @property
    def grads(self):
        return self.grad_shard

    @property
    def decay_flags(self):
        return self.decay_shard

    @property
    def device(self):
        return self.grad_shard.device

    @property
    def numel(self):
        return self.shard_numel

    def shard_of(self, full: torch.Tensor) -> torch.Tensor:
        """This rank's shard (shard layout) of an arena-layout tensor."""
        return torch.cat([full[a:a + ln] for _, a, _, ln in self.shard_ranges])

    def gather_full(self, shard: torch.Tensor) -> torch.Tensor:
        """Arena-layout tensor assembled from every rank's shard (all-gather per bucket)."""
        full = torch.zeros(self.arena.numel, dtype=shard.dtype, device=shard.device)
        for bi, _, so, ln in self.shard_ranges:
            b0, b1, _ = self.buckets[bi]
            dist.all_gather_into_tensor(full[b0:b1], shard[so:so + ln].contiguous(), group=self.group)
        return full

    def gather_full_host(self, shard: torch.Tensor, keep: bool) -> torch.Tensor | None:
        """The arena-layout tensor of ``gather_full`` in HOST memory, only where ``keep``
        (the checkpoint writer): every rank joins the per-bucket all-gathers through one
        bucket-sized device buffer, the others drop each bucket at once, so a non-writing rank
        never holds the full tensor on the device or the host (Llama-7B: 27 GB per moment)."""
        full = torch.zeros(self.arena.numel, dtype=shard.dtype) if keep else None
        tmp = None
        for bi, _, so, ln in self.shard_ranges:
            b0, b1, _ = self.buckets[bi]
            if tmp is None or tmp.numel() < b1 - b0:
                tmp = torch.empty(b1 - b0, dtype=shard.dtype, device=shard.device)
            dist.all_gather_into_tensor(tmp[:b1 - b0], shard[so:so + ln].contiguous(), group=self.group)
            if keep:
                full[b0:b1].copy_(tmp[:b1 - b0])
        return full

    def _tail_collective(self, t, op):
        return dist.reduce_scatter_tensor(t.out, t.wire, op=op, group=self.group, async_op=True)

    def _on_grad(self, p):
        if self.check_gathers and self._sync and not any(self._arrived):
            pend = [bi for bi, h in enumerate(self._pgather) if h is not None]
            if pend:
                raise RuntimeError(f"ZeRO-1: the weight gathers of buckets {pend} were not waited "
                                   "for before the backward (an op read weights unguarded)")
        super()._on_grad(p)

    def _launch(self, bi):
        if self._handles[bi] is not None:
            return
        if self.launch_log is not None:
            self.launch_log.append(bi)
        b0, b1, _ = self.buckets[bi]
        _, _, so, ln = self.shard_ranges[bi]
        if self.timing:
            self._t_ready[bi] = self._mark()
        op = dist.ReduceOp.AVG if self._use_avg_op else dist.ReduceOp.SUM
        h = dist.reduce_scatter_tensor(self.grad_shard[so:so + ln], self.arena.grads[b0:b1], op=op,
                                       group=self.group, async_op=True)
        self._handles[bi] = h
        if self.timing and self._cuda:
            if self._tstream is None:
                self._tstream = torch.cuda.Stream()
            with torch.cuda.stream(self._tstream):
                h.wait()
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(self._tstream)
            self._t_done[bi] = ev
        if self._watchdog is not None:
            self._watchdog.add(self.step, bi, h, b1 - b0)

    def finish(self):
        """Launch stragglers, wait for every reduce-scatter; the rank's averaged gradient
        shard is then in ``grad_shard``."""
        if not self._sync:
            return
        # the next optimizer step rewrites the weight shard: no gather may still read it
        self.wait_params()
        if self.timing:
            self._bwd_end = self._mark()
        self._ready = [True] * len(self.buckets)
        self._flush()
        for bi, h in enumerate(self._handles):
            h.wait()
            if self.timing and not self._cuda:
                self._t_done[bi] = time.perf_counter()
        if not self._use_avg_op:
            self.grad_shard.div_(self.world)
        so_of = {bi: (so, ln) for bi, _, so, ln in self.shard_ranges}
        self._finish_tails(lambda t: self.grad_shard[so_of[t.bucket][0]:so_of[t.bucket][0] + so_of[t.bucket][1]])
        self._handles = [None] * len(self.buckets)
        self._arrived = [set() for _ in self.buckets]
        self._ready = [False] * len(self.buckets)
        self._cursor = 0
        self.step += 1

    def gather_params(self, overlap: bool | None = None):
        """All-gather the updated bf16 weight shards into the full compute arena, bucket by
        bucket, in FORWARD order (the arena is laid out in reverse module order, so the first
        layers' weights sit in the last buckets).  With ``overlap`` (default, unless
        ORION_ZERO1_OVERLAP=0) this returns at once and the forward pre-hooks installed by
        ``install_gather_hooks`` wait only for the buckets that hold each module's weights:
        the gathers of the later layers run under the forward of the earlier ones instead of
        ahead of the whole forward (at N = 8 that is 13.5 GB x 7/8 of bf16
        Llama-7B weights per step).  Without hooks, or with ``overlap=False``, every gather
        is waited for here."""
        if overlap is None:
            overlap = self.overlap_gather and bool(self._hooks)
        self.wait_params()
        for bi, _, so, ln in reversed(self.shard_ranges):
            b0, b1, _ = self.buckets[bi]
            self._pgather[bi] = dist.all_gather_into_tensor(
                self.arena.params[b0:b1], self.param_shard[so:so + ln], group=self.group, async_op=True)
        if not overlap:
            self.wait_params()

    def wait_params(self, buckets=None):
        """Order the current stream after the weight gathers of ``buckets`` (all by default);
        on a CPU (gloo) group this blocks until they are done."""
        for bi in (range(len(self._pgather)) if buckets is None else buckets):
            h = self._pgather[bi]
            if h is not None:
                h.wait()
                self._pgather[bi] = None

    def install_gather_hooks(self, model: torch.nn.Module):
        """Where the overlapped weight gathers are waited for: a forward pre-hook on every
        module that owns parameters (layers used through their own forward) and a guard
        called by every weight-taking fused op in ``orion_amd.ops`` (the models' top-level
        forwards hand one op the weights of several modules), each waiting only for the
        buckets that hold the weights it is about to read.  The optimizer step
        (``finish``) and the checkpoint gathers wait for everything themselves (AdamW
        rewrites the shard a gather may still be reading)."""
        slot_of = {id(s.param): s for s in self.arena.slots}
        self._bucket_starts = [b0 for b0, _, _ in self.buckets]
        bucket = self._bucket_of
        # fused ops read weights of other modules from the model's top-level forward: they
        # call the guard with their tensor arguments (ops.add_param_guard; held weakly)
        from .. import ops
        self._remove_guard = ops.add_param_guard(self._param_guard)

        for mod in model.modules():
            bs = set()
            for p in mod.parameters(recurse=False):
                sl = slot_of.get(id(p))
                if sl is None:
                    continue
                bs.update(range(bucket(sl.offset), bucket(sl.offset + max(sl.numel, 1) - 1) + 1))
            if bs:
                need = sorted(bs)
                self._hooks.append(mod.register_forward_pre_hook(
                    lambda _m, _a, need=need: self.wait_params(need)))

    def _bucket_of(self, off):
        """Index of the bucket holding arena element ``off`` (last start <= off)."""
        starts = self._bucket_starts
        lo, hi = 0, len(starts) - 1
        while lo < hi:
            mid = (lo + hi + 1) // 2
            if starts[mid] <= off:
                lo = mid
            else:
                hi = mid - 1
        return lo

    def _param_guard(self, ts):
        """Wait for the weight gathers of the buckets that the tensors ``ts`` (views of the
        compute arena, any other tensor is ignored) live in."""
        if not any(h is not None for h in self._pgather):
            return
        prm = self.arena.params
        base, esize = prm.data_ptr(), prm.element_size()
        end = base + prm.numel() * esize
        need = set()
        for t in ts:
            p0 = t.data_ptr()
            if base <= p0 < end:
                o0 = (p0 - base) // esize
                need.update(range(self._bucket_of(o0), self._bucket_of(o0 + max(t.numel(), 1) - 1) + 1))
        if need:
            self.wait_params(sorted(need))

    def reduce_sumsq(self, sumsq: torch.Tensor):
        """Global squared gradient norm from the shards' partial sums (gradient clipping)."""
        dist.all_reduce(sumsq, op=dist.ReduceOp.SUM, group=self.group)


def zero1_pad_names(model, bucket_mb: float | None, grad_dtype, world: int):
    """(names after which the arena pads to world x ALIGN, pad_to) for a ZeRO-1 layout whose
    buckets are exactly the reducer's (the plan is a pure function of the slot sizes)."""
    from ..train.flat import ALIGN, arena_order
    named, uses = arena_order(model)
    n_params = sum(p.numel() for _, p in named)
    if bucket_mb is None or bucket_mb <= 0:
        bucket_mb = default_bucket_mb(n_params)
    esize = torch.empty((), dtype=grad_dtype).element_size()
    plan = plan_buckets([(n, p.numel(), uses.get(id(p), 1) > 1) for n, p in named], bucket_mb, esize)
    return {named[idx[-1]][0] for idx in plan}, world * ALIGN


def all_reduce_scalar(t: torch.Tensor, op="mean", group=None):
    """R3: scalar all-reduce for logging (loss, token counts)."""
    if not (dist.is_available() and dist.is_initialized()):
        return t
    t = t.clone()
    if op == "max":
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        if op == "mean":
            t /= dist.get_world_size(group)
    return t
