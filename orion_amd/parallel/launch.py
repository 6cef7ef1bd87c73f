"""Single-node rank launcher: one process per GPU, started BEFORE anything touches the GPU.

``python bench.py --gpus 8`` (no ``WORLD_SIZE`` in the environment) must produce an 8-rank
RCCL job by itself, exactly like ``torch.distributed.run --nproc-per-node 8`` would.  The
parent never initialises HIP (it does not even import torch): it picks a free rendezvous
port on 127.0.0.1, starts N children of the same command line with
``RANK/LOCAL_RANK/WORLD_SIZE/LOCAL_WORLD_SIZE/MASTER_ADDR/MASTER_PORT`` set, forwards their
output, and exits with the first non-zero child status (terminating the rest, so one
crashed rank cannot leave the others blocked inside a collective forever).

Children are started with ``subprocess`` (fork+exec of a fresh interpreter), never with
``os.exec*`` from a process that has initialised the GPU.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time

ENV_KEYS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def in_launched_job() -> bool:
    """True when this process is a rank of an already-launched job (torchrun or us)."""
    return "WORLD_SIZE" in os.environ


def rank_env(rank: int, world: int, port: int, base: dict | None = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # dmabuf IPC is the only one the host driver supports (RCCL peer mappings)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn_ranks(world: int, argv: list[str] | None = None, poll: float = 0.2,
                timeout: float | None = None) -> int:
    """Run ``[python] + argv`` as ``world`` ranks on this node; returns the job's exit code."""
    argv = list(sys.argv if argv is None else argv)
    port = free_port()
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen([sys.executable] + argv, env=rank_env(r, world, port),
                                      start_new_session=True))
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            states = [p.poll() for p in procs]
            bad = [s for s in states if s not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(s == 0 for s in states):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                rc = 124
                break
            time.sleep(poll)
    finally:
        if rc != 0:
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
            deadline = time.monotonic() + 20
            for p in procs:
                try:
                    p.wait(timeout=max(0.1, deadline - time.monotonic()))
                except subprocess.TimeoutExpired:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
                    p.wait()
    if rc != 0:
        print(f"[orion_amd.launch] job failed: rank exit codes {[p.returncode for p in procs]}",
              file=sys.stderr, flush=True)
    return rc if rc >= 0 else 128 - rc


def check_world(expected: int) -> tuple[int, int, int]:
    """(world, rank, local_rank) of this process; raises if the job's size is not ``expected``."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != expected:
        raise SystemExit(f"--gpus {expected} but the launched job has WORLD_SIZE={world}")
    return world, rank, local_rank


def device_for(local_rank: int, local_world: int, backend: str):
    """The HIP device of this rank.  RCCL needs one rank per device: fail loudly if the node
    shows fewer devices than ranks instead of silently doubling ranks up on a GPU."""
    import torch
    n = torch.cuda.device_count()
    if backend == "nccl":
        if n < local_world:
            raise SystemExit(f"{local_world} RCCL ranks on this node but only {n} visible GPU(s)")
        return torch.device("cuda", local_rank)
    # gloo rehearsal: ranks may share a device (or run on the CPU)
    return torch.device("cuda", local_rank % n) if n else torch.device("cpu")


def init_process_group(backend: str, dev=None):
    """``torch.distributed`` init for a rank.  RCCL (``nccl``): eager communicator setup on
    this rank's device, and collectives on a HIGH-priority HIP stream, so a bucket's
    all-reduce is dispatched ahead of the backward GEMM workgroups queued on the compute
    stream instead of behind them (the overlap the bucketed reducer relies on).
    ``ORION_RCCL_HIGH_PRIO=0`` keeps the default-priority stream."""
    import torch.distributed as dist
    if backend != "nccl":
        dist.init_process_group(backend)
        return
    opts = None
    if os.environ.get("ORION_RCCL_HIGH_PRIO", "1") != "0":
        try:
            from torch.distributed import ProcessGroupNCCL
            opts = ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
        except (ImportError, AttributeError):
            opts = None
    dist.init_process_group("nccl", device_id=dev, pg_options=opts)
