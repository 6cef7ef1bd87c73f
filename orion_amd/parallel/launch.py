"""Single-node rank launcher: one process per GPU, started BEFORE anything touches the GPU.

``python bench.py --gpus 8`` (no ``WORLD_SIZE`` in the environment) must produce an 8-rank
RCCL job by itself, exactly like ``torch.distributed.run --nproc-per-node 8`` would.  The
parent never initialises HIP (it does not even import torch): it picks a free rendezvous
port on 127.0.0.1, starts N children of the same command line with
``RANK/LOCAL_RANK/WORLD_SIZE/LOCAL_WORLD_SIZE/MASTER_ADDR/MASTER_PORT`` set, forwards their
output, and exits with the first non-zero child status (terminating the rest, so one
crashed rank cannot leave the others blocked inside a collective forever).

Lifecycle guarantees (a rank that outlives its job keeps a GPU busy for whoever comes next):

* a SIGTERM / SIGINT / SIGHUP delivered to the parent is forwarded to every rank's process
  group (each rank runs in a session of its own, so its helpers go with it), then the
  parent waits a grace period, SIGKILLs what is left and exits 128 + signal;
* every rank is armed with ``prctl(PR_SET_PDEATHSIG, SIGKILL)`` between fork and exec, so
  even a SIGKILLed parent (no handler runs) takes its ranks with it; a rank whose parent
  died before the ``prctl`` took effect exits at once;
* ``init_process_group`` passes a finite timeout (``ORION_PG_TIMEOUT_S``, default 600 s)
  and turns on RCCL's asynchronous error handling, so a collective that never completes
  becomes a non-zero exit instead of a hang that lasts the driver's whole budget.

Children are started with ``subprocess`` (fork+exec of a fresh interpreter), never with
``os.exec*`` from a process that has initialised the GPU.
"""
from __future__ import annotations

import ctypes
import datetime
import os
import signal
import socket
import subprocess
import sys
import time

ENV_KEYS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
PR_SET_PDEATHSIG = 1
_FORWARDED = (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)


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


def _die_with_parent(parent_pid: int):
    """preexec_fn of a rank (runs in the child between fork and exec): the kernel sends
    SIGKILL to the child when the parent exits, whatever way it exits."""
    def arm():
        try:
            libc = ctypes.CDLL(None, use_errno=True)
            libc.prctl(PR_SET_PDEATHSIG, int(signal.SIGKILL), 0, 0, 0)
        except OSError:
            pass
        if os.getppid() != parent_pid:  # the parent died before the prctl: follow it now
            os._exit(1)
    return arm


def _terminate(procs, grace: float = 20.0, sig=signal.SIGTERM):
    """Signal every live rank's process group, wait up to ``grace`` s, then SIGKILL."""
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, sig)
            except (ProcessLookupError, PermissionError):
                pass
    deadline = time.monotonic() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()


class _Signalled(Exception):
    def __init__(self, signum):
        super().__init__(signum)
        self.signum = signum


def spawn_ranks(world: int, argv: list[str] | None = None, poll: float = 0.2,
                timeout: float | None = None, grace: float = 20.0) -> int:
    """Run ``[python] + argv`` as ``world`` ranks on this node; returns the job's exit code."""
    argv = list(sys.argv if argv is None else argv)
    port = free_port()
    procs: list[subprocess.Popen] = []

    fired = []

    def on_signal(signum, _frame):
        if fired:  # already shutting down: a repeated signal must not abort the clean-up
            return
        fired.append(signum)
        raise _Signalled(signum)

    previous = {s: signal.signal(s, on_signal) for s in _FORWARDED}
    rc = 0
    try:
        me = os.getpid()
        for r in range(world):
            procs.append(subprocess.Popen([sys.executable] + argv, env=rank_env(r, world, port),
                                          start_new_session=True,
                                          preexec_fn=_die_with_parent(me)))
        t0 = time.monotonic()
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
    except _Signalled as e:
        rc = 128 + int(e.signum)
        print(f"[orion_amd.launch] signal {int(e.signum)}: terminating {len(procs)} rank(s)",
              file=sys.stderr, flush=True)
        # forward the signal itself first (ranks exit through their own handlers)
        _terminate(procs, grace, sig=e.signum if e.signum != signal.SIGHUP else signal.SIGTERM)
    finally:
        if rc != 0:
            _terminate(procs, grace)
        for s, h in previous.items():
            signal.signal(s, h)
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


def pg_timeout() -> datetime.timedelta:
    """Collective timeout of every process group this package creates."""
    return datetime.timedelta(seconds=float(os.environ.get("ORION_PG_TIMEOUT_S", "600")))


def rccl_debug_env(log_dir: str, rank: int) -> str:
    """Route RCCL's INFO log (topology, rings/trees, channels) of this rank to a file before
    the communicator exists; returns the file's path.  Leaves a user's own NCCL_DEBUG alone."""
    try:
        os.makedirs(log_dir, exist_ok=True)
    except OSError:  # read-only tree: the log goes to the temp dir instead of failing the job
        import tempfile
        log_dir = os.path.join(tempfile.gettempdir(), "orion_rccl_logs")
        os.makedirs(log_dir, exist_ok=True)
    path = os.path.join(log_dir, f"rccl_rank{rank}.log")
    if "NCCL_DEBUG" not in os.environ:
        os.environ["NCCL_DEBUG"] = "INFO"
        os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,GRAPH,TUNING")
        os.environ["NCCL_DEBUG_FILE"] = path
    return os.environ.get("NCCL_DEBUG_FILE", path)


def init_process_group(backend: str, dev=None):
    """``torch.distributed`` init for a rank, with a finite collective timeout.  RCCL
    (``nccl``): eager communicator setup on this rank's device, asynchronous error handling
    (a timed-out collective tears the process down with a non-zero status), and collectives
    on a HIGH-priority HIP stream, so a bucket's all-reduce is dispatched ahead of the
    backward GEMM workgroups queued on the compute stream instead of behind them (the
    overlap the bucketed reducer relies on).  ``ORION_RCCL_HIGH_PRIO=0`` keeps the
    default-priority stream."""
    import torch.distributed as dist
    timeout = pg_timeout()
    if backend != "nccl":
        dist.init_process_group(backend, timeout=timeout)
        return
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    opts = None
    if os.environ.get("ORION_RCCL_HIGH_PRIO", "1") != "0":
        try:
            from torch.distributed import ProcessGroupNCCL
            opts = ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
        except (ImportError, AttributeError):
            opts = None
    dist.init_process_group("nccl", device_id=dev, pg_options=opts, timeout=timeout)
