"""Node-local GPU slot pool for concurrent trials (MI355X addition).

A node runs several workers; each trial that needs GPUs leases ``k`` device
ids through exclusive ``flock`` locks on per-device files, so independent
worker *processes* never place two trials on one GPU.  The lease is exported
to the trial as ``HIP_VISIBLE_DEVICES`` (and ``CUDA_VISIBLE_DEVICES``/
``ROCR_VISIBLE_DEVICES`` left untouched).  Locks die with the process, so a
crashed worker cannot leak a GPU.

The lock belongs to the open lock file, which the trial process inherits
(``Consumer`` passes ``lease.fds`` to the child): a GPU stays locked exactly as long
as some process that may be using it lives.  A worker that is SIGKILLed mid-trial
therefore does not free its GPU while its trial (or its trial's torchrun launcher)
still runs -- the reaper may re-queue the trial, but no other worker can place it,
or anything else, on that device until the orphan has exited.
"""
from __future__ import annotations

import fcntl
import os
import tempfile
import time


def visible_gpu_ids():
    """Device ids this node may hand out: $ORION_GPUS, else $HIP_VISIBLE_DEVICES, else
    every device torch reports (device_count does not initialise the GPU runtime)."""
    for var in ("ORION_GPUS", "HIP_VISIBLE_DEVICES"):
        val = os.environ.get(var)
        if val:
            return [v.strip() for v in val.split(",") if v.strip()]
    try:
        import torch
        return [str(i) for i in range(torch.cuda.device_count())]
    except Exception:
        return []


class GPULease:
    def __init__(self, ids, fds):
        self.ids = ids
        self._fds = fds

    @property
    def fds(self):
        """The open lock files (to hand to the trial process: ``Popen(pass_fds=...)``)."""
        return tuple(self._fds)

    def env(self):
        return {"HIP_VISIBLE_DEVICES": ",".join(self.ids)} if self.ids else {}

    def release(self):
        for fd in self._fds:
            try:
                fcntl.flock(fd, fcntl.LOCK_UN)
            finally:
                os.close(fd)
        self._fds = []

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.release()


class GPUSlotPool:
    def __init__(self, gpu_ids=None, lock_dir=None):
        self.gpu_ids = list(gpu_ids) if gpu_ids is not None else visible_gpu_ids()
        self.lock_dir = lock_dir or os.path.join(tempfile.gettempdir(), "orion_amd_gpu_slots")
        os.makedirs(self.lock_dir, exist_ok=True)

    def try_acquire(self, k):
        if k <= 0:
            return GPULease([], [])
        got, fds = [], []
        for gid in self.gpu_ids:
            fd = os.open(os.path.join(self.lock_dir, f"gpu{gid}.lock"), os.O_CREAT | os.O_RDWR, 0o666)
            try:
                fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
            except OSError:
                os.close(fd)
                continue
            got.append(gid)
            fds.append(fd)
            if len(got) == k:
                return GPULease(got, fds)
        GPULease(got, fds).release()
        return None

    def acquire(self, k, timeout=None, poll=0.5):
        if k > len(self.gpu_ids):
            raise RuntimeError(f"trial needs {k} GPUs but only {len(self.gpu_ids)} are visible")
        t0 = time.monotonic()
        while True:
            lease = self.try_acquire(k)
            if lease is not None:
                return lease
            if timeout is not None and time.monotonic() - t0 > timeout:
                raise TimeoutError(f"no {k} free GPU(s) within {timeout}s")
            time.sleep(poll)
