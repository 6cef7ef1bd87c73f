"""Token data for training: synthetic batches and nanoGPT ``train.bin``/``val.bin``.

``MemmapTokens`` reads nanoGPT-format shards (flat ``uint16`` token ids) through
``numpy.memmap`` and samples random ``block_size + 1`` windows; a background
thread assembles the next batches into pinned host memory and copies them to
the GPU on a side HIP stream, so the training stream never waits on the disk
or on host-to-device copies.
"""
from __future__ import annotations

import os
import queue
import threading

import numpy as np
import torch


class SyntheticTokens:
    """Random token ids of a fixed shape, pre-generated on the device (bench / plumbing)."""

    def __init__(self, vocab_size, batch_size, block_size, device, seed=0, pool=4):
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        self.pool = [(torch.randint(0, vocab_size, (batch_size, block_size), device=device, generator=g),
                      torch.randint(0, vocab_size, (batch_size, block_size), device=device, generator=g))
                     for _ in range(pool)]
        self.i = 0

    def next(self):
        b = self.pool[self.i % len(self.pool)]
        self.i += 1
        return b


class MemmapTokens:
    def __init__(self, path, batch_size, block_size, device, seed=0, prefetch=4, dtype=np.uint16):
        if not os.path.isfile(path):
            raise FileNotFoundError(path)
        self.data = np.memmap(path, dtype=dtype, mode="r")
        if len(self.data) <= block_size + 1:
            raise ValueError(f"{path}: {len(self.data)} tokens < block_size + 1")
        self.B, self.T = batch_size, block_size
        self.device = torch.device(device)
        self.rng = np.random.default_rng(seed)
        self.q = queue.Queue(maxsize=prefetch)
        self._stop = threading.Event()
        self.pin = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.pin else None
        self.thread = threading.Thread(target=self._work, daemon=True)
        self.thread.start()

    def _host_batch(self):
        ix = self.rng.integers(0, len(self.data) - self.T - 1, size=self.B)
        buf = np.stack([np.asarray(self.data[i:i + self.T + 1], dtype=np.int64) for i in ix])
        t = torch.from_numpy(buf)
        return t.pin_memory() if self.pin else t

    def _work(self):
        while not self._stop.is_set():
            host = self._host_batch()
            if self.pin:
                with torch.cuda.stream(self.stream):
                    dev = host.to(self.device, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                item = (dev, ev)
            else:
                item = (host, None)
            while not self._stop.is_set():
                try:
                    self.q.put(item, timeout=0.5)
                    break
                except queue.Full:
                    continue

    def next(self):
        t, ev = self.q.get()
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
            t.record_stream(torch.cuda.current_stream(self.device))
        return t[:, :-1], t[:, 1:]

    def close(self):
        self._stop.set()


def get_batch_source(data_dir, split, batch_size, block_size, device, vocab_size, seed=0):
    """nanoGPT layout ``<data_dir>/<split>.bin`` if present, else synthetic tokens."""
    if data_dir:
        path = os.path.join(data_dir, f"{split}.bin")
        if os.path.isfile(path):
            return MemmapTokens(path, batch_size, block_size, device, seed=seed)
    return SyntheticTokens(vocab_size, batch_size, block_size, device, seed=seed)
