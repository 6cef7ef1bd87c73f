"""RCCL all-reduce bus-bandwidth sweep (xGMI), one process per GPU.

``python -m orion_amd.parallel.busbw --gpus 8`` spawns the ranks itself
(``parallel/launch.py``) and prints one JSON line per message size with the
algorithm bandwidth (bytes / time) and the bus bandwidth
``algbw * 2 (N-1) / N`` -- the per-rank link traffic of a ring all-reduce, the
number that is comparable across N and against the 7 x ~153 GB/s xGMI links of
an MI355X.  Sizes default to 8 MB .. 1 GB (the DDP bucket range of
``parallel/ddp.py`` and beyond), fp32 and bf16.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def allreduce_busbw(buf, iters: int = 10, warmup: int = 2, group=None) -> float:
    """Median bus bandwidth (GB/s) of an in-place SUM all-reduce of ``buf`` over ``group``."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world < 2:
        return None
    cuda = buf.is_cuda

    def sync():
        if cuda:
            torch.cuda.synchronize()

    for _ in range(warmup):
        dist.all_reduce(buf, group=group)
    sync()
    times = []
    for _ in range(iters):
        dist.barrier(group=group)
        sync()
        t0 = time.perf_counter()
        dist.all_reduce(buf, group=group)
        sync()
        times.append(time.perf_counter() - t0)
    t = torch.tensor([sorted(times)[len(times) // 2]], dtype=torch.float64,
                     device=buf.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    nbytes = buf.numel() * buf.element_size()
    return round(nbytes / float(t) * 2 * (world - 1) / world / 1e9, 2)


def rccl_summary(path: str) -> dict | None:
    """Topology facts from one rank's RCCL INFO log (``launch.rccl_debug_env``): channel
    count, the first rings, the collective/p2p channel line and the RCCL version."""
    import re
    try:
        with open(path, errors="replace") as f:
            text = f.read()
    except OSError:
        return None
    chans = re.findall(r"Channel (\d+)/(\d+) :\s*([\d ]+)", text)
    out = {"log": path}
    if chans:
        out["channels"] = max(int(t) for _, t, _ in chans)
        out["rings"] = [" ".join(r.split()) for _, _, r in chans[:2]]
    m = re.search(r"(\d+) coll channels,.*", text)
    if m:
        out["coll_channels"] = m.group(0).strip()
    m = re.search(r"RCCL version[^\n]*", text) or re.search(r"NCCL version[^\n]*", text)
    if m:
        out["version"] = m.group(0).strip()
    m = re.findall(r"Trees? \[0\][^\n]*", text)
    if m:
        out["tree0"] = m[0].strip()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--sizes-mb", default="8,32,64,128,256,512,1024")
    ap.add_argument("--dtypes", default="float32,bfloat16")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--backend", default="nccl")
    args = ap.parse_args(argv)
    from orion_amd.parallel import launch
    if args.gpus > 1 and not launch.in_launched_job():
        return launch.spawn_ranks(args.gpus, ["-m", "orion_amd.parallel.busbw"] + sys.argv[1:])
    import torch
    import torch.distributed as dist
    world, rank, local_rank = launch.check_world(args.gpus)
    dev = launch.device_for(local_rank, int(os.environ.get("LOCAL_WORLD_SIZE", world)), args.backend)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    launch.init_process_group(args.backend, dev if args.backend == "nccl" else None)
    for dt in args.dtypes.split(","):
        dtype = getattr(torch, dt)
        for mb in (float(x) for x in args.sizes_mb.split(",")):
            n = int(mb * 2**20) // torch.empty((), dtype=dtype).element_size()
            buf = torch.ones(n, dtype=dtype, device=dev)
            bw = allreduce_busbw(buf, iters=args.iters)
            if rank == 0:
                print(json.dumps({"op": "all_reduce", "dtype": dt, "size_mb": mb, "n_gpus": world,
                                  "backend": args.backend, "busbw_gbps": bw}), flush=True)
            del buf
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
