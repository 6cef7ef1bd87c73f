"""The bench.py contract the round driver relies on: one JSON line from rank 0 with the
whole-job throughput, for N=1 and (rehearsed with gloo, both ranks on the one GPU of the
test box) N=2 launched by torch.distributed.run."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _check(rec, n, steps, warmup, mb):
    assert KEYS <= set(rec), KEYS - set(rec)
    assert rec["n_gpus"] == n and rec["steps"] == steps and rec["warmup"] == warmup
    assert rec["dtype"] == "bf16" and rec["scaling"] == "weak" and rec["higher_is_better"] is True
    cfg = rec["config"]
    assert cfg["seq_len"] == 1024 and cfg["global_batch"] == mb * n and cfg["parallelism"] == f"dp{n}"
    # value is the whole-job token rate, consistent with ms_per_step
    tok = mb * 1024 * n
    assert abs(rec["value"] - tok / (rec["ms_per_step"] / 1000)) / rec["value"] < 0.01
    assert rec["loss"] == rec["loss"] and 9.0 < rec["loss"] < 12.5


def test_bench_single_gpu_contract():
    out = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--micro-batch", "4"],
                         cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    _check(_json_line(out.stdout), 1, 2, 1, 4)


def test_bench_two_ranks_gloo_rehearsal():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--micro-batch", "4", "--dist-backend", "gloo"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    _check(_json_line(out.stdout), 2, 2, 1, 4)


def test_bench_self_spawns_two_ranks():
    """No launcher: ``bench.py --gpus 2`` starts its own two ranks (gloo, sharing the one GPU
    of the test box -- RCCL refuses two ranks on one device, and device_for says so)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "--micro-batch", "4", "--dist-backend", "gloo"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    _check(_json_line(out.stdout), 2, 2, 1, 4)
