"""Lifecycle of a self-launched multi-rank job (orion_amd/parallel/launch.py) on the CPU:
a signal or a hard kill of the launcher must not leave ranks behind (they would hold GPUs on
the 8-GPU node), and a collective that never completes must end the job with a message that
names the stuck bucket.  Reference counterpart: the multi-worker invariants of
tests/functional/demo/test_demo.py:60-100 (every process of the job accounted for)."""
import os
import signal
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _clean_env():
    env = {k: v for k, v in os.environ.items() if k not in
           ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return env


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    # a zombie is dead for our purposes
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split()[2] != "Z"
    except OSError:
        return False


def _start_job(tmp_path, world=2):
    """A launcher whose ranks write their pid to a file and then sleep forever."""
    rank_script = tmp_path / "rank.py"
    rank_script.write_text(textwrap.dedent(f"""
        import os, time
        open(os.path.join({str(tmp_path)!r}, "rank%s.pid" % os.environ["RANK"]), "w").write(str(os.getpid()))
        time.sleep(600)
    """))
    launcher = tmp_path / "launcher.py"
    launcher.write_text(textwrap.dedent(f"""
        import sys
        from orion_amd.parallel.launch import spawn_ranks
        sys.exit(spawn_ranks({world}, [{str(rank_script)!r}], grace=5))
    """))
    p = subprocess.Popen([sys.executable, str(launcher)], env=_clean_env(), cwd=ROOT,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    deadline = time.monotonic() + 60
    pids = []
    while time.monotonic() < deadline:
        files = [tmp_path / f"rank{r}.pid" for r in range(world)]
        if all(f.exists() and f.read_text() for f in files):
            pids = [int(f.read_text()) for f in files]
            break
        time.sleep(0.1)
    assert len(pids) == world, "ranks did not start"
    return p, pids


def _wait_gone(pids, timeout=15.0):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if not any(_alive(pid) for pid in pids):
            return True
        time.sleep(0.1)
    return False


@pytest.mark.parametrize("sig", [signal.SIGTERM, signal.SIGINT])
def test_signal_to_launcher_terminates_every_rank(tmp_path, sig):
    p, pids = _start_job(tmp_path)
    p.send_signal(sig)
    rc = p.wait(timeout=30)
    assert rc == 128 + int(sig), (rc, p.stderr.read())
    assert _wait_gone(pids), f"ranks survived the launcher's {sig!r}: {pids}"


def test_sigkill_of_launcher_takes_ranks_down(tmp_path):
    """No handler runs on SIGKILL: the ranks' PR_SET_PDEATHSIG does the work."""
    p, pids = _start_job(tmp_path, world=3)
    p.kill()
    p.wait(timeout=30)
    try:
        assert _wait_gone(pids), f"ranks survived a SIGKILLed launcher: {pids}"
    finally:
        for pid in pids:
            if _alive(pid):
                os.kill(pid, signal.SIGKILL)


def test_bench_parent_killed_leaves_no_rank(tmp_path):
    """The real entry point: ``bench.py --gpus 2`` (self-spawned gloo ranks on the CPU),
    killed while its ranks are training."""
    env = _clean_env()
    env["ORION_BENCH_LOGDIR"] = str(tmp_path)
    p = subprocess.Popen([sys.executable, "bench.py", "--gpus", "2", "--model", "gpt2-tiny",
                          "--device", "cpu", "--seq-len", "64", "--micro-batch", "2",
                          "--steps", "100000", "--warmup", "1"], cwd=ROOT, env=env,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    deadline = time.monotonic() + 120
    kids = []
    while time.monotonic() < deadline and len(kids) < 2:
        try:
            out = subprocess.run(["pgrep", "-P", str(p.pid)], capture_output=True, text=True).stdout
        except FileNotFoundError:
            pytest.skip("pgrep not available")
        kids = [int(x) for x in out.split()]
        time.sleep(0.2)
    assert len(kids) == 2, "bench did not spawn its ranks"
    time.sleep(3)  # let them get into the training loop
    p.send_signal(signal.SIGTERM)
    p.wait(timeout=60)
    try:
        assert _wait_gone(kids, 30), f"bench ranks survived: {kids}"
    finally:
        for pid in kids:
            if _alive(pid):
                os.kill(pid, signal.SIGKILL)


def test_failed_rank_ends_the_job(tmp_path):
    """One rank exiting non-zero terminates the others and the launcher reports its status."""
    rank_script = tmp_path / "rank.py"
    rank_script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(7)
        time.sleep(600)
    """))
    out = subprocess.run([sys.executable, "-c",
                          f"import sys; from orion_amd.parallel.launch import spawn_ranks; "
                          f"sys.exit(spawn_ranks(2, [{str(rank_script)!r}], grace=5))"],
                         env=_clean_env(), cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert out.returncode == 7, out.stderr
    assert "rank exit codes" in out.stderr


def test_stuck_collective_names_the_bucket(tmp_path):
    """Rank 1 never joins the all-reduce: rank 0's watchdog must end it (exit 124) with a
    message naming the bucket, well before the process group's own timeout."""
    script = tmp_path / "stuck.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        import torch, torch.distributed as dist
        from orion_amd.parallel.launch import init_process_group
        from orion_amd.parallel.ddp import GradBucketReducer
        from orion_amd.train.flat import FlatArena
        from orion_amd.models.gpt2 import build_gpt2
        init_process_group("gloo")
        torch.manual_seed(0)
        arena = FlatArena(build_gpt2("gpt2-tiny", block_size=32), dtype=torch.float32)
        red = GradBucketReducer(arena, bucket_mb=0.05, watchdog_s=2.0)
        if dist.get_rank() == 1:
            time.sleep(60)
            sys.exit(0)
        red.set_sync(True)
        for s in red.buckets[0][2]:
            red._on_grad(s.param)
        time.sleep(60)
    """))
    env = _clean_env()
    env["ORION_PG_TIMEOUT_S"] = "120"
    t0 = time.monotonic()
    out = subprocess.run([sys.executable, "-c",
                          f"import sys; from orion_amd.parallel.launch import spawn_ranks; "
                          f"sys.exit(spawn_ranks(2, [{str(script)!r}], grace=5))"],
                         env=env, cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert out.returncode == 124, out.stderr[-2000:]
    assert "bucket 0" in out.stderr and "step 0" in out.stderr, out.stderr[-2000:]
    assert time.monotonic() - t0 < 60
