"""Consumer: runs one reserved trial of the user's black box (component C8).

Parity with ``src/orion/core/worker/consumer.py``: in a fresh temporary
directory the trial's config file (if the user passed a template) and command
line are rendered, ``METAOPT_RESULTS_PATH`` names a results file, the script is
executed as a child process, and its JSON results complete the trial; a
non-zero exit marks it ``broken``.

MI355X-node additions:

* GPU placement: with ``gpus_per_trial = k > 0`` the trial leases k devices
  from the node's :class:`~orion_amd.core.gpus.GPUSlotPool` and sees them as
  ``HIP_VISIBLE_DEVICES``; k > 1 trials of a Python script are launched through
  ``torch.distributed.run --standalone --nproc-per-node k`` (one rank per GPU,
  RCCL over xGMI);
* liveness: from reservation on -- while the trial waits for its GPU lease and
  while the child runs -- the trial's ``heartbeat`` is refreshed; if a refresh finds
  the trial no longer ``reserved`` (a reaper re-queued it because this worker
  looked dead), the child is stopped and the trial is abandoned without writing
  anything, so no trial is ever completed twice;
* the GPU lease follows the process that uses the GPUs: the child inherits the lease's
  lock files (``pass_fds``), so a SIGKILLed worker's devices stay locked while its
  orphaned trial lives, and the child gets ``PR_SET_PDEATHSIG`` (SIGTERM) so such an
  orphan is told to stop at once instead of training on for a result nobody records;
* ``trial_timeout``: the child is killed and the trial marked ``broken``;
* SIGINT/SIGTERM of the worker: the child is terminated and the trial is
  returned to the pool as ``interrupted`` (the reference had the status but
  never set it);
* a script that is not executable but ends in ``.py`` runs under the current
  interpreter (the reference required a shebang + exec bit);
* ``trial_runner="fork"``: a ``.py`` script of a one-GPU (or CPU) trial is forked from the
  worker's fork server (``core/forkserver.py``: torch and the package imported once per
  worker) instead of started as a new interpreter -- same environment, lease descriptors,
  session, death signal and exit-status contract, seconds less start-up per trial.
"""
from __future__ import annotations

import json
import logging
import os
import signal
import subprocess
import sys
import tempfile
import time

from .trial import Trial

log = logging.getLogger(__name__)


# prctl resolved once, in the parent, at import: the preexec_fn below runs in the child
# between fork and exec, where importing a module or dlopen-ing a library can deadlock on a
# lock another thread of the worker held at fork time (pymongo's monitor threads, the fork
# server's reader thread) -- so the child only makes the call
try:
    import ctypes as _ctypes
    _PRCTL = _ctypes.CDLL(None, use_errno=True).prctl
    _PRCTL.restype = _ctypes.c_int
except (OSError, AttributeError):  # pragma: no cover - no libc prctl (non-Linux)
    _PRCTL = None
_PR_SET_PDEATHSIG = 1
_SIGTERM = int(signal.SIGTERM)


def _term_with_parent(parent_pid):
    """preexec_fn of a trial process: SIGTERM when the worker dies (any way it dies)."""
    prctl = _PRCTL

    def arm():
        if prctl is not None:
            prctl(_PR_SET_PDEATHSIG, _SIGTERM, 0, 0, 0)
        if os.getppid() != parent_pid:
            os._exit(1)
    return arm


class TrialInterrupted(Exception):
    pass


class TrialLost(Exception):
    """The reservation was taken away (stale heartbeat re-queued by another worker)."""


class Consumer:
    def __init__(self, experiment, gpu_pool=None, gpus_per_trial=0, heartbeat=30.0,
                 trial_timeout=None, worker_id=None, trial_runner="exec"):
        self.experiment = experiment
        self.space = experiment.space
        if self.space is None:
            raise RuntimeError("Experiment object provided to Consumer has not yet completed "
                               "initialization.")
        self.template = experiment.template
        self.script_path = experiment.metadata["user_script"]
        self.tmp_dir = os.path.join(tempfile.gettempdir(), "orion")
        os.makedirs(self.tmp_dir, exist_ok=True)
        self.gpus_per_trial = int(gpus_per_trial or 0)
        self.gpu_pool = gpu_pool
        if self.gpus_per_trial and self.gpu_pool is None:
            from .gpus import GPUSlotPool
            self.gpu_pool = GPUSlotPool()
        self.heartbeat = float(heartbeat or 30.0)
        self.trial_timeout = trial_timeout
        self.worker_id = worker_id
        if trial_runner not in ("exec", "fork"):
            raise ValueError(f"trial_runner must be 'exec' or 'fork', not {trial_runner!r}")
        self.trial_runner = trial_runner
        self._forkserver = None
        if self._forkable():  # start it now: its imports overlap the first reservation
            try:
                from .forkserver import ForkServer
                self._forkserver = ForkServer()
            except OSError as exc:
                log.warning("fork server unavailable (%s); starting trials as new processes", exc)
                self.trial_runner = "exec"

    # ------------------------------------------------------------------ public
    def consume(self, trial):
        """Evaluate ``trial``; returns the final status string."""
        with tempfile.TemporaryDirectory(prefix=self.experiment.name + "_", dir=self.tmp_dir) as wd:
            try:
                done = self._consume(trial, wd)
            except TrialInterrupted:
                log.warning("worker interrupted: trial %s -> interrupted", trial.id)
                self.experiment.set_trial_status(trial, "interrupted", only_if="reserved")
                raise KeyboardInterrupt
            except TrialLost:
                log.warning("trial %s was re-queued while this worker held it; abandoning it",
                            trial.id)
                return "lost"
        if done is not None:
            if not self.experiment.push_completed_trial(done, only_if_reserved=True):
                log.warning("trial %s is no longer reserved by this worker; result dropped", trial.id)
                return "lost"
            return "completed"
        log.debug("### Save %s as broken.", trial)
        self.experiment.set_trial_status(trial, "broken", only_if="reserved")
        return "broken"

    # ------------------------------------------------------------------ internals
    def _consume(self, trial, workdir):
        conf = tempfile.NamedTemporaryFile(mode="w", prefix="trial_", suffix=self._conf_suffix(),
                                           dir=workdir, delete=False)
        conf.close()
        res = tempfile.NamedTemporaryFile(mode="w", prefix="results_", suffix=".log", dir=workdir,
                                          delete=False)
        res.close()
        cmd_args = self.template.render(trial, conf.name)
        self._last_beat = time.monotonic()
        lease = None
        if self.gpus_per_trial:
            lease = self._acquire_lease(trial)
        try:
            rc = self._run(res.name, cmd_args, trial, lease)
        finally:
            if lease is not None:
                lease.release()
        if rc != 0:
            log.error("Something went wrong. Check logs. Process returned with code %d !", rc)
            return None
        try:
            with open(res.name) as f:
                results = json.load(f)
        except (OSError, json.JSONDecodeError) as exc:
            log.error("trial %s produced no readable results: %s", trial.id, exc)
            return None
        if isinstance(results, dict):  # convenience: {"objective": v, ...}
            results = [dict(name=k, type="objective" if k == "objective" else "constraint", value=v)
                       for k, v in results.items()]
        trial.results = [Trial.Result(name=r["name"], type=r["type"], value=r["value"]) for r in results]
        if trial.objective is None:
            log.error("trial %s reported no objective", trial.id)
            return None
        return trial

    def _conf_suffix(self):
        cfg = self.template.config_path
        return os.path.splitext(cfg)[1] if cfg else ".conf"

    def _beat(self, trial, force=False):
        """Refresh the trial's heartbeat every ``self.heartbeat`` seconds; raise
        :class:`TrialLost` when the trial is no longer ours."""
        now = time.monotonic()
        if force or now - self._last_beat >= self.heartbeat:
            self._last_beat = now
            if not self.experiment.update_heartbeat(trial):
                raise TrialLost(trial.id)

    def _acquire_lease(self, trial, poll=0.5):
        """Wait for ``gpus_per_trial`` devices while keeping the reservation alive."""
        if self.gpus_per_trial > len(self.gpu_pool.gpu_ids):
            raise RuntimeError(f"trial needs {self.gpus_per_trial} GPUs but only "
                               f"{len(self.gpu_pool.gpu_ids)} are visible")
        while True:
            lease = self.gpu_pool.try_acquire(self.gpus_per_trial)
            if lease is not None:
                if not self.experiment.record_lease(trial, lease.ids):
                    lease.release()
                    raise TrialLost(trial.id)
                self._last_beat = time.monotonic()
                return lease
            self._beat(trial)
            time.sleep(min(poll, self.heartbeat))

    def command(self, cmd_args):
        script = self.script_path
        if os.access(script, os.X_OK) and not (self.gpus_per_trial > 1 and script.endswith(".py")):
            base = [script]
        elif script.endswith(".py"):
            base = [sys.executable, script]
        else:
            base = [script]
        if self.gpus_per_trial > 1 and script.endswith(".py"):
            base = [sys.executable, "-m", "torch.distributed.run", "--standalone",
                    "--local-addr", "127.0.0.1", f"--nproc-per-node={self.gpus_per_trial}", script]
        return base + list(cmd_args)

    def _forkable(self):
        return (self.trial_runner == "fork" and self.script_path.endswith(".py")
                and self.gpus_per_trial <= 1)

    def launch_process(self, results_filename, cmd_args, extra_env=None, pass_fds=()):
        env = dict(os.environ)
        env["METAOPT_RESULTS_PATH"] = str(results_filename)
        env["ORION_RESULTS_PATH"] = str(results_filename)
        env["ORION_EXPERIMENT_NAME"] = str(self.experiment.name)
        env.update(extra_env or {})
        if self._forkable():
            argv = [self.script_path] + list(cmd_args)
            log.debug("forking %s", argv)
            try:
                if self._forkserver is None:
                    from .forkserver import ForkServer
                    self._forkserver = ForkServer()
                return self._forkserver.spawn(argv, env, pass_fds=pass_fds)
            except OSError as exc:  # fall back to a new process for this and later trials
                log.warning("fork server unavailable (%s); starting trials as new processes", exc)
                self.trial_runner = "exec"
        cmd = self.command(cmd_args)
        log.debug("launching %s", cmd)
        try:
            return subprocess.Popen(cmd, env=env, start_new_session=True, pass_fds=tuple(pass_fds),
                                    preexec_fn=_term_with_parent(os.getpid()))
        except OSError as exc:
            log.error("Failed to execute script to evaluate trial: %s", exc)
            return None

    def close(self):
        """Stop the fork server (if one was started)."""
        if self._forkserver is not None:
            self._forkserver.close()
            self._forkserver = None

    def _run(self, results_filename, cmd_args, trial, lease):
        extra = {"ORION_TRIAL_ID": str(trial.id)}
        fds = ()
        if lease is not None:
            extra.update(lease.env())
            fds = lease.fds
        proc = self.launch_process(results_filename, cmd_args, extra, pass_fds=fds)
        if proc is None:
            return -1
        t0 = time.monotonic()
        prev = {}
        interrupted = []

        def _on_signal(signum, _frame):
            interrupted.append(signum)

        for s in (signal.SIGINT, signal.SIGTERM):
            try:
                prev[s] = signal.signal(s, _on_signal)
            except ValueError:  # not the main thread
                pass
        try:
            while True:
                try:
                    return proc.wait(timeout=min(self.heartbeat, 1.0) if interrupted == [] else 0.1)
                except subprocess.TimeoutExpired:
                    pass
                if interrupted:
                    self._kill(proc)
                    raise TrialInterrupted()
                if self.trial_timeout and time.monotonic() - t0 > self.trial_timeout:
                    log.error("trial %s exceeded its %ss timeout", trial.id, self.trial_timeout)
                    self._kill(proc)
                    return -9
                try:
                    self._beat(trial)
                except TrialLost:
                    self._kill(proc)
                    raise
        finally:
            for s, h in prev.items():
                signal.signal(s, h)

    @staticmethod
    def _kill(proc):
        try:
            os.killpg(proc.pid, signal.SIGTERM)
            proc.wait(timeout=10)
        except (subprocess.TimeoutExpired, ProcessLookupError, PermissionError):
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            proc.wait()
