"""Fork server for trial processes (``--trial-runner fork``).

A short GPU trial of a Python black box spends most of its wall time starting up: the
interpreter, ``import torch`` and the extension's imports took ~4 s of each 4.5 s GPT-2-tiny
trial on the MI355X box (docs/PERFORMANCE.md, HPO section).  The reference forks nothing --
every trial is a fresh ``subprocess`` (``src/orion/core/worker/consumer.py:118-130``) -- and
so does the default runner here.  With the fork server, each worker starts ONE helper
process that imports the heavy modules once (``torch`` and the ``orion_amd`` Python
package; nothing that initialises the GPU, so every trial still brings up its own HIP
context) and then forks a fresh child per trial that runs the script with ``runpy`` as
``__main__``.

The child looks to the consumer like a ``subprocess.Popen``: its own session (so
``killpg`` reaches everything it starts), the trial's environment, working directory and
argv, the GPU lease's lock descriptors (sent over the socket with ``SCM_RIGHTS``, so the
lease stays held exactly as long as the trial lives), ``PR_SET_PDEATHSIG`` chained through
the server (worker dies -> server gets SIGTERM -> trial gets SIGTERM), and an exit status
(``SystemExit`` codes, 1 on an uncaught exception, -signal when killed) reported back over
the socket.

Protocol (one AF_UNIX stream socket, JSON lines): request ``{"argv": [...], "env": {...},
"cwd": str}`` with the lease fds as ancillary data -> reply ``{"pid": n}`` or ``{"error": msg}``;
asynchronous ``{"exit": pid, "rc": code}`` when a child ends.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

DEFAULT_PRELOAD = ("torch", "numpy", "orion_amd", "orion_amd.models", "orion_amd.train")


def _pdeathsig(sig=signal.SIGTERM):
    try:
        import ctypes
        ctypes.CDLL(None, use_errno=True).prctl(1, int(sig), 0, 0, 0)  # PR_SET_PDEATHSIG
    except OSError:
        pass


# ----------------------------------------------------------------------------- server side
def _run_child(argv, env, cwd, fds):
    """In the forked child: become the trial process, run the script, never return."""
    code = 1
    try:
        os.setsid()
        _pdeathsig()
        for s in (signal.SIGINT, signal.SIGTERM, signal.SIGCHLD):
            signal.signal(s, signal.SIG_DFL)
        os.environ.clear()
        os.environ.update(env)
        os.chdir(cwd)
        sys.argv = list(argv)
        script = argv[0]
        sys.path[0] = os.path.dirname(os.path.abspath(script))
        import runpy
        try:
            runpy.run_path(script, run_name="__main__")
            code = 0
        except SystemExit as e:
            c = e.code
            code = 0 if c is None else (c if isinstance(c, int) else 1)
            if not isinstance(c, (int, type(None))):
                print(c, file=sys.stderr)
        except BaseException:  # noqa: BLE001 - the trial's own failure, reported as rc 1
            import traceback
            traceback.print_exc()
            code = 1
    finally:
        try:
            _interpreter_shutdown()
            sys.stdout.flush()
            sys.stderr.flush()
        finally:
            os._exit(code & 0xFF)  # ``fds`` (the lease's lock descriptors) stay open until here


def _interpreter_shutdown():
    """What a normal interpreter exit does before the process ends, which ``os._exit`` alone
    skips: join the non-daemon threads the script started, then run the ``atexit`` handlers
    (logging.shutdown, result writers, tracker flushes) -- so a forked trial keeps the
    ``Popen`` contract of an exec'd one."""
    import atexit
    import threading
    try:
        threading._shutdown()  # the interpreter's own join of non-daemon threads
    except BaseException:  # noqa: BLE001 - a failing thread join must not skip the atexit handlers
        import traceback
        traceback.print_exc()
    atexit._run_exitfuncs()  # prints (does not raise) a handler's exception, as at exit


def serve(sock: socket.socket, preload=DEFAULT_PRELOAD):
    """Server loop: preload, then fork one child per request until the socket closes."""
    _pdeathsig()
    for mod in preload:
        try:
            __import__(mod)
        except Exception as exc:  # noqa: BLE001 - a missing optional module only costs speed
            print(f"[orion forkserver] preload {mod} failed: {exc}", file=sys.stderr, flush=True)

    # forking a process whose HIP runtime is up is not supported: the preload must not touch
    # the GPU (torch.cuda.is_available() would); refuse to fork if something did
    torch = sys.modules.get("torch")
    gpu_up = bool(torch is not None and torch.cuda.is_initialized())

    def send(msg):
        sock.sendall((json.dumps(msg) + "\n").encode())

    def reap():
        # polled from the loop (a SIGCHLD handler that writes to the socket could interrupt
        # a send in progress); SIGCHLD stays SIG_DFL so exited children wait to be reaped
        while True:
            try:
                pid, status = os.waitpid(-1, os.WNOHANG)
            except ChildProcessError:
                return
            if pid == 0:
                return
            rc = -os.WTERMSIG(status) if os.WIFSIGNALED(status) else os.WEXITSTATUS(status)
            send({"exit": pid, "rc": rc})

    import select
    buf = b""
    fds: list = []  # descriptors received since the last complete request line
    while True:
        reap()
        if not select.select([sock], [], [], 0.05)[0]:
            continue
        data, new_fds, _, _ = socket.recv_fds(sock, 1 << 16, 16)
        if not data:
            for fd in fds + list(new_fds):
                os.close(fd)
            break  # the worker closed the socket (or died): children get SIGTERM via PDEATHSIG
        # a request longer than one recv (a big environment) brings its descriptors with its
        # FIRST chunk: keep them until the newline that completes the request arrives
        fds += list(new_fds)
        buf += data
        while b"\n" in buf:
            line, buf = buf.split(b"\n", 1)
            try:
                req = json.loads(line)
                req = dict(argv=list(req["argv"]), env=dict(req["env"]), cwd=str(req["cwd"]))
            except (ValueError, KeyError, TypeError) as exc:
                req = None
                err = f"malformed request: {exc}"
            if gpu_up or req is None:
                send({"error": err if req is None else "the GPU was initialised in the fork server; not forking"})
                for fd in fds:
                    os.close(fd)
                fds = []
                continue
            try:
                pid = os.fork()
            except OSError as exc:
                send({"error": str(exc)})
                for fd in fds:
                    os.close(fd)
                fds = []
                continue
            if pid == 0:
                sock.close()
                _run_child(req["argv"], req["env"], req["cwd"], fds)
            for fd in fds:
                os.close(fd)
            fds = []
            send({"pid": pid})


# ----------------------------------------------------------------------------- client side
class ForkedTrial:
    """``subprocess.Popen``-like handle of a trial forked by :class:`ForkServer`."""

    def __init__(self, server: "ForkServer", pid: int):
        self._server = server
        self.pid = pid
        self.returncode = None

    def poll(self):
        if self.returncode is None:
            self.returncode = self._server._exits.get(self.pid)
        return self.returncode

    def wait(self, timeout=None):
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._server._cv:
            while self.pid not in self._server._exits:
                if not self._server._alive:
                    self.returncode = -signal.SIGKILL
                    return self.returncode
                left = None if deadline is None else deadline - time.monotonic()
                if left is not None and left <= 0:
                    raise subprocess.TimeoutExpired(f"forked trial {self.pid}", timeout)
                self._server._cv.wait(left)
            self.returncode = self._server._exits[self.pid]
        return self.returncode


class ForkServer:
    """One per worker process; ``spawn`` is the fork-server analogue of ``Popen``."""

    def __init__(self, preload=DEFAULT_PRELOAD, python=sys.executable):
        parent, child = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
        env = dict(os.environ)
        env["ORION_FORKSERVER_FD"] = str(child.fileno())
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = os.pathsep.join(p for p in (root, env.get("PYTHONPATH")) if p)
        self.proc = subprocess.Popen([python, "-m", "orion_amd.core.forkserver", ",".join(preload)],
                                     env=env, pass_fds=(child.fileno(),), start_new_session=True)
        child.close()
        self._sock = parent
        self._cv = threading.Condition()
        self._exits: dict[int, int] = {}
        self._replies: list = []
        self._alive = True
        self._reader = threading.Thread(target=self._read, daemon=True)
        self._reader.start()
        self._spawn_lock = threading.Lock()

    def _read(self):
        buf = b""
        try:
            while True:
                data = self._sock.recv(1 << 16)
                if not data:
                    break
                buf += data
                while b"\n" in buf:
                    line, buf = buf.split(b"\n", 1)
                    msg = json.loads(line)
                    with self._cv:
                        if "exit" in msg:
                            self._exits[int(msg["exit"])] = int(msg["rc"])
                        else:
                            self._replies.append(msg)
                        self._cv.notify_all()
        except OSError:
            pass
        with self._cv:
            self._alive = False
            self._cv.notify_all()

    def spawn(self, argv, env, cwd=None, pass_fds=()) -> ForkedTrial:
        req = (json.dumps({"argv": list(argv), "env": dict(env), "cwd": cwd or os.getcwd()}) + "\n").encode()
        with self._spawn_lock:
            socket.send_fds(self._sock, [req], list(pass_fds))
            with self._cv:
                while not self._replies:
                    if not self._alive:
                        raise OSError("trial fork server exited")
                    self._cv.wait(30.0)
                msg = self._replies.pop(0)
        if "error" in msg:
            raise OSError(msg["error"])
        return ForkedTrial(self, int(msg["pid"]))

    def close(self):
        try:
            self._sock.close()
        finally:
            try:
                self.proc.terminate()
                self.proc.wait(timeout=10)
            except (subprocess.TimeoutExpired, OSError):
                self.proc.kill()


if __name__ == "__main__":
    _fd = int(os.environ.pop("ORION_FORKSERVER_FD"))
    _mods = tuple(m for m in (sys.argv[1] if len(sys.argv) > 1 else "").split(",") if m)
    serve(socket.socket(fileno=_fd), _mods)
