"""Build the in-tree HIP extension ``orion_amd/_C.so`` with hipcc (gfx950).

No hipify, no JIT cache, no setuptools magic: every ``csrc/*.hip`` kernel file
is compiled by ``hipcc --offload-arch=gfx950`` into an object with no torch
headers (fast, pure kernel code), the host sources ``csrc/*.cpp`` (the op
bindings, the hipBLASLt wrapper) are compiled against the torch headers, and
everything is linked into one shared object that
registers ``torch.ops.orion_amd.*`` on load.  Objects are rebuilt only when a
source or header is newer than the object.

Usage: ``python -m orion_amd.build [-j N] [--force] [--verbose]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shlex
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.environ.get("ORION_AMD_CSRC", os.path.join(ROOT, "csrc"))
# ORION_AMD_DEBUG=1: -O1 -g with device-side bounds asserts on the global indices of the
# hand-written kernels (ORION_DASSERT in csrc/common.h), built beside the release library
# as orion_amd/_C_debug.so; load it with ORION_AMD_EXT=orion_amd/_C_debug.so.
DEBUG = os.environ.get("ORION_AMD_DEBUG") == "1"
_SUFFIX = "_debug" if DEBUG else ""
BUILD = os.environ.get("ORION_AMD_BUILD_DIR", os.path.join(ROOT, "build", "csrc" + _SUFFIX))
OUT = os.environ.get("ORION_AMD_EXT", os.path.join(ROOT, "orion_amd", f"_C{_SUFFIX}.so"))
ARCH = os.environ.get("ORION_AMD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return ce.include_paths(), ce.library_paths(), abi


# per-source extra flags (see the comment at the top of each file)
FILE_FLAGS = {"attn_fwd.hip": ["-fno-honor-nans", "-fno-slp-vectorize"],
              "attn_bwd_split.hip": ["-fno-honor-nans", "-fno-slp-vectorize"],
              "xent.hip": ["-fno-honor-nans", "-fno-slp-vectorize"]}


def _newest_header():
    hs = glob.glob(os.path.join(CSRC, "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build(jobs: int | None = None, force: bool = False, verbose: bool = False) -> str:
    incs, libdirs, abi = _torch_paths()
    os.makedirs(BUILD, exist_ok=True)
    hdr_time = _newest_header()
    opt = ["-O1", "-g", "-DORION_DEBUG=1"] if DEBUG else ["-O3"]
    common = [*opt, "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              "-Wno-unused-result", "-Wno-unused-command-line-argument", f"-I{CSRC}"]
    kern = [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
            *common]
    py_inc = sysconfig.get_paths()["include"]
    bind = [HIPCC, *common, *[f"-I{i}" for i in incs], f"-I{py_inc}",
            "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    jobs_list = []
    objs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))) + sorted(glob.glob(os.path.join(CSRC, "*.cpp"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        base = bind if src.endswith(".cpp") else kern
        name = os.path.basename(src)
        extra = FILE_FLAGS.get(name, [])
        # A/B builds: ORION_AMD_FLAGS_<STEM> (e.g. ORION_AMD_FLAGS_XENT) adds flags to one
        # source; ORION_AMD_ATTN_FLAGS to both attention sources
        extra = extra + os.environ.get("ORION_AMD_FLAGS_" + name.split(".")[0].upper(), "").split()
        if name.startswith("attn_"):
            extra = extra + os.environ.get("ORION_AMD_ATTN_FLAGS", "").split()
        cmd = base + extra + ["-c", src, "-o", obj]
        # the effective command is part of the staleness check: an object built with A/B
        # flags is rebuilt by the next default build (and vice versa), not kept by mtime
        stamp = obj + ".cmd"
        sig = hashlib.sha256("\0".join(cmd).encode()).hexdigest()
        same_cmd = os.path.exists(stamp) and open(stamp).read().strip() == sig
        stale = force or not same_cmd or not os.path.exists(obj) or \
            os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_time)
        if stale:
            if os.path.exists(stamp):
                os.remove(stamp)
            jobs_list.append((cmd, stamp, sig))
    jobs = jobs or min(8, os.cpu_count() or 4)
    if jobs_list:
        with cf.ThreadPoolExecutor(jobs) as ex:
            futs = [ex.submit(_run, c, verbose) for c, _, _ in jobs_list]
            for f in futs:
                f.result()
        for _, stamp, sig in jobs_list:
            with open(stamp, "w") as fh:
                fh.write(sig + "\n")
    newest_obj = max(os.path.getmtime(o) for o in objs)
    if force or jobs_list or not os.path.exists(OUT) or os.path.getmtime(OUT) < newest_obj:
        tlib = libdirs[0]
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", OUT + ".tmp",
                # hipBLASLt: the copy torch ships and loads (csrc/blaslt.cpp)
                f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lhipblaslt",
                f"-Wl,-rpath,{tlib}"]
        _run(link, verbose)
        os.replace(OUT + ".tmp", OUT)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    out = build(a.jobs, a.force, a.verbose)
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
