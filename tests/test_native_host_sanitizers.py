"""Host-side launcher logic under ASan + UBSan (SURVEY.md §5 race detection / sanitizers):
tests/native/host_logic.cpp links the csrc/*.hip launchers compiled host-only with
``-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined`` and exercises split
planning, scratch sizing and argument rejection.  No GPU: nothing is launched."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
SOURCES = ["tests/native/host_logic.cpp", "csrc/gemm.hip", "csrc/gemm16.hip", "csrc/wgrad.hip",
           "csrc/layernorm.hip", "csrc/rmsnorm_rope.hip", "csrc/activations.hip"]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_launcher_host_logic_under_asan_ubsan(tmp_path):
    import concurrent.futures as cf
    exe = str(tmp_path / "host_logic")
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined"]

    def compile_one(src):
        obj = str(tmp_path / (os.path.basename(src) + ".o"))
        lang = ["-x", "hip", "--offload-arch=gfx950"] if src.endswith(".hip") else []
        cmd = [HIPCC, *lang, "-O1", "-g", "-std=c++17", f"-I{ROOT}/csrc", *san, "-c",
               os.path.join(ROOT, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-3000:]
        return obj

    with cf.ThreadPoolExecutor(min(6, os.cpu_count() or 2)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", *objs, "-fsanitize=address,undefined", "-o", exe],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "host logic ok" in r.stdout
