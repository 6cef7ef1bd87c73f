"""Static audit of the kernels' inline-asm LDS reads (CPU only: hipcc cross-compiles gfx950).

hipcc treats an ``asm volatile("ds_read_... %0")`` statement's output as written when the
statement ends, so it may copy or read that register before the LDS data has landed -- the
hazard of cdna_hip_programming.md §5.7 item 1 (round 5 hit it in a kernel draft: a fragment
concatenated from two ``ds_read_b64_tr_b16`` halves before the ``s_waitcnt`` read stale
registers on some waves).  This test compiles the sources that issue LDS reads from inline
asm to assembly and checks, instruction by instruction, that no instruction reads a register
an LDS read is still filling: a register becomes readable only after an ``s_waitcnt
lgkmcnt(N)`` that retires its read (LDS reads retire in issue order)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
SOURCES = ["gemm16.hip", "attn_fwd.hip", "attn_bwd_split.hip", "wgrad.hip"]

_READ = re.compile(r"^(ds_read\w*)\s+(v\[(\d+):(\d+)\]|v(\d+))")
_REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def _regs(text):
    out = set()
    for m in _REG.finditer(text):
        if m.group(1):
            out.update((m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def audit(asm: str):
    """[(function, line, instruction)] of instructions that read a register an LDS read has
    not yet filled (per straight-line order; a branch target resets the state)."""
    bad = []
    fn = None
    pending = []  # issue-ordered list of register sets of outstanding LDS reads
    for ln in asm.split("\n"):
        t = ln.split(";")[0].strip()
        if not t:
            continue
        if t.endswith(":"):
            if not t.startswith("."):
                fn = t[:-1]
            pending = []  # conservative at block boundaries: the compiler waits before joins
            continue
        if t.startswith("s_waitcnt"):
            m = re.search(r"lgkmcnt\((\d+)\)", t)
            if m:
                n = int(m.group(1))
                pending = pending[len(pending) - n:] if n else []
            continue
        m = _READ.match(t)
        if m:
            if m.group(3):
                dst = {("v", r) for r in range(int(m.group(3)), int(m.group(4)) + 1)}
            else:
                dst = {("v", int(m.group(5)))}
            srcs = _regs(t.split(",", 1)[1]) if "," in t else set()
            if any(srcs & p for p in pending):
                bad.append((fn, ln.strip()))
            pending.append(dst)
            continue
        if t.startswith(("s_", ".")):
            continue
        parts = t.split(None, 1)
        if len(parts) < 2:
            continue
        ops = parts[1].split(",")
        srcs = _regs(",".join(ops[1:])) if len(ops) > 1 else set()
        if t.startswith(("buffer_store", "global_store", "ds_write", "ds_bpermute", "ds_swizzle")):
            srcs = _regs(parts[1])
        if any(srcs & p for p in pending):
            bad.append((fn, ln.strip()))
        dst = _regs(ops[0]) if not t.startswith(("buffer_", "global_", "ds_")) else set()
        if dst:  # an overwritten register is no longer an outstanding read's destination
            pending = [p - dst for p in pending]
    return bad


@pytest.mark.parametrize("src", SOURCES)
def test_no_register_read_before_its_lds_read_landed(src, tmp_path):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path / (src + ".s")
    r = subprocess.run([HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{CSRC}", "-S",
                        "--cuda-device-only", "-o", str(out), os.path.join(CSRC, src)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    bad = audit(out.read_text())
    assert not bad, f"{len(bad)} reads of pending LDS destinations, e.g. {bad[:5]}"


def test_audit_catches_the_hazard():
    asm = "\n".join(["k:", "ds_read_b64_tr_b16 v[4:5], v1", "ds_read_b64_tr_b16 v[6:7], v1 offset:512",
                     "v_mov_b32_e32 v10, v5", "s_waitcnt lgkmcnt(0)", "v_mov_b32_e32 v11, v7"])
    bad = audit(asm)
    assert len(bad) == 1 and "v10, v5" in bad[0][1]
    ok = "\n".join(["k:", "ds_read_b128 v[4:7], v1", "ds_read_b128 v[8:11], v1 offset:64", "s_waitcnt lgkmcnt(1)",
                    "v_mfma_f32_16x16x32_bf16 a[0:3], v[4:7], v[4:7], a[0:3]"])
    assert audit(ok) == []
