"""The rocprofv3 post-processing scripts on synthetic CSVs (no GPU): per-shape grouping of a
kernel trace (scripts/prof_shapes.py) and the whole-step PMC table (scripts/pmc_step_summary.py)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRACE_COLS = ["Kind", "Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "LDS_Block_Size",
              "VGPR_Count", "Accum_VGPR_Count", "Workgroup_Size_X", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"]


def _trace(path, kernels):
    """kernels: list of (name, grid_x, duration_ns) in dispatch order."""
    t = 1000
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, TRACE_COLS)
        w.writeheader()
        for i, (name, grid, ns) in enumerate(kernels):
            w.writerow(dict(Kind="KERNEL_DISPATCH", Dispatch_Id=i + 1, Kernel_Name=name, Start_Timestamp=t,
                            End_Timestamp=t + ns, LDS_Block_Size=0, VGPR_Count=128, Accum_VGPR_Count=0,
                            Workgroup_Size_X=256, Grid_Size_X=grid, Grid_Size_Y=1, Grid_Size_Z=1))
            t += ns + 10


def _step():
    # one step: two GEMM shapes under one kernel name, an elementwise kernel, the optimizer
    return [("Cijk_gemm", 256 * 768, 200_000), ("Cijk_gemm", 256 * 3072, 400_000),
            ("orion::ln_bwd_kernel<4, 3>", 256 * 768, 90_000), ("orion::adamw_flat_kernel<float>", 256 * 4096, 700_000)]


def test_prof_shapes_groups_by_launch_shape(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p, [("init_kernel", 256, 5_000)] + _step() * 3)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "prof_shapes.py"), str(p), "--steps", "2"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rows = [ln for ln in r.stdout.splitlines() if "Cijk_gemm" in ln]
    assert len(rows) == 2  # one kernel name, two launch shapes
    us = sorted(float(ln.split()[2]) for ln in rows)
    assert us == [200.0, 400.0]
    assert "init_kernel" not in r.stdout  # only whole steady-state steps are counted


def test_pmc_step_summary_utilisation_and_traffic(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import pmc_step_summary as pss
    kernels = _step()
    for p, counters in (("m", lambda ns: {"SQ_VALU_MFMA_BUSY_CYCLES": 0.5 * ns * 2.0 * 1024,
                                          "GRBM_GUI_ACTIVE": 8 * ns * 2.0}),
                        ("f", lambda ns: {"FETCH_SIZE": float(ns)}),      # KiB: 1 KiB per ns
                        ("w", lambda ns: {"WRITE_SIZE": float(ns)})):
        d = tmp_path / p
        d.mkdir()
        _trace(d / "run_kernel_trace.csv", kernels)
        with open(d / "run_counter_collection.csv", "w", newline="") as f:
            w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writeheader()
            for i, (name, _, ns) in enumerate(kernels):
                for cn, cv in counters(ns).items():
                    w.writerow(dict(Dispatch_Id=i + 1, Kernel_Name=name, Counter_Name=cn, Counter_Value=cv))
    m = pss.load(str(tmp_path), "m")
    assert len(m) == 4 and m[1][2] == 200_000
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_step_summary.py"), str(tmp_path)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    gemm = [ln for ln in r.stdout.splitlines() if ln.startswith("GEMM hipBLASLt")][0].split()
    # 50 % MFMA busy by construction at a 2.0 GHz effective clock (GRBM_GUI_ACTIVE / 8 / ns);
    # 2 KiB per ns of kernel time = 2.048 TB/s
    assert gemm[-4] == "50.0%"
    assert gemm[-3] == "2.00"
    assert gemm[-2] == f"{2 * 1024 * 600_000 / 1e9:.2f}"
    assert gemm[-1] == "2.05"
    # the optional LDS pass: conflict cycles per LDS-active cycle, LDS / any waits per wave cycle
    d = tmp_path / "l"
    d.mkdir()
    _trace(d / "run_kernel_trace.csv", kernels)
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (name, _, ns) in enumerate(kernels):
            for cn, cv in (("SQ_LDS_BANK_CONFLICT", 1.0 * ns), ("SQ_LDS_IDX_ACTIVE", 4.0 * ns),
                           ("SQ_WAIT_INST_LDS", 1.0 * ns), ("SQ_WAIT_ANY", 3.0 * ns),
                           ("SQ_WAVE_CYCLES", 10.0 * ns)):
                w.writerow(dict(Dispatch_Id=i + 1, Kernel_Name=name, Counter_Name=cn, Counter_Value=cv))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_step_summary.py"), str(tmp_path)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    gemm = [ln for ln in r.stdout.splitlines() if ln.startswith("GEMM hipBLASLt")][0].split()
    assert gemm[-3:] == ["25.0%", "10.0%", "30.0%"], gemm


def test_pmc_step_summary_skips_warmup_steps():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import pmc_step_summary as pss
    ks = [("tune", {}, 1), ("adamw_flat_kernel", {}, 1), ("gemm", {}, 2), ("adamw_flat_kernel", {}, 1),
          ("gemm", {}, 3), ("adamw_flat_kernel", {}, 1)]
    assert pss.steady(ks, 0) == ks
    assert pss.steady(ks, 1) == ks[2:]
    assert pss.steady(ks, 2) == ks[4:]
    assert pss.steady(ks, 9) == ks  # fewer steps than asked: keep everything


def test_pmc_step_summary_groups_gemm16_by_epilogue():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import pmc_step_summary as pss
    g = pss.group
    assert g("void orion::gemm16_kernel<true, true, 4, false>(orion::GemmArgs)").endswith("weight gradients (split-K)")
    assert "GELU' + bias-grad" in g("void orion::gemm16_kernel<false, true, 3, false>(orion::GemmArgs)")
    assert "bias + GELU" in g("void orion::gemm16_kernel<false, false, 2, false>(orion::GemmArgs)")
    assert g("void orion::gemm16_kernel<false, true, 0, false>(orion::GemmArgs)") == "GEMM gemm16 input gradients"
    assert g("Custom_Cijk_Alik_Bljk_BBS_BH_MT256x256x64") == "GEMM hipBLASLt (forward)"
    assert g("void orion::attn_bwd_kv_kernel<64, true, false>(orion::AttnParams)") == "attention bwd dK/dV"
    assert "SwiGLU epilogue" in g("void orion::gemm16_kernel<false, false, 9, false>(orion::GemmArgs)")
    assert "RoPE" in g("void orion::gemm16_kernel<false, false, 8, false>(orion::GemmArgs)")
    assert "exp epilogue" in g("void orion::gemm16_kernel<false, false, 6, false>(orion::GemmArgs)")
    assert "NT operand" in g("void orion::gemm16_kernel<true, false, 4, false>(orion::GemmArgs)")
