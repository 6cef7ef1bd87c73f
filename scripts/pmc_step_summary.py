#!/usr/bin/env python3
"""Per-kernel-group counters of a whole training step (scripts/pmc_step.sh output).

For each kernel group (scripts/prof_summary.py's categories, GEMM kernels split by family):
time from the kernel trace of the MFMA pass, MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) -- GRBM_GUI_ACTIVE comes summed over the 8 XCDs (it reads
~15.7 per ns of kernel time at ~1.96 GHz) -- and HBM-side traffic (TCC FETCH_SIZE + WRITE_SIZE, KiB) as
bytes and achieved bandwidth over the group's kernel time.  Counter passes come from separate
runs of the same step; kernels are matched by dispatch order within each run.

Optional pass l (PMC_LDS=1 in scripts/pmc_step.sh): LDS bank-conflict cycles per LDS-active
cycle and the LDS / any-dependency wait share of wave cycles per group; the effective clock
column is GRBM_GUI_ACTIVE / 8 / kernel time.

usage: python scripts/pmc_step_summary.py gpurun_out/pmc_TAG
"""
import collections
import csv
import glob
import os
import sys

SIMDS = 256 * 4
XCDS = 8


def group(name):
    n = name.lower()
    if "gemm_phased" in n:
        return "GEMM in-tree phased (weight gradients)"
    if "gemm16_kernel<true, true, 4" in n:
        return "GEMM gemm16 weight gradients (split-K)"
    if "gemm16_kernel<false, true, 3" in n:
        return "GEMM gemm16 dgrad + GELU' + bias-grad epilogue"
    if "gemm16_kernel<false, false, 2" in n:
        return "GEMM gemm16 fwd + bias + GELU epilogue"
    if "gemm16_kernel<false, true, 5" in n:
        return "GEMM gemm16 dgrad + SwiGLU' epilogue"
    for key, g in (("gemm16_kernel<true, false, 4", "GEMM gemm16 weight gradients (NT operand)"),
                   ("gemm16_kernel<false, false, 6", "GEMM gemm16 LM-head fwd + exp epilogue"),
                   ("gemm16_kernel<false, true, 7", "GEMM gemm16 LM-head dgrad (row-scaled)"),
                   ("gemm16_kernel<false, false, 8", "GEMM gemm16 fwd + RoPE epilogue"),
                   ("gemm16_kernel<false, false, 9", "GEMM gemm16 fwd + SwiGLU epilogue")):
        if key in n:
            return g
    if "gemm16_kernel" in n:
        return "GEMM gemm16 input gradients"
    if "cijk" in n or "gemm[" in n:
        return "GEMM hipBLASLt (forward)"
    for key, g in (("attn_fwd", "attention forward"), ("attn_bwd_kv", "attention bwd dK/dV"),
                   ("attn_bwd_dq", "attention bwd dQ"), ("attn_delta", "attention delta"),
                   ("ln_fwd", "LayerNorm fwd"), ("ln_bwd", "LayerNorm bwd"),
                   ("bias_gelu_fwd", "bias+GELU fwd"), ("bias_gelu_bwd", "bias+GELU bwd"),
                   ("xent", "cross-entropy"), ("adamw", "AdamW"), ("colsum", "column sums"),
                   ("slab_sum", "split-K slab sums"), ("rms_fwd", "RMSNorm fwd"), ("rms_bwd", "RMSNorm bwd"),
                   ("swiglu_fwd", "SwiGLU fwd"), ("swiglu_bwd", "SwiGLU bwd"), ("rope", "RoPE"),
                   ("sumsq", "gradient norm")):
        if key in n:
            return g
    return "other"


def load(d, p):
    """{dispatch index in run order: (kernel name, {counter: value}, duration ns)}"""
    cc = glob.glob(os.path.join(d, p, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, p, "**", "*kernel_trace.csv"), recursive=True)
    if not cc:
        return {}
    dur = {}
    if kt:
        for r in csv.DictReader(open(kt[0])):
            dur[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    per = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(cc[0])):
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[i] = r["Kernel_Name"]
    return {k: (names[k], per[k], dur.get(k, 0)) for k in sorted(per)}


def steady(ks, skip):
    """The dispatches after the ``skip``-th optimizer kernel (warmup steps, and with them one-time
    work such as the hipBLASLt wrapper's first-use solution sweep, csrc/blaslt.cpp)."""
    if skip <= 0:
        return ks
    ends = [i for i, k in enumerate(ks) if "adamw" in k[0]]
    return ks[ends[skip - 1] + 1:] if len(ends) >= skip else ks


def main():
    d = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    m, f, w, lp = load(d, "m"), load(d, "f"), load(d, "w"), load(d, "l")
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    other = collections.defaultdict(float)
    mk, fk, wk, lk = (steady(list(x.values()), skip) for x in (m, f, w, lp))
    for i, (name, c, ns) in enumerate(mk):
        g = agg[group(name)]
        g["n"] += 1
        if group(name) == "other":
            other[name[:70]] += ns
        g["ns"] += ns
        g["mfma"] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        g["active"] += c.get("GRBM_GUI_ACTIVE", 0.0)
        if i < len(fk) and fk[i][0] == name:
            g["fetch"] += fk[i][1].get("FETCH_SIZE", 0.0) * 1024
        if i < len(wk) and wk[i][0] == name:
            g["write"] += wk[i][1].get("WRITE_SIZE", 0.0) * 1024
        if i < len(lk) and lk[i][0] == name:  # optional pass l: LDS / wait counters
            lc = lk[i][1]
            for key in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES",
                        "SQ_BUSY_CYCLES", "SQ_WAIT_ANY"):
                g[key] += lc.get(key, 0.0)
    tot = sum(g["ns"] for g in agg.values())
    what = f"after {skip} warmup step(s)" if skip else "the whole bench run"
    print(f"{len(mk)} dispatches, {tot / 1e6:.2f} ms of kernels ({what}, under the counter passes)")
    extra = bool(lk)
    hdr = f"{'group':44s} {'ms':>8s} {'%':>5s} {'MFMA util':>9s} {'clk GHz':>7s} {'L2-EA GB':>8s} {'TB/s':>6s}"
    if extra:  # LDS bank-conflict cycles per LDS-active cycle; LDS / any waits per wave cycle
        hdr += f" {'LDS conf':>8s} {'LDS wait':>8s} {'any wait':>8s}"
    print(hdr)
    for k, g in sorted(agg.items(), key=lambda x: -x[1]["ns"]):
        util = g["mfma"] / (g["active"] / XCDS * SIMDS) if g["active"] else 0.0
        # effective clock: GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS)
        clk = g["active"] / XCDS / g["ns"] if g["ns"] else 0.0
        gb = (g["fetch"] + g["write"]) / 1e9
        tbs = gb / (g["ns"] / 1e9) / 1e3 if g["ns"] else 0.0
        line = (f"{k:44s} {g['ns'] / 1e6:8.2f} {100 * g['ns'] / tot:5.1f} {100 * util:8.1f}% {clk:7.2f} "
                f"{gb:8.2f} {tbs:6.2f}")
        if extra:
            conf = g["SQ_LDS_BANK_CONFLICT"] / g["SQ_LDS_IDX_ACTIVE"] if g["SQ_LDS_IDX_ACTIVE"] else 0.0
            wl = g["SQ_WAIT_INST_LDS"] / g["SQ_WAVE_CYCLES"] if g["SQ_WAVE_CYCLES"] else 0.0
            wa = g["SQ_WAIT_ANY"] / g["SQ_WAVE_CYCLES"] if g["SQ_WAVE_CYCLES"] else 0.0
            line += f" {100 * conf:7.1f}% {100 * wl:7.1f}% {100 * wa:7.1f}%"
        print(line)
    print("largest kernels in 'other' (ms):")
    for k, ns in sorted(other.items(), key=lambda x: -x[1])[:8]:
        print(f"  {k:70s} {ns / 1e6:8.2f}")


if __name__ == "__main__":
    main()
