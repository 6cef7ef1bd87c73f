#!/usr/bin/env python3
"""Per-launch-shape kernel times from a rocprofv3 kernel trace (``*_kernel_trace.csv``).

The stats file groups kernels by name only; one GEMM kernel name can serve several layer
shapes.  This groups the dispatches of the last ``--steps`` whole optimizer steps (step
boundaries = the fused AdamW kernel) by (name, grid, registers, LDS), so every GEMM shape of
the step shows up as its own row with its per-call time.

usage: scripts/prof_shapes.py gpurun_out/prof_TAG/run_kernel_trace.csv [--steps 2] [--top 40]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--boundary", default="adamw")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    marks = [i for i, r in enumerate(rows) if args.boundary in r["Kernel_Name"]]
    if len(marks) < args.steps + 1:
        raise SystemExit(f"need {args.steps + 1} '{args.boundary}' dispatches, found {len(marks)}")
    seg = rows[marks[-args.steps - 1] + 1:marks[-1] + 1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        key = (r["Kernel_Name"][:56], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]),
               int(r["Workgroup_Size_X"]), r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"])
        agg[key][0] += 1
        agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    total = sum(t for _, t in agg.values()) / args.steps
    print(f"{total:.2f} ms/step of kernels over the last {args.steps} steps")
    print(f"{'ms/step':>8} {'calls':>6} {'us/call':>8} {'WGs':>8}  vgpr/agpr lds  kernel")
    for (name, grid, wg, vg, ag, lds), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:args.top]:
        print(f"{t / args.steps:8.3f} {c / args.steps:6.1f} {t / c * 1000:8.1f} {grid // wg:8d}  "
              f"{vg:>4}/{ag:<4} {lds:>6}  {name}")


if __name__ == "__main__":
    main()
