#!/usr/bin/env python3
"""Condense a rocprofv3 kernel_stats.csv: per-step ms per kernel (short names) and per category.

usage: python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv --steps 5
       python scripts/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steady

``--steady`` reads the kernel TRACE instead and counts only the kernels dispatched after the
first optimizer step's AdamW kernel up to and including the last one: whole steady-state
steps, without model construction, arena initialisation or first-step allocations (which a
stats file averaged over all steps folds into the per-step numbers).
"""
import argparse
import csv
import re


def short(name):
    if name.startswith(("Cijk_", "Custom_Cijk")):
        m = re.search(r"MT(\d+x\d+x\d+)", name)
        lay = re.search(r"Cijk_(A\w\w\w_B\w\w\w)", name)
        return f"gemm[{lay.group(1) if lay else '?'} {m.group(1) if m else '?'}]"
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    name = name.replace("orion::", "")
    name = re.sub(r"at::native::(\(anonymous namespace\)::)?", "at::", name)
    return name[:70]


def category(s):
    if s.startswith("gemm") or s.startswith("wgrad"):
        return "gemm"
    for k in ("attn", "xent", "ln_", "gelu", "colsum", "slab_sum", "adamw", "sumsq", "rms", "rope", "swiglu"):
        if k in s:
            return k.strip("_")
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--steady", action="store_true", help="trace CSV: steady-state steps only")
    a = ap.parse_args()
    rows = []
    if a.steady:
        with open(a.csv) as f:
            tr = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
        ends = [i for i, r in enumerate(tr) if "adamw_flat" in r["Kernel_Name"]]
        if len(ends) < 2:
            raise SystemExit("--steady needs a trace with at least two optimizer steps")
        a.steps = len(ends) - 1
        for r in tr[ends[0] + 1: ends[-1] + 1]:
            rows.append((short(r["Kernel_Name"]), 1,
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    else:
        with open(a.csv) as f:
            for r in csv.DictReader(f):
                rows.append((short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6))
    agg = {}
    for n, c, t in rows:
        k = agg.setdefault(n, [0, 0.0])
        k[0] += c
        k[1] += t
    tot = sum(v[1] for v in agg.values())
    print(f"total {tot / a.steps:.2f} ms/step over {a.steps} {'steady-state ' if a.steady else ''}steps")
    print(f"{'kernel':72s} {'calls/st':>8s} {'ms/step':>8s} {'%':>6s}")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{n:72s} {c / a.steps:8.1f} {t / a.steps:8.3f} {100 * t / tot:6.2f}")
    cats = {}
    for n, (c, t) in agg.items():
        cats[category(n)] = cats.get(category(n), 0.0) + t
    ranked = sorted(cats.items(), key=lambda kv: -kv[1])
    print("\nby category (ms/step):", ", ".join(f"{k}={v / a.steps:.2f}" for k, v in ranked))


if __name__ == "__main__":
    main()
