"""Median kernel time per rocprofv3 sqlite output: python rocpd_median.py <glob> [name-substring]"""
import glob
import sqlite3
import sys

pat = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for f in sorted(glob.glob(pat)):
    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f'select "{name}", "end" - "start" from kernels').fetchall()
    d = sorted(t for n, t in rows if sub in n)
    if d:
        print(f"{f}: n={len(d)} median_us={d[len(d) // 2] / 1000:.1f}")
