#!/usr/bin/env python3
"""Print the kernel sequence of the last optimizer step from a rocprofv3 kernel_trace.csv
(step boundary = adamw_flat_kernel), with duration, grid and short names; GEMMs are
aggregated by (name, grid) so each GEMM shape of the model shows on one line."""
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "adamw_flat" in r["Kernel_Name"]]
a, b = ends[-2] + 1, ends[-1] + 1
seq = rows[a:b]
agg = {}
for r in seq:
    n = short(r["Kernel_Name"])
    key = (n, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    v = agg.setdefault(key, [0, 0.0])
    v[0] += 1
    v[1] += d
tot = sum(v[1] for v in agg.values())
span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
print(f"step kernels: {len(seq)}  busy {tot / 1e3:.2f} ms  span {span / 1e3:.2f} ms")
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
for (n, gx, gy, gz, wg), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{n:60s} grid=({gx},{gy},{gz}) wg={wg:4s} x{c:3d}  {t / 1e3:7.3f} ms  {t / c:8.1f} us/call")
