#!/usr/bin/env python3
"""Table of scripts/bench_gemm.py results per variant from scripts/ab_variants.sh logs:
python scripts/ab_table.py TAG [field]  (field: hip_ms by default)."""
import collections
import glob
import json
import sys

tag = sys.argv[1]
field = sys.argv[2] if len(sys.argv) > 2 else "hip_ms"
d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"gpurun_out/abv_{tag}__C_*.log")):
    v = f.split(f"abv_{tag}__C_")[1].rsplit("_r", 1)[0]
    for ln in open(f):
        if ln.startswith('{"shape"'):
            r = json.loads(ln)
            d[r["shape"]][v].append(r[field])
vs = sorted({v for s in d.values() for v in s})
print("%-26s" % "shape" + "".join("%16s" % v for v in vs))
for sh, m in d.items():
    print("%-26s" % sh + "".join("%16s" % "/".join("%.3f" % x for x in m[v]) for v in vs))
