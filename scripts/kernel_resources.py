#!/usr/bin/env python3
"""Per-kernel register / occupancy / spill report for a HIP source (compile-time, no GPU).

usage: python scripts/kernel_resources.py csrc/attention.hip [extra hipcc flags]
"""
import re
import subprocess
import sys

src, extra = sys.argv[1], sys.argv[2:]
cmd = ["hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-munsafe-fp-atomics", "-Icsrc", "-c", src,
       "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    body = m.group(1)
    if body.startswith("Function Name:"):
        cur = {"name": body.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in body:
        k, v = body.split(":", 1)
        cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "SGPRs", "Occupancy [waves/SIMD]", "VGPRs Spill", "SGPRs Spill", "LDS Size [bytes/block]"]
print("%-60s %5s %5s %5s %4s %6s %6s %6s" % ("kernel", "vgpr", "agpr", "sgpr", "occ", "vspill", "sspill", "lds"))
for r in rows:
    name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    print("%-60s %5s %5s %5s %4s %6s %6s %6s" % ((name[:60],) + tuple(r.get(k, "-") for k in keys)))
