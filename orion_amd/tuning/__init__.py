"""Measured GEMM-solution tables for hipBLASLt/rocBLAS (PyTorch TunableOp format).

``gemm_*_mi355x.csv`` were produced on an MI355X by ``scripts/tune_gemms.sh``
(TunableOp benchmarking every hipBLASLt and rocBLAS solution per GEMM shape).
:func:`use_tuned_gemms` enables TunableOp in read-only mode and loads a table
through ``torch.cuda.tunable``, so runs pick the measured-fastest library
kernel for every tuned shape with no tuning cost (untuned shapes keep the
library default).  Call it after ``torch.cuda.set_device``.
"""
from __future__ import annotations

import glob
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def committed_tables():
    return sorted(glob.glob(os.path.join(HERE, "gemm_*_mi355x.csv")))


def merged_table(tables=None, out_dir=None):
    """Concatenate the committed tables (one header of Validator lines, union of the
    GEMM entries; later tables win on a duplicate shape) into one TunableOp file."""
    tables = committed_tables() if tables is None else tables
    if not tables:
        return None
    validators, entries = [], {}
    for t in tables:
        with open(t) as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                parts = line.split(",")
                if parts[0] == "Validator":
                    if line not in validators:
                        validators.append(line)
                elif len(parts) >= 3:
                    entries[(parts[0], parts[1])] = line
    import tempfile
    out_dir = out_dir or tempfile.gettempdir()
    path = os.path.join(out_dir, f"orion_amd_gemms_{os.getpid()}.csv")
    with open(path, "w") as f:
        f.write("\n".join(validators + list(entries.values())) + "\n")
    return path


def default_table():
    return merged_table()


def use_tuned_gemms(table=None, verbose=False):
    """Load a committed table into TunableOp; returns the number of tuned GEMM entries."""
    import torch
    if os.environ.get("PYTORCH_TUNABLEOP_TUNING") == "1":
        return 0  # a tuning run manages TunableOp itself
    table = table or default_table()
    if table is None or not torch.cuda.is_available():
        return 0
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    if hasattr(tun, "record_untuned_enable"):
        tun.record_untuned_enable(False)
    ok = tun.read_file(table)
    n = len(tun.get_results()) if ok else 0
    if verbose or not ok:
        print(f"[orion_amd] TunableOp table {os.path.basename(table)}: loaded={ok} entries={n}", flush=True)
    return n
