"""Measured GEMM-solution tables for hipBLASLt/rocBLAS (PyTorch TunableOp format).

``gemm_*_mi355x.csv`` were produced on an MI355X by ``scripts/tune_gemms.sh``
(TunableOp benchmarking every hipBLASLt and rocBLAS solution per GEMM shape).
:func:`use_tuned_gemms` points TunableOp at a table in read-only mode, so runs
pick the measured-fastest library kernel per shape with no tuning cost.
"""
import glob
import tempfile
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def use_tuned_gemms(table=None):
    """Enable TunableOp with a committed table (no-op if the caller configured it)."""
    if "PYTORCH_TUNABLEOP_ENABLED" in os.environ:
        return None
    if table is None:
        tables = sorted(glob.glob(os.path.join(HERE, "gemm_*_mi355x.csv")))
        if not tables:
            return None
        table = tables[0]
    # TunableOp opens "<stem><device ordinal>.csv" when the name has no %d: materialise one
    # copy per ordinal in a private cache dir so every rank of a multi-GPU job finds it.
    stem = os.path.splitext(os.path.basename(table))[0]
    cache = os.path.join(tempfile.gettempdir(), f"orion_amd_tunableop_{os.getuid()}")
    os.makedirs(cache, exist_ok=True)
    with open(table, "rb") as f:
        content = f.read()
    for ordinal in range(16):
        dst = os.path.join(cache, f"{stem}{ordinal}.csv")
        try:
            with open(dst, "rb") as f:
                if f.read() == content:
                    continue
        except OSError:
            pass
        tmpf = f"{dst}.{os.getpid()}.tmp"
        with open(tmpf, "wb") as f:
            f.write(content)
        os.replace(tmpf, dst)
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "0"
    os.environ["PYTORCH_TUNABLEOP_RECORD_UNTUNED"] = "0"
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.path.join(cache, f"{stem}.csv")
    return table
