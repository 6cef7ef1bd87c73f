"""Measured GEMM-solution tables for hipBLASLt/rocBLAS (PyTorch TunableOp format).

``gemm_*_mi355x.csv`` were produced on an MI355X by ``scripts/tune_gemms.sh``
(TunableOp benchmarking every hipBLASLt and rocBLAS solution per GEMM shape).
:func:`use_tuned_gemms` points TunableOp at a table in read-only mode, so runs
pick the measured-fastest library kernel per shape with no tuning cost.
"""
import glob
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
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "0"
    os.environ["PYTORCH_TUNABLEOP_RECORD_UNTUNED"] = "0"
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = table
    return table
