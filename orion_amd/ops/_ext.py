"""Locate and load the in-tree HIP extension (``orion_amd/_C.so``).

The extension registers its kernels as ``torch.ops.orion_amd.*`` through
``TORCH_LIBRARY`` (see ``csrc/bindings.cpp``), so loading it is a plain
``torch.ops.load_library`` -- no pybind11 module, no JIT cache.  It is built by
``python -m orion_amd.build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import os
import threading

import torch

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ORION_AMD_EXT selects an alternative build (same-box A/B benchmarking of kernel variants)
EXT_PATH = os.environ.get("ORION_AMD_EXT", os.path.join(_PKG_DIR, "_C.so"))

_lock = threading.Lock()
_loaded = False


def ext_available() -> bool:
    return _loaded or os.path.isfile(EXT_PATH)


def ext_loaded() -> bool:
    """True once ``_C.so`` has been loaded into this process."""
    return _loaded


def load_ext(required: bool = False) -> bool:
    """Load ``_C.so`` once.  With ``required=True`` a missing build raises."""
    global _loaded
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        if not os.path.isfile(EXT_PATH):
            if required:
                raise RuntimeError(
                    f"orion_amd HIP extension not built ({EXT_PATH} missing). "
                    "Run `python -m orion_amd.build`, or set ORION_AMD_OPS=torch to use "
                    "stock PyTorch GPU ops deliberately.")
            return False
        torch.ops.load_library(EXT_PATH)
        _loaded = True
        return True


def C():
    """The ``torch.ops.orion_amd`` namespace (extension loaded on first use)."""
    load_ext(required=True)
    return torch.ops.orion_amd
