"""RMSNorm entry point (implementation shared with :mod:`orion_amd.ops.layernorm`)."""
from .layernorm import rms_norm_hip  # noqa: F401
