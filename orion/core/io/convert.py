"""``orion.core.io.convert`` (reference `src/orion/core/io/convert.py:26-132`) -> :mod:`orion_amd.io.convert`."""
from orion_amd.io.convert import (  # noqa: F401
    BaseConverter, Converter, JSONConverter, YAMLConverter, infer_converter_from_file_type)
