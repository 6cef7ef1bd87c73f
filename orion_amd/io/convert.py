"""Config-file converters (component C10).

Parity with ``src/orion/core/io/convert.py``: a converter is chosen from the
file extension (``.yml``/``.yaml`` -> YAML, ``.json`` -> JSON); ``parse`` reads
a file into Python data, ``generate`` writes data back.  YAML is loaded with
``yaml.safe_load`` (the reference's bare ``yaml.load`` breaks on PyYAML >= 6 and
would execute tags -- SURVEY.md §5.1 item 13).
"""
from __future__ import annotations

import json
import os

import yaml

from ..utils import Registry


class BaseConverter:
    file_extensions: tuple = ()

    def parse(self, filepath):
        raise NotImplementedError

    def generate(self, filepath, data):
        raise NotImplementedError


class YAMLConverter(BaseConverter):
    file_extensions = (".yml", ".yaml")

    def parse(self, filepath):
        with open(filepath) as f:
            return yaml.safe_load(f)

    def generate(self, filepath, data):
        with open(filepath, "w") as f:
            yaml.safe_dump(data, f, default_flow_style=False)


class JSONConverter(BaseConverter):
    file_extensions = (".json",)

    def parse(self, filepath):
        with open(filepath) as f:
            return json.load(f)

    def generate(self, filepath, data):
        with open(filepath, "w") as f:
            json.dump(data, f)


CONVERTERS = Registry("BaseConverter")
CONVERTERS.register(YAMLConverter)
CONVERTERS.register(JSONConverter)


def Converter(of_type, *args, **kwargs):  # noqa: N802  (factory with the reference's name)
    """Instantiate a converter by (case-insensitive) class name."""
    return CONVERTERS.create(of_type, *args, **kwargs)


def infer_converter_from_file_type(config_path, regex=None, default_keyword=""):
    ext = os.path.splitext(config_path)[1].lower()
    for klass in (YAMLConverter, JSONConverter):
        if ext in klass.file_extensions:
            return klass()
    raise NotImplementedError("Supporting only (YAML, JSON) file types for now. "
                              "Provided: '{}'".format(config_path))
