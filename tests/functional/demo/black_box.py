#!/usr/bin/env python3
"""1-D quadratic black box: f(x) = 4 (x - 34.56789)^2 + 23.4, reports value and gradient.
Same function and result names as the reference demo (tests/functional/demo/black_box.py)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))))
from orion.client import report_results  # noqa: E402  (Oríon-compatible import path)


def function(x):
    z = x - 34.56789
    return 4 * z ** 2 + 23.4, 8 * z


def execute():
    parser = argparse.ArgumentParser()
    parser.add_argument("-x", type=float, required=True)
    inputs = parser.parse_args()
    y, dy = function(inputs.x)
    report_results([dict(name="example_objective", type="objective", value=y),
                    dict(name="example_gradient", type="gradient", value=[dy])])


if __name__ == "__main__":
    execute()
