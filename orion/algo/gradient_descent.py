"""``orion.algo.gradient_descent`` (reference test plugin
`tests/functional/gradient_descent_algo/src/orion/algo/gradient_descent.py:16`)
-> :mod:`orion_amd.algo.gradient_descent`."""
from orion_amd.algo.gradient_descent import Gradient_Descent  # noqa: F401
