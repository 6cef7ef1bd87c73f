"""``orion.client`` -> :mod:`orion_amd.client`."""
from orion_amd.client import *  # noqa: F401,F403
from orion_amd.client import report_results, IS_METAOPT_ON, RESULTS_FILENAME  # noqa: F401
