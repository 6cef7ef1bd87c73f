"""Drop-in import names of the original Oríon API, served by orion_amd.

Black-box scripts written for Oríon (``from orion.client import report_results``)
and algorithm plugins (``from orion.algo.base import BaseAlgorithm``) run
unchanged against this framework.
"""
