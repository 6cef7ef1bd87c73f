"""``orion.core.utils.format_trials`` (reference `src/orion/core/utils/format_trials.py:16-55`)
-> :mod:`orion_amd.core.format_trials`."""
from orion_amd.core.format_trials import get_trial_results, trial_to_tuple, tuple_to_trial  # noqa: F401
