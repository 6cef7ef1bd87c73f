"""Trial <-> point conversion (component C15, ``src/orion/core/utils/format_trials.py``)."""
from __future__ import annotations

from .trial import Trial


def trial_to_tuple(trial, space):
    """Parameter values of ``trial`` as a tuple ordered like ``space``."""
    assert len(trial.params) == len(space)
    for order, param in enumerate(trial.params):
        assert space[order].name == param.name, (space[order].name, param.name)
    return tuple(p.value for p in trial.params)


def tuple_to_trial(data, space):
    assert len(data) == len(space)
    params = [dict(name=space[i].name, type=space[i].type, value=_plain(data[i]))
              for i in range(len(space))]
    return Trial(params=params)


def get_trial_results(trial):
    """{'objective': float|None, 'constraint': [..], 'gradient': tuple|None}."""
    obj = trial.objective
    grad = trial.gradient
    return {
        "objective": obj.value if obj else None,
        "constraint": [r.value for r in trial.results if r.type == "constraint"],
        "gradient": tuple(grad.value) if grad else None,
    }


def _plain(v):
    if hasattr(v, "tolist"):
        return v.tolist()
    return v
