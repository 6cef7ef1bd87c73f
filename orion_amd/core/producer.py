"""Producer (component C7, ``src/orion/core/worker/producer.py``): feeds newly
completed trials to the algorithm (``observe``) and registers ``pool_size`` new
suggestions as ``new`` trials."""
from __future__ import annotations

import logging

from . import format_trials

log = logging.getLogger(__name__)


class Producer:
    def __init__(self, experiment):
        self.experiment = experiment
        self.space = experiment.space
        if self.space is None:
            raise RuntimeError("Experiment object provided to Producer has not yet completed "
                               "initialization.")
        self.algorithm = experiment.algorithms
        self.num_new_trials = experiment.pool_size

    def produce(self):
        points = self.algorithm.suggest(self.num_new_trials)
        trials = [format_trials.tuple_to_trial(p, self.space) for p in points]
        log.debug("registering %d new trial(s)", len(trials))
        self.experiment.register_trials(trials)
        return len(trials)

    def update(self):
        trials = self.experiment.fetch_completed_trials()
        trials = [t for t in trials if t.objective is not None]
        if trials:
            points = [format_trials.trial_to_tuple(t, self.space) for t in trials]
            results = [format_trials.get_trial_results(t) for t in trials]
            self.algorithm.observe(points, results)
        return len(trials)
