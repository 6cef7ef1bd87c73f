"""Producer (component C7, ``src/orion/core/worker/producer.py``): feeds newly
completed trials to the algorithm (``observe``) and registers new suggestions as
``new`` trials.

Budget (fixed rather than copied): the reference always
registered ``pool_size`` points (``producer.py:35-45``), so W workers could overshoot
``max_trials`` by ~W x pool_size trials -- each one a GPU training run here.  ``produce``
asks for at most ``max_trials`` minus the trials that are still going to count
(every status but ``broken``), and nothing once that is reached."""
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

    def budget(self):
        """How many more trials may be registered (a read-only estimate): ``pool_size``, capped
        by what is left of ``max_trials`` after the registered non-broken trials.  ``produce``
        takes its tokens atomically (``Experiment.claim_budget``)."""
        max_trials = getattr(self.experiment, "max_trials", float("inf"))
        n = self.num_new_trials
        if max_trials is not None and max_trials != float("inf"):
            live = self.experiment.count_trials(
                ("new", "reserved", "suspended", "interrupted", "completed"))
            n = min(n, int(max_trials) - live)
        return max(0, n)

    def produce(self, owner=None):
        """Register up to ``pool_size`` suggestions, never past ``max_trials``: the tokens are
        taken as a recorded claim on the experiment's budget counter (compare-and-swap) before
        the algorithm is asked, the trials are inserted under claim-derived ids once the claim
        is confirmed, and whatever is not inserted is given back when the claim is settled."""
        take = getattr(self.experiment, "take_budget", None)
        if take is not None:
            n, cid = take(self.num_new_trials, owner)
        else:
            n, cid = self.budget(), None
        if n <= 0:
            return 0
        inserted = 0
        try:
            points = self.algorithm.suggest(n) or []
            trials = [format_trials.tuple_to_trial(p, self.space) for p in points[:n]]
            if cid is not None:
                if not self.experiment.confirm_claim(cid):
                    log.warning("budget claim %s was recovered while suggesting; dropping %d point(s)",
                                cid, len(trials))
                    return 0
                for i, t in enumerate(trials):
                    t._id = self.experiment.claim_trial_id(cid, i)
            log.debug("registering %d new trial(s)", len(trials))
            inserted = None  # unknown until the insert returns: settle counts the store
            self.experiment.register_trials(trials)
            inserted = len(trials)
        finally:
            if cid is not None:
                self.experiment.settle_budget(cid, inserted)
        return inserted

    def update(self):
        trials = self.experiment.fetch_completed_trials()
        trials = [t for t in trials if t.objective is not None]
        if trials:
            points = [format_trials.trial_to_tuple(t, self.space) for t in trials]
            results = [format_trials.get_trial_results(t) for t in trials]
            self.algorithm.observe(points, results)
        return len(trials)
