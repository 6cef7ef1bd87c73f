"""The worker loop ``workon`` (component C16, ``src/orion/core/worker/__init__.py``).

Same protocol as the reference: try to reserve a trial; if one was reserved,
consume it; otherwise pull completed trials into the algorithm, stop if the
experiment is done, else produce ``pool_size`` new trials.  Workers on one or
many nodes coordinate only through the store's compare-and-swap.

Additions: exponential idle back-off instead of a hot spin on the database,
a stale-reservation reaper (heartbeat timeout), a broken-trial budget,
``workon_pool`` to run several workers (each its own process, each leasing its
own GPUs) on one MI355X node, and a trial budget that holds: a worker does not
reserve another trial while completed + reserved trials already reach
``max_trials`` (it waits for the running ones to complete or break), and the
producer never registers more than the budget leaves (``producer.py``).
"""
from __future__ import annotations

import logging
import multiprocessing as mp
import os
import socket
import time

from .consumer import Consumer
from .producer import Producer

log = logging.getLogger(__name__)


def workon(experiment, gpus_per_trial=0, heartbeat=30.0, trial_timeout=None, max_broken=3,
           worker_id=None, gpu_pool=None, idle_sleep=(0.01, 1.0), trial_runner="exec"):
    """Run the produce/consume loop until the experiment is done.  Returns its stats."""
    consumer = Consumer(experiment, gpu_pool=gpu_pool, gpus_per_trial=gpus_per_trial,
                        heartbeat=heartbeat, trial_timeout=trial_timeout,
                        worker_id=worker_id or f"{socket.gethostname()}:{os.getpid()}",
                        trial_runner=trial_runner)
    try:
        return _workon(experiment, consumer, max_broken, idle_sleep)
    finally:
        consumer.close()


def _workon(experiment, consumer, max_broken, idle_sleep):
    worker_id = consumer.worker_id
    producer = Producer(experiment)
    broken = 0
    sleep = idle_sleep[0]
    # a reservation whose heartbeat is older than this is re-queued (floor: 30 s, or
    # ORION_STALE_AFTER_MIN_S for tests that exercise the reaper)
    stale_after = max(3 * consumer.heartbeat, float(os.environ.get("ORION_STALE_AFTER_MIN_S", "30")))
    log.debug("#####  Init Experiment  #####")
    budgeted = experiment.max_trials not in (None, float("inf"))
    while True:
        trial = None
        if not budgeted or experiment.count_trials(("completed", "reserved")) < experiment.max_trials:
            trial = experiment.reserve_trial(score_handle=producer.algorithm.score, worker=worker_id)
        if trial is None:
            producer.update()
            if experiment.finish_if_done():
                break
            experiment.fix_lost_trials(stale_after)
            experiment.reconcile_budget()
            if (experiment.count_trials(("new", "suspended", "interrupted")) == 0
                    and producer.produce(owner=worker_id) > 0):
                sleep = idle_sleep[0]
            else:
                time.sleep(sleep)
                sleep = min(sleep * 2, idle_sleep[1])
            continue
        sleep = idle_sleep[0]
        status = consumer.consume(trial)
        if status == "broken":
            broken += 1
            if max_broken is not None and broken >= max_broken:
                log.error("worker %s stops: %d broken trials", worker_id, broken)
                break
    stats = experiment.stats
    log.info("#####  Search finished successfully  #####")
    log.info("\nRESULTS\n=======\n%s\n", stats)
    if stats.get("best_trials_id") is not None:
        best = experiment.storage.read("trials", {"_id": stats["best_trials_id"]})
        if best:
            log.info("\nBEST PARAMETERS\n===============\n%s", best[0].get("params"))
    return stats


def _worker_main(factory, kwargs):
    exp = factory()
    workon(exp, **kwargs)


def workon_pool(experiment_factory, n_workers, **kwargs):
    """Run ``n_workers`` worker processes on this node; ``experiment_factory()`` must
    rebuild the (already configured) experiment inside each process."""
    if n_workers <= 1:
        return workon(experiment_factory(), **kwargs)
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker_main, args=(experiment_factory, kwargs)) for _ in range(n_workers)]
    for p in procs:
        p.start()
    code = 0
    for p in procs:
        p.join()
        code = code or p.exitcode
    if code:
        log.error("a worker process exited with status %s", code)
    return code
