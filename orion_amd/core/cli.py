"""``orion`` command line (component C13, ``src/orion/core/cli.py``).

    orion [-n NAME] [--config orion.yaml] [--max-trials N] [--pool-size K]
          [--workers W] [--gpus-per-trial G] script.py [script args with ~priors]

Builds the layered configuration, opens the configured store, creates or
resumes the experiment (retrying once on a concurrent-creation race) and runs
the worker loop -- with ``--workers W`` as W processes on this node, each
leasing ``--gpus-per-trial`` GPUs per trial.
"""
from __future__ import annotations

import logging
import sys

from . import config as rc
from .experiment import create_experiment
from .worker import workon, workon_pool
from ..store import Database

log = logging.getLogger(__name__)


def _open_storage(db_opts):
    opts = {k: v for k, v in dict(db_opts).items() if v is not None}
    dbtype = opts.pop("type", "sqlite")
    log.debug("Creating %s database client with args: %s", dbtype, opts)
    return Database(of_type=dbtype, **opts)


def infer_experiment(argv=None):
    cmdargs, cmdconfig = rc.fetch_orion_args(rc.CLI_DOC_HEADER, argv)
    expconfig = rc.merge_env_vars(rc.fetch_default_options())
    tmp = rc.merge_orion_config(expconfig, {}, cmdconfig, cmdargs)
    storage = _open_storage(tmp["database"])
    name = tmp["name"]
    if name is None:
        raise RuntimeError("Could not infer experiment's name. Please use either `name` cmd line "
                           "arg or provide one in orion's configuration file.")
    execution = dict(tmp.get("execution") or {})
    exp = create_experiment(name, storage, dict(expconfig=expconfig, cmdconfig=cmdconfig,
                                                cmdargs=cmdargs))
    return exp, execution, dict(tmp["database"])


class _Rebuild:
    """Picklable factory re-opening the store and the configured experiment in a worker."""

    def __init__(self, name, db_opts, user):
        self.name, self.db_opts, self.user = name, db_opts, user

    def __call__(self):
        from .experiment import Experiment
        storage = _open_storage(self.db_opts)
        exp = Experiment(self.name, storage, user=self.user)
        exp.configure(exp.configuration)
        return exp


def main(argv=None):
    exp, execution, db_opts = infer_experiment(argv)
    kw = dict(gpus_per_trial=execution.get("gpus_per_trial", 0),
              heartbeat=execution.get("heartbeat", 30.0),
              trial_timeout=execution.get("trial_timeout"),
              max_broken=execution.get("max_broken", 3),
              trial_runner=execution.get("trial_runner") or "exec")
    n = int(execution.get("workers", 1) or 1)
    if n > 1:
        # a crashed worker process makes the CLI fail instead of reporting success
        return 1 if workon_pool(_Rebuild(exp.name, db_opts, exp.metadata["user"]), n, **kw) else 0
    workon(exp, **kw)
    return 0


if __name__ == "__main__":
    sys.exit(main())
