"""Layered configuration resolution (components C12 + C17).

Precedence, lowest to highest (reference ``resolve_config.py:10-31``,
``cli.py:76-77``):

1. built-in defaults (``max_trials=inf``, ``pool_size=10``, database);
2. default config files: ``<site_data>/orion_config.yaml.example``,
   ``<site_config>/orion_config.yaml``, ``<user_config>/orion_config.yaml``
   (XDG paths under the app name ``orion.core``, as in the reference; a
   ``name`` key there is ignored);
3. environment: ``METAOPT_DB_NAME``, ``METAOPT_DB_TYPE``, ``METAOPT_DB_ADDRESS``
   (and ``ORION_DB_*`` aliases);
4. the experiment document already in the database (resume);
5. the ``--config`` YAML given on the command line;
6. command-line arguments.

Default database: the SQLite file store (no server needed); MongoDB with
``type: mongodb``.
"""
from __future__ import annotations

import argparse
import logging
import os
import textwrap
from collections import defaultdict
from copy import deepcopy

import yaml

from .. import __version__

log = logging.getLogger(__name__)


# --------------------------------------------------------------------------- app dirs (C17)
class AppDirs:
    """XDG directories for an application (what the reference vendors ``appdirs`` for)."""

    def __init__(self, appname="orion.core", appauthor="MILA"):
        self.appname = appname
        self.appauthor = appauthor

    @staticmethod
    def _first(env, default):
        val = os.environ.get(env, "")
        return (val.split(os.pathsep)[0] if val else default)

    @property
    def user_config_dir(self):
        base = os.environ.get("XDG_CONFIG_HOME") or os.path.expanduser("~/.config")
        return os.path.join(base, self.appname)

    @property
    def user_data_dir(self):
        base = os.environ.get("XDG_DATA_HOME") or os.path.expanduser("~/.local/share")
        return os.path.join(base, self.appname)

    @property
    def site_config_dir(self):
        return os.path.join(self._first("XDG_CONFIG_DIRS", "/etc/xdg"), self.appname)

    @property
    def site_data_dir(self):
        return os.path.join(self._first("XDG_DATA_DIRS", "/usr/local/share"), self.appname)


DIRS = AppDirs("orion.core", "MILA")

DEF_CMD_MAX_TRIALS = (float("inf"), "inf/until preempted")
DEF_CMD_POOL_SIZE = (10, "10")


def default_config_paths():
    return [
        os.path.join(DIRS.site_data_dir, "orion_config.yaml.example"),
        os.path.join(DIRS.site_config_dir, "orion_config.yaml"),
        os.path.join(DIRS.user_config_dir, "orion_config.yaml"),
    ]


# (environment variables, config key, default) -- first variable set wins
ENV_VARS_DB = [
    (("METAOPT_DB_NAME", "ORION_DB_NAME"), "name", "orion"),
    (("METAOPT_DB_TYPE", "ORION_DB_TYPE"), "type", "sqlite"),
    (("METAOPT_DB_ADDRESS", "ORION_DB_ADDRESS"), "host", None),
]
ENV_VARS = dict(database=ENV_VARS_DB)


def nesteddict():
    return defaultdict(nesteddict)


def is_exe(path):
    return os.path.isfile(path) and os.access(path, os.X_OK)


CLI_DOC_HEADER = """
orion:
  Orion cli script for asynchronous distributed optimization (MI355X build)
"""


def build_parser(description=CLI_DOC_HEADER):
    parser = argparse.ArgumentParser(formatter_class=argparse.RawDescriptionHelpFormatter,
                                     description=textwrap.dedent(description))
    parser.add_argument("-V", "--version", action="version", version="orion " + __version__)
    parser.add_argument("-v", "--verbose", action="count", default=0,
                        help="logging levels of information about the process (-v: INFO. -vv: DEBUG)")
    og = parser.add_argument_group("Orion arguments (optional)",
                                   description="These arguments determine orion's behaviour")
    og.add_argument("-n", "--name", type=str, metavar="stringID",
                    help="experiment's unique name; use an existing name to resume an experiment "
                         "(default: None - specified either here or in a config)")
    og.add_argument("--max-trials", type=int, metavar="#",
                    help="number of jobs/trials to be completed (default: %s)" % DEF_CMD_MAX_TRIALS[1])
    og.add_argument("--pool-size", type=int, metavar="#",
                    help="number of points produced per suggestion round (default: %s)"
                         % DEF_CMD_POOL_SIZE[1])
    og.add_argument("-c", "--config", type=argparse.FileType("r"), metavar="path-to-config",
                    help="user provided orion configuration file")
    xg = parser.add_argument_group("Execution (MI355X node)")
    xg.add_argument("--workers", type=int, metavar="#",
                    help="concurrent worker processes on this node (default 1)")
    xg.add_argument("--gpus-per-trial", type=int, metavar="#",
                    help="GPUs given to each trial via HIP_VISIBLE_DEVICES (default 0 = CPU trial)")
    xg.add_argument("--trial-timeout", type=float, metavar="seconds",
                    help="kill a trial (status broken) after this wall time")
    xg.add_argument("--heartbeat", type=float, metavar="seconds",
                    help="liveness period of reserved trials (stale ones are re-queued)")
    xg.add_argument("--max-broken", type=int, metavar="#",
                    help="stop the worker after this many broken trials (default 3)")
    xg.add_argument("--trial-runner", choices=("exec", "fork"),
                    help="exec: a new process per trial (default); fork: .py trials forked from a "
                         "per-worker server that imported torch once (orion_amd/core/forkserver.py)")
    ug = parser.add_argument_group(
        "User script related arguments",
        description="These arguments determine user's script behaviour "
                    "and they can serve as orion's parameter declaration.")
    ug.add_argument("user_script", type=str, metavar="path-to-script", help="your experiment's script")
    ug.add_argument("user_args", nargs=argparse.REMAINDER, metavar="...",
                    help="Command line arguments to your script (if any). A configuration file "
                         "intended to be used with 'userscript' must be given as a path in the "
                         "**first positional** argument OR using `--config=<path>` keyword argument.")
    return parser


_EXEC_KEYS = ("workers", "gpus_per_trial", "trial_timeout", "heartbeat", "max_broken", "trial_runner")


def fetch_orion_args(description=CLI_DOC_HEADER, argv=None):
    """Parse the command line -> (cmdargs, cmdconfig).  cmdargs['metadata'] carries
    orion_version, user_script (absolute when executable) and user_args."""
    args = vars(build_parser(description).parse_args(argv))
    verbose = args.pop("verbose")
    if verbose == 1:
        logging.basicConfig(level=logging.INFO)
    elif verbose >= 2:
        logging.basicConfig(level=logging.DEBUG)
    args["metadata"] = {"orion_version": __version__}
    orion_file = args.pop("config")
    config = {}
    if orion_file:
        log.debug("Found orion configuration file at: %s", os.path.abspath(orion_file.name))
        config = yaml.safe_load(orion_file) or {}
    user_script = args.pop("user_script")
    abs_script = os.path.abspath(user_script)
    if is_exe(abs_script) or os.path.isfile(abs_script):
        user_script = abs_script
    args["metadata"]["user_script"] = user_script
    args["metadata"]["user_args"] = args.pop("user_args")
    execution = {k: args.pop(k) for k in _EXEC_KEYS}
    args["execution"] = {k: v for k, v in execution.items() if v is not None}
    return args, config


def fetch_default_options():
    cfg = nesteddict()
    cfg["name"] = None
    cfg["max_trials"] = DEF_CMD_MAX_TRIALS[0]
    cfg["pool_size"] = DEF_CMD_POOL_SIZE[0]
    for signifier, env_vars in ENV_VARS.items():
        for _, key, default in env_vars:
            cfg[signifier][key] = default
    for path in default_config_paths():
        try:
            with open(path) as f:
                data = yaml.safe_load(f)
        except OSError as exc:
            log.debug(exc)
            continue
        if not isinstance(data, dict):
            continue
        for k, v in data.items():
            if k in ENV_VARS and isinstance(v, dict):
                for vk, vv in v.items():
                    cfg[k][vk] = vv
            elif k != "name":
                cfg[k] = v
    return cfg


def merge_env_vars(config):
    newcfg = deepcopy(config)
    for signif, evars in ENV_VARS.items():
        for names, key, _ in evars:
            for var in names:
                val = os.getenv(var)
                if val is not None:
                    newcfg[signif][key] = val
                    break
    return newcfg


def merge_orion_config(config, dbconfig, cmdconfig, cmdargs):
    """cmdargs > cmdconfig > dbconfig > config."""
    exp = deepcopy(config)
    for cfg in (dbconfig, cmdconfig):
        for k, v in (cfg or {}).items():
            if v is None:  # unset (a new experiment's attributes): keep the layer below
                continue
            if k in ENV_VARS and isinstance(v, dict):
                for vk, vv in v.items():
                    exp[k][vk] = vv
            else:
                exp[k] = v
    for k, v in (cmdargs or {}).items():
        if v is None:
            continue
        if k in ("metadata", "execution") and isinstance(v, dict):
            if not isinstance(exp.get(k), dict):
                exp[k] = {}
            for vk, vv in v.items():
                exp[k][vk] = vv
        else:
            exp[k] = v
    return exp


def to_plain(d):
    """nesteddict -> plain dicts (for storage / comparison)."""
    if isinstance(d, dict):
        return {k: to_plain(v) for k, v in d.items()}
    return d
