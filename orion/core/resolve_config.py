"""``orion.core.resolve_config`` (reference `src/orion/core/resolve_config.py:96-297`)
-> :mod:`orion_amd.core.config`."""
from orion_amd.core.config import (  # noqa: F401
    CLI_DOC_HEADER, DEF_CMD_MAX_TRIALS, DEF_CMD_POOL_SIZE, DIRS, ENV_VARS, ENV_VARS_DB,
    default_config_paths, fetch_default_options, fetch_orion_args, is_exe, merge_env_vars,
    merge_orion_config, nesteddict)
