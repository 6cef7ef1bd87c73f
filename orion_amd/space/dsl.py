"""The ``~`` prior DSL and the per-trial script template (component C11).

Behaviour kept from the reference (``src/orion/core/io/space_builder.py``):

* a command-line token ``-x~'uniform(-50, 50)'`` declares dimension ``/x`` and is
  rendered for a trial as ``-x=<value>`` (``space_builder.py:291-328, 372-389``);
* a string value ``'orion~loguniform(1e-5, 1)'`` anywhere inside a YAML/JSON
  config template declares dimension ``/path/to/key`` (list positions included);
  each trial gets its own rendered copy of the file (``space_builder.py:263-289,
  347-370``);
* the template is named by ``--config=<path>`` or is the first positional argument
  when that is an existing file;
* prior names: ``uniform(a, b)`` = U[a, b) (not scipy's loc/scale), ``normal`` /
  ``gaussian``, ``loguniform`` (scipy ``reciprocal``), ``choices(...)``,
  ``discrete=True`` -> :class:`Integer`, and any scipy.stats distribution by name
  (continuous -> Real, discrete -> Integer); the error messages are the
  reference's, so tooling that matches on them keeps working.

Design (this framework's own):

* :func:`parse_prior` turns an expression into a dimension through a table of
  prior constructors; the call is parsed with :mod:`ast`, arguments must be
  literals (no ``eval``);
* :class:`ScriptTemplate` is an immutable value built once by
  :meth:`ScriptTemplate.parse` and owned by the experiment.  The command line is
  kept as a tuple of tokens -- literal strings and parameter *holes* -- in the
  user's original order, and the config template as a parsed document plus the
  paths of its holes.  :meth:`ScriptTemplate.render` is a pure function of the
  trial (it writes only the file it is given).  No process-wide singletons.
* deviation: holes render at their original position in the command line (the
  reference moved every parameter after all other arguments); positional
  arguments therefore keep their place relative to the parameters.
* ``enum(...)`` (= ``choices``) and ``random(...)`` (= ``uniform``), promised by the
  reference's docstring (``space_builder.py:86-104``) but never implemented, exist.

:class:`DimensionBuilder` and :class:`SpaceBuilder` are the reference-shaped entry
points (``build(name, expr)``, ``build_from(argv)`` / ``build_to(path, trial)``)
over the same machinery.
"""
from __future__ import annotations

import ast
import copy
import logging
import os
import re
from dataclasses import dataclass, field
from typing import Any

from scipy.stats import distributions as sp_dists

from .dimensions import Categorical, Dimension, Integer, Real, Space
from ..io.convert import infer_converter_from_file_type

log = logging.getLogger(__name__)

CONFIG_FLAG = "--config="
CONFIG_MARKER = "orion~"
# a command-line token declaring a dimension: optional dashes, a name, '~', the prior
_ARG_PRIOR = re.compile(r"^(?P<prefix>\W*(?P<name>[A-Za-z0-9_-]+))~(?P<expr>.*)$")


# ============================================================================ priors
class _BadForm(Exception):
    """The expression is not ``name(args...)``."""


def _call_of(expression: str):
    """'name(a, k=v)' -> (name, args, kwargs); literal arguments only."""
    try:
        node = ast.parse(expression.strip(), mode="eval").body
    except SyntaxError as exc:
        raise _BadForm(expression) from exc
    if not (isinstance(node, ast.Call) and isinstance(node.func, ast.Name)):
        raise _BadForm(expression)
    if any(kw.arg is None for kw in node.keywords) or any(isinstance(a, ast.Starred) for a in node.args):
        raise RuntimeError(f"Only literal arguments are allowed in a prior: {expression!r}")
    try:
        args = [ast.literal_eval(a) for a in node.args]
        kwargs = {kw.arg: ast.literal_eval(kw.value) for kw in node.keywords}
    except (ValueError, SyntaxError) as exc:
        raise RuntimeError(f"Only literal arguments are allowed in a prior: {expression!r}") from exc
    return node.func.id, args, kwargs


def _numeric_kind(kwargs):
    """Real, or Integer when the prior carries ``discrete=True`` (consumed here)."""
    return Integer if kwargs.pop("discrete", False) else Real


def _prior_uniform(name, args, kwargs):
    kind = _numeric_kind(kwargs)
    if len(args) == 2:  # U[low, high): scipy wants (loc=low, scale=high-low)
        low, high = args
        return kind(name, "uniform", low, high - low, **kwargs)
    return kind(name, "uniform", *args, **kwargs)


def _prior_normal(name, args, kwargs):
    return _numeric_kind(kwargs)(name, "norm", *args, **kwargs)


def _prior_loguniform(name, args, kwargs):
    return _numeric_kind(kwargs)(name, "reciprocal", *args, **kwargs)


def _prior_choices(name, args, kwargs):
    if not args:
        raise TypeError("Parameter '{}': Expected argument with categories.".format(name))
    if len(args) == 1 and isinstance(args[0], (dict, list, tuple)):
        return Categorical(name, args[0], **kwargs)
    return Categorical(name, tuple(args), **kwargs)


PRIORS = {
    "uniform": _prior_uniform, "random": _prior_uniform,
    "normal": _prior_normal, "gaussian": _prior_normal,
    "loguniform": _prior_loguniform,
    "choices": _prior_choices, "enum": _prior_choices,
}


def _scipy_prior(name, prior, args, kwargs):
    if hasattr(sp_dists._continuous_distns, prior):
        return _numeric_kind(kwargs)(name, prior, *args, **kwargs)
    if hasattr(sp_dists._discrete_distns, prior):
        return Integer(name, prior, *args, **kwargs)
    raise TypeError("Parameter '{0}': '{1}' does not correspond to a supported "
                    "distribution.".format(name, prior))


def parse_prior(name: str, expression: str) -> Dimension:
    """Dimension ``name`` with the prior written in ``expression`` (e.g. ``uniform(0, 1)``).
    Every failure is a ``TypeError`` naming the parameter (``RuntimeError`` for
    non-literal arguments)."""
    try:
        prior, args, kwargs = _call_of(expression)
        ctor = PRIORS.get(prior)
        dim = ctor(name, args, kwargs) if ctor else _scipy_prior(name, prior, args, kwargs)
    except _BadForm as exc:
        raise TypeError("Parameter '{0}': Please provide a valid form for prior:\n"
                        "'distribution(*args, **kwargs)'\nProvided: '{1}'".format(name, expression)) from exc
    except ValueError as exc:
        raise TypeError("Parameter '{}': Incorrect arguments.".format(name)) from exc
    # draw once: arguments scipy accepts at construction but cannot sample with fail here
    try:
        dim.sample()
    except TypeError as exc:
        raise TypeError("Parameter '{0}': Incorrect arguments for distribution '{1}'.\n"
                        "Scipy Docs::\n\n{2}".format(name, dim.prior_name, dim.prior.__doc__)) from exc
    except ValueError as exc:
        raise TypeError("Parameter '{0}': Incorrect arguments.".format(name)) from exc
    return dim


# ============================================================================ template
@dataclass(frozen=True)
class Hole:
    """A command-line token that becomes ``<prefix>=<value>`` for each trial."""
    dim: str
    prefix: str


def _walk_leaves(node, path=()):
    """Yield (path, value) for every leaf of a parsed YAML/JSON document, depth first in
    document order; list positions are path components too."""
    if isinstance(node, dict):
        for k, v in node.items():
            yield from _walk_leaves(v, path + (str(k),))
    elif isinstance(node, list):
        for i, v in enumerate(node):
            yield from _walk_leaves(v, path + (str(i),))
    else:
        yield path, node


def _set_leaf(doc, path, value):
    node = doc
    for key in path[:-1]:
        node = node[int(key)] if isinstance(node, list) else node[key]
    last = path[-1]
    if isinstance(node, list):
        node[int(last)] = value
    else:
        node[last] = value


def _plain(v):
    """numpy scalars/arrays -> plain Python for YAML/JSON/CLI rendering."""
    return v.tolist() if hasattr(v, "tolist") else v


@dataclass(frozen=True)
class ScriptTemplate:
    """The user's command line (and optional config file) with the parameters cut out.

    ``argv`` holds ``str`` tokens (passed through) and :class:`Hole` tokens (rendered);
    ``config_path`` / ``config_as_flag`` say where the config template came from and how
    the rendered copy is passed; ``config_doc`` is the parsed template and
    ``config_holes`` maps dimension names to their paths inside it."""

    space: Space
    argv: tuple = ()
    config_path: str | None = None
    config_as_flag: bool = True
    config_doc: Any = None
    config_holes: dict = field(default_factory=dict)

    # ------------------------------------------------------------------ parse
    @classmethod
    def parse(cls, argv) -> "ScriptTemplate":
        space = Space()
        tokens = []
        config_path, as_flag = None, True
        for tok in argv:
            m = _ARG_PRIOR.match(tok)
            if m is not None:
                dim_name = "/" + m.group("name")
                space.register(parse_prior(dim_name, m.group("expr")))
                tokens.append(Hole(dim_name, m.group("prefix")))
            elif tok.startswith(CONFIG_FLAG):
                if config_path:
                    raise ValueError("Already found one configuration file in: %s" % config_path)
                config_path = tok[len(CONFIG_FLAG):]
            else:
                tokens.append(tok)
        if config_path is None:
            first = next((i for i, t in enumerate(tokens) if isinstance(t, str)), None)
            if first is not None and os.path.isfile(tokens[first]):
                config_path, as_flag = tokens.pop(first), False
        doc, holes = None, {}
        if config_path:
            doc = infer_converter_from_file_type(config_path).parse(config_path)
            for path, leaf in _walk_leaves(doc):
                if not (isinstance(leaf, str) and leaf.startswith(CONFIG_MARKER)):
                    continue
                dim_name = "/" + "/".join(path)
                dim = parse_prior(dim_name, leaf[len(CONFIG_MARKER):])
                if dim_name in space:
                    raise ValueError("Conflict for name '{}' in script configuration "
                                     "and arguments.".format(dim_name))
                space.register(dim)
                holes[dim_name] = path
        log.debug("Built search space:\n%s", space)
        return cls(space, tuple(tokens), config_path, as_flag, doc, holes)

    # ------------------------------------------------------------------ render
    def render(self, trial, config_out: str | None = None) -> list:
        """Command-line arguments for ``trial``; with a config template, the trial's
        config file is written to ``config_out`` first."""
        values = {p.name: _plain(p.value) for p in trial.params}
        out = []
        if self.config_path:
            self.render_config(values, config_out)
            out.append(CONFIG_FLAG + config_out if self.config_as_flag else config_out)
        for tok in self.argv:
            if isinstance(tok, Hole):
                if tok.dim in values:
                    out.append(f"{tok.prefix}={values[tok.dim]}")
            else:
                out.append(tok)
        return out

    def render_config(self, values: dict, path: str):
        doc = copy.deepcopy(self.config_doc)
        for dim_name, where in self.config_holes.items():
            if dim_name in values:
                _set_leaf(doc, where, values[dim_name])
        infer_converter_from_file_type(self.config_path).generate(path, doc)


# ============================================================================ entry points
class DimensionBuilder:
    """``build(name, expression) -> Dimension`` (reference ``space_builder.py:69-215``)."""

    def build(self, name, expression):
        return parse_prior(name, expression)


class SpaceBuilder:
    """``build_from(argv) -> Space`` then ``build_to(config_out, trial) -> argv``
    (reference ``space_builder.py:218-389``), backed by one :class:`ScriptTemplate`."""

    def __init__(self):
        self.template: ScriptTemplate | None = None

    def build_from(self, cmd_args):
        self.template = ScriptTemplate.parse(list(cmd_args))
        return self.template.space

    def build_to(self, config_path, trial):
        return self.template.render(trial, config_path)

    @property
    def userconfig(self):
        return self.template.config_path if self.template else None

    @property
    def is_userconfig_an_option(self):
        return None if not self.userconfig else self.template.config_as_flag
