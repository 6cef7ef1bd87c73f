"""The ``~`` prior DSL and user-script templating (component C11).

Parity with ``src/orion/core/io/space_builder.py``:

* command-line priors:  ``-x~'uniform(-50, 50)'``  ->  dimension ``/x``;
  rendered back as ``-x=<value>`` (``space_builder.py:291-328, 372-389``);
* config-file priors: string values ``'orion~loguniform(1e-5, 1)'`` anywhere in
  a YAML/JSON template -> dimension ``/path/to/key`` (list indices included);
  the template is re-rendered per trial (``space_builder.py:263-289, 347-370``);
* ``--config=<path>`` or the first positional argument names the template;
* prior names: ``uniform(a, b)`` = U[a, b) (NOT scipy's loc/scale),
  ``normal``/``gaussian``, ``loguniform`` (scipy ``reciprocal``),
  ``choices(...)``, ``discrete=True`` -> Integer, and any scipy.stats
  continuous (Real) or discrete (Integer) distribution by name.

MI355X-build deviations (documented in SURVEY.md §5.1):

* the expression is parsed with :mod:`ast` and only literal arguments are
  accepted -- no ``eval`` (item 7);
* builders are plain objects owned by the experiment, not process singletons
  (item 1);
* ``enum(...)`` (alias of ``choices``) and ``random(...)`` (alias of
  ``uniform``) are implemented (reference docstring promised them,
  ``space_builder.py:86-104``).
"""
from __future__ import annotations

import ast
import collections
import copy
import logging
import os
import re

from scipy.stats import distributions as sp_dists

from .dimensions import Categorical, Integer, Real, Space
from ..io.convert import infer_converter_from_file_type

log = logging.getLogger(__name__)


def _real_or_int(kwargs):
    return Integer if kwargs.pop("discrete", False) else Real


def _parse_call(expression):
    """'name(arg, k=v)' -> (name, args, kwargs) with literal arguments only."""
    try:
        node = ast.parse(expression.strip(), mode="eval").body
    except SyntaxError as exc:
        raise IndexError(expression) from exc
    if not isinstance(node, ast.Call) or not isinstance(node.func, ast.Name):
        raise IndexError(expression)
    try:
        args = tuple(ast.literal_eval(a) for a in node.args)
        kwargs = {kw.arg: ast.literal_eval(kw.value) for kw in node.keywords}
    except (ValueError, SyntaxError) as exc:
        raise RuntimeError(f"Only literal arguments are allowed in a prior: {expression!r}") from exc
    if any(k is None for k in kwargs):
        raise RuntimeError(f"**kwargs expansion is not allowed in a prior: {expression!r}")
    return node.func.id, args, kwargs


class DimensionBuilder:
    """Build a :class:`Dimension` from ``name`` and a prior expression string."""

    def __init__(self):
        self.name = None

    # ------------------------------------------------------------ prior constructors
    def choices(self, *args, **kwargs):
        name = self.name
        if not args:
            raise TypeError("Parameter '{}': Expected argument with categories.".format(name))
        if isinstance(args[0], (dict, list, tuple)) and len(args) == 1:
            return Categorical(name, *args, **kwargs)
        return Categorical(name, args, **kwargs)

    enum = choices

    def uniform(self, *args, **kwargs):
        """U[a, b) -- note: NOT scipy's (loc, scale) convention."""
        klass = _real_or_int(kwargs)
        if len(args) == 2:
            return klass(self.name, "uniform", args[0], args[1] - args[0], **kwargs)
        return klass(self.name, "uniform", *args, **kwargs)

    random = uniform

    def gaussian(self, *args, **kwargs):
        return self.normal(*args, **kwargs)

    def normal(self, *args, **kwargs):
        klass = _real_or_int(kwargs)
        return klass(self.name, "norm", *args, **kwargs)

    def loguniform(self, *args, **kwargs):
        klass = _real_or_int(kwargs)
        return klass(self.name, "reciprocal", *args, **kwargs)

    _BUILTIN = ("choices", "enum", "uniform", "random", "gaussian", "normal", "loguniform")

    # ------------------------------------------------------------ build
    def _build(self, name, expression):
        self.name = name
        prior, args, kwargs = _parse_call(expression)
        if prior in self._BUILTIN:
            return getattr(self, prior)(*args, **kwargs)
        if hasattr(sp_dists._continuous_distns, prior):
            klass = _real_or_int(kwargs)
        elif hasattr(sp_dists._discrete_distns, prior):
            klass = Integer
        else:
            raise TypeError("Parameter '{0}': '{1}' does not correspond to a supported "
                            "distribution.".format(name, prior))
        return klass(name, prior, *args, **kwargs)

    def build(self, name, expression):
        try:
            dim = self._build(name, expression)
        except ValueError as exc:
            raise TypeError("Parameter '{}': Incorrect arguments.".format(name)) from exc
        except IndexError as exc:
            raise TypeError("Parameter '{0}': Please provide a valid form for prior:\n"
                            "'distribution(*args, **kwargs)'\nProvided: '{1}'".format(
                                name, expression)) from exc
        try:  # warm-up: fail early on unusable arguments
            dim.sample()
        except TypeError as exc:
            raise TypeError("Parameter '{0}': Incorrect arguments for distribution '{1}'.\n"
                            "Scipy Docs::\n\n{2}".format(name, dim.prior_name,
                                                         dim.prior.__doc__)) from exc
        except ValueError as exc:
            raise TypeError("Parameter '{0}': Incorrect arguments.".format(name)) from exc
        return dim


class SpaceBuilder:
    """Build a :class:`Space` from a user's command line (and config template), and
    render concrete command lines / config files for trials."""

    USERCONFIG_OPTION = "--config="
    USERCONFIG_KEYWORD = "orion~"
    USERARGS_SEARCH = r"\W*([a-zA-Z0-9_-]+)~(.*)"
    USERARGS_TMPL = r"(.*)~(.*)"

    def __init__(self):
        self.userconfig = None
        self.is_userconfig_an_option = None
        self.userargs_tmpl = None
        self.userconfig_tmpl = None
        self.dimbuilder = DimensionBuilder()
        self.space = None
        self.converter = None

    def build_from(self, cmd_args):
        """Parse ``cmd_args`` (list of str) into a :class:`Space`."""
        self.userargs_tmpl = None
        self.userconfig_tmpl = None
        self.space = Space()
        self.userconfig, self.is_userconfig_an_option = self._build_from_args(cmd_args)
        if self.userconfig:
            self._build_from_config(self.userconfig)
        log.debug("Built search space:\n%s", self.space)
        return self.space

    def _build_from_config(self, config_path):
        self.converter = infer_converter_from_file_type(config_path)
        self.userconfig_tmpl = self.converter.parse(config_path)
        stack = collections.deque([("", self.userconfig_tmpl)])
        while stack:
            namespace, stuff = stack.pop()
            if isinstance(stuff, dict):
                for k, v in stuff.items():
                    stack.append(("/".join([namespace, str(k)]), v))
            elif isinstance(stuff, list):
                for pos, thing in enumerate(stuff):
                    stack.append(("/".join([namespace, str(pos)]), thing))
            elif isinstance(stuff, str) and stuff.startswith(self.USERCONFIG_KEYWORD):
                dim = self.dimbuilder.build(namespace, stuff[len(self.USERCONFIG_KEYWORD):])
                try:
                    self.space.register(dim)
                except ValueError as exc:
                    raise ValueError("Conflict for name '{}' in script configuration "
                                     "and arguments.".format(namespace)) from exc

    def _build_from_args(self, cmd_args):
        userconfig = None
        is_option = None
        self.userargs_tmpl = collections.defaultdict(list)
        pat = re.compile(self.USERARGS_SEARCH)
        prefix_pat = re.compile(self.USERARGS_TMPL)
        for arg in cmd_args:
            found = pat.findall(arg)
            if len(found) != 1:
                if arg.startswith(self.USERCONFIG_OPTION):
                    if userconfig:
                        raise ValueError("Already found one configuration file in: %s" % userconfig)
                    userconfig = arg[len(self.USERCONFIG_OPTION):]
                    is_option = True
                else:
                    self.userargs_tmpl[None].append(arg)
                continue
            name, expression = found[0]
            namespace = "/" + name
            self.space.register(self.dimbuilder.build(namespace, expression))
            pref = prefix_pat.findall(arg)
            assert len(pref) == 1 and pref[0][1] == expression, "Parsing prefix problem."
            self.userargs_tmpl[namespace] = pref[0][0] + "="
        if not userconfig and self.userargs_tmpl[None]:
            if os.path.isfile(self.userargs_tmpl[None][0]):
                userconfig = self.userargs_tmpl[None].pop(0)
                is_option = False
        return userconfig, is_option

    # ------------------------------------------------------------ rendering
    def build_to(self, config_path, trial):
        """Write the trial's config file (if templated) and return its command-line args."""
        if self.userconfig:
            self._build_to_config(config_path, trial)
        return self._build_to_args(config_path, trial)

    def _build_to_config(self, config_path, trial):
        inst = copy.deepcopy(self.userconfig_tmpl)
        for param in trial.params:
            stuff = inst
            for key in param.name.split("/")[1:]:
                if isinstance(stuff, list):
                    key = int(key)
                    if key >= len(stuff):
                        break
                elif key not in stuff:
                    break
                if isinstance(stuff[key], str):
                    stuff[key] = _plain(param.value)
                else:
                    stuff = stuff[key]
        self.converter.generate(config_path, inst)

    def _build_to_args(self, config_path, trial):
        out = []
        if self.userconfig:
            out.append(self.USERCONFIG_OPTION + config_path if self.is_userconfig_an_option
                       else config_path)
        out.extend(self.userargs_tmpl[None])
        for param in trial.params:
            if param.name in self.userargs_tmpl:
                out.append(self.userargs_tmpl[param.name] + str(_plain(param.value)))
        return out


def _plain(v):
    """numpy scalars/arrays -> plain Python for YAML/JSON/CLI rendering."""
    if hasattr(v, "tolist"):
        return v.tolist()
    return v
