#!/usr/bin/env python3
"""Dependency-free lint for the Python sources (no flake8/pylint in this image; the
reference runs them from tox.ini).  Checks, per file:

* it compiles;
* no unused imports (module-level ``import x`` / ``from m import x`` whose bound name is
  never referenced; ``__init__.py`` re-exports, ``__all__`` members and ``# noqa`` lines
  are exempt);
* no tabs, no trailing whitespace, lines <= 120 characters;
* no bare ``except:``.

usage: python scripts/lint.py [paths...]   (default: orion_amd orion bin scripts tests *.py)
Exit status 1 with one line per finding.
"""
from __future__ import annotations

import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = ["orion_amd", "orion", "bin", "scripts", "tests", "bench.py", "train.py", "sample.py",
           "__graft_entry__.py"]
MAX_LINE = 120


def py_files(paths):
    for p in paths:
        p = os.path.join(ROOT, p) if not os.path.isabs(p) else p
        if os.path.isfile(p):
            if p.endswith(".py") or (os.path.basename(os.path.dirname(p)) == "bin"):
                yield p
            continue
        for d, dirs, files in os.walk(p):
            dirs[:] = [x for x in dirs if not x.startswith((".", "__pycache__"))]
            for f in files:
                if f.endswith(".py"):
                    yield os.path.join(d, f)
                elif os.path.basename(d) == "bin" and not f.startswith("."):
                    yield os.path.join(d, f)


def _names_used(tree):
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            base = node
            while isinstance(base, ast.Attribute):
                base = base.value
            if isinstance(base, ast.Name):
                used.add(base.id)
    return used


def _all_names(tree):
    out = set()
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__"
                                                for t in node.targets):
            if isinstance(node.value, (ast.List, ast.Tuple)):
                out |= {e.value for e in node.value.elts if isinstance(e, ast.Constant)}
    return out


def lint_file(path):
    rel = os.path.relpath(path, ROOT)
    try:
        src = open(path, encoding="utf-8").read()
    except UnicodeDecodeError:
        return []
    if path.endswith("bin/orion") or "/bin/" in path:
        if not src.startswith("#!") or "python" not in src.splitlines()[0]:
            return []
    out = []
    try:
        tree = ast.parse(src, filename=path)
    except SyntaxError as e:
        return [f"{rel}:{e.lineno}: syntax error: {e.msg}"]
    lines = src.splitlines()
    for i, line in enumerate(lines, 1):
        if "\t" in line:
            out.append(f"{rel}:{i}: tab character")
        if line != line.rstrip():
            out.append(f"{rel}:{i}: trailing whitespace")
        if len(line) > MAX_LINE:
            out.append(f"{rel}:{i}: line longer than {MAX_LINE} ({len(line)})")
    for node in ast.walk(tree):
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            out.append(f"{rel}:{node.lineno}: bare except")
    if os.path.basename(path) != "__init__.py":
        used = _names_used(tree) | _all_names(tree)
        for node in tree.body:
            if not isinstance(node, (ast.Import, ast.ImportFrom)):
                continue
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            if "noqa" in lines[node.lineno - 1]:
                continue
            for alias in node.names:
                name = (alias.asname or alias.name).split(".")[0]
                if name != "*" and name not in used:
                    out.append(f"{rel}:{node.lineno}: unused import {alias.name}")
    return out


def main(argv=None):
    paths = (argv if argv is not None else sys.argv[1:]) or DEFAULT
    findings = []
    for f in sorted(set(py_files(paths))):
        findings += lint_file(f)
    for x in findings:
        print(x)
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main())
