"""The repository passes its own dependency-free lint (scripts/lint.py: compiles, no unused
imports, no tabs / trailing whitespace / >120-char lines, no bare except) -- the role of
the reference's flake8/pylint tox environments (tox.ini)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def test_repository_is_lint_clean(capsys):
    import lint
    rc = lint.main([])
    out = capsys.readouterr().out
    assert rc == 0, out
