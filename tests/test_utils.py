"""C14 utilities: Registry (plugin factory) and SingletonType."""
import pytest

from orion_amd.utils import Registry, SingletonType
from orion_amd.store import Database, backend_names
from orion_amd.io.convert import Converter, JSONConverter
from orion_amd.algo.base import OptimizationAlgorithm, BaseAlgorithm


def test_registry_case_insensitive_and_aliases():
    reg = Registry("Thing")

    @reg.register(aliases=("alias",))
    class FooBar:
        def __init__(self, x=1):
            self.x = x

    assert reg.create("foobar", x=3).x == 3
    assert isinstance(reg.create("FOOBAR"), FooBar)
    assert isinstance(reg.create("alias"), FooBar)
    assert "FooBar" in reg and "nope" not in reg
    assert reg.types == [FooBar]
    with pytest.raises(NotImplementedError, match="type = 'nope'"):
        reg.create("nope")


def test_singleton_type():
    class S(metaclass=SingletonType):
        def __init__(self, v=0):
            self.v = v

    a = S(5)
    assert S() is a and a.v == 5
    with pytest.raises(ValueError):
        S(6)
    S.reset()
    assert S(7).v == 7


def test_factories_use_registries(tmp_path):
    assert {"sqlite", "memory", "mongodb"} <= set(backend_names())
    db = Database("MemoryDB")
    db.write("c", {"a": 1})
    assert db.count("c") == 1
    assert isinstance(Converter("jsonconverter"), JSONConverter)
    assert "random" in OptimizationAlgorithm.typenames
    assert all(issubclass(t, BaseAlgorithm) for t in OptimizationAlgorithm.types)
    with pytest.raises(NotImplementedError):
        Database("nosuchdb")


def test_third_party_algorithm_plugin_discovery(tmp_path):
    """Reference parity (tests/functional/gradient_descent_algo, installed by tox): an
    algorithm shipped by ANOTHER distribution is found through the `OptimizationAlgorithm`
    entry-point group.  A minimal installed distribution (module + .dist-info with
    entry_points.txt) is put on sys.path of a fresh interpreter."""
    import os
    import subprocess
    import sys
    import textwrap
    (tmp_path / "stub_orion_plugin.py").write_text(textwrap.dedent('''
        from orion_amd.algo.base import BaseAlgorithm

        class StubAlgo(BaseAlgorithm):
            def suggest(self, num=1):
                return [tuple(0.5 for _ in self.space)] * num

            def observe(self, points, results):
                pass
    '''))
    di = tmp_path / "stub_orion_plugin-0.1.dist-info"
    di.mkdir()
    (di / "METADATA").write_text("Metadata-Version: 2.1\nName: stub-orion-plugin\nVersion: 0.1\n")
    (di / "entry_points.txt").write_text("[OptimizationAlgorithm]\nstubalgo = stub_orion_plugin:StubAlgo\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent('''
        from orion.algo.base import OptimizationAlgorithm
        from orion_amd.space import Space, Real
        space = Space()
        space.register(Real("/x", "uniform", 0, 1))
        algo = OptimizationAlgorithm("stubalgo", space)
        print(type(algo).__name__, algo.suggest(2), "stubalgo" in OptimizationAlgorithm.typenames)
    ''')
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([str(tmp_path), root]))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split()[0] == "StubAlgo" and out.stdout.strip().endswith("True"), out.stdout
