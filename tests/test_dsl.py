"""Prior DSL and templating (reference: tests/unittests/core/test_space_builder.py)."""
import json

import numpy as np
import pytest
import yaml

from orion_amd.core.trial import Trial
from orion_amd.space import DimensionBuilder, SpaceBuilder


@pytest.fixture
def dimbuilder():
    return DimensionBuilder()


class TestDimensionBuilder:
    def test_uniform_is_a_to_b(self, dimbuilder):
        dim = dimbuilder.build("yolo", "uniform(-3, 5)")
        assert dim.type == "real" and dim.interval() == (-3.0, 5.0)

    def test_uniform_discrete(self, dimbuilder):
        dim = dimbuilder.build("yolo", "uniform(-3, 5, discrete=True)")
        assert dim.type == "integer" and dim.interval() == (-3, 5)

    def test_loguniform_is_reciprocal(self, dimbuilder):
        dim = dimbuilder.build("lr", "loguniform(1e-5, 1)")
        assert dim.prior_name == "reciprocal" and dim.interval() == (1e-5, 1)

    @pytest.mark.parametrize("name", ["gaussian", "normal"])
    def test_normal(self, dimbuilder, name):
        dim = dimbuilder.build("yolo", f"{name}(3, 5)")
        assert dim.prior_name == "norm" and dim.type == "real"

    def test_choices(self, dimbuilder):
        assert dimbuilder.build("y", "choices(['adam', 'sgd'])").categories == ("adam", "sgd")
        assert dimbuilder.build("y", "choices('adam', 'sgd')").categories == ("adam", "sgd")
        d = dimbuilder.build("y", "choices({'a': 0.3, 'b': 0.7})")
        assert d.categories == ("a", "b")

    def test_enum_and_random_aliases(self, dimbuilder):
        assert dimbuilder.build("y", "enum(['a', 'b'])").type == "categorical"
        assert dimbuilder.build("y", "random(-1, 1)").interval() == (-1.0, 1.0)

    def test_scipy_continuous_and_discrete(self, dimbuilder):
        assert dimbuilder.build("y", "alpha(0.9, low=0, high=10)").type == "real"
        assert dimbuilder.build("y", "poisson(mu=3)").type == "integer"

    def test_choices_needs_categories(self, dimbuilder):
        with pytest.raises(TypeError, match="Expected argument with categories"):
            dimbuilder.build("y", "choices()")

    def test_unknown_distribution(self, dimbuilder):
        with pytest.raises(TypeError, match="does not correspond to a supported distribution"):
            dimbuilder.build("y", "lalala(1, 2)")

    def test_bad_form(self, dimbuilder):
        with pytest.raises(TypeError, match="valid form for prior"):
            dimbuilder.build("y", "uniform 1, 2")

    def test_bad_arguments(self, dimbuilder):
        with pytest.raises(TypeError, match="Incorrect arguments"):
            dimbuilder.build("y", "uniform(5, 2)")

    def test_no_code_execution(self, dimbuilder):
        with pytest.raises(RuntimeError, match="literal"):
            dimbuilder.build("y", "uniform(__import__('os').getpid(), 2)")


@pytest.fixture
def yaml_tmpl(tmp_path):
    data = {"yo": 5,
            "training": {"lr0": "orion~loguniform(0.0001, 0.3)",
                         "mbs": "orion~uniform(32, 256, discrete=True)"},
            "layers": [{"width": 64, "type": "relu"},
                       {"width": "orion~uniform(32, 256, discrete=True)",
                        "type": "orion~choices(['relu', 'sigmoid'])"}]}
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(data))
    return str(p)


class TestSpaceBuilder:
    def test_args_only(self):
        sb = SpaceBuilder()
        s = sb.build_from(["-x~uniform(-50, 50)", "--y~normal(0, 1)", "--plain", "5"])
        assert list(s.keys()) == ["/x", "/y"]
        t = Trial(params=[dict(name="/x", type="real", value=3.5), dict(name="/y", type="real", value=-1.0)])
        # parameters render where they stood on the command line (the reference moved them last)
        assert sb.build_to(None, t) == ["-x=3.5", "--y=-1.0", "--plain", "5"]

    def test_config_option(self, yaml_tmpl, tmp_path):
        sb = SpaceBuilder()
        s = sb.build_from([f"--config={yaml_tmpl}", "--seed~choices([1, 2])"])
        assert set(s.keys()) == {"/seed", "/training/lr0", "/training/mbs", "/layers/1/width", "/layers/1/type"}
        params = [dict(name=n, type=s[n].type, value=v) for n, v in
                  (("/layers/1/type", "relu"), ("/layers/1/width", 100), ("/seed", 2),
                   ("/training/lr0", 0.01), ("/training/mbs", 64))]
        out = str(tmp_path / "inst.yaml")
        args = sb.build_to(out, Trial(params=params))
        assert args[0] == "--config=" + out and "--seed=2" in args
        inst = yaml.safe_load(open(out))
        assert inst["training"] == {"lr0": 0.01, "mbs": 64}
        assert inst["layers"][1] == {"width": 100, "type": "relu"} and inst["yo"] == 5

    def test_positional_config(self, yaml_tmpl, tmp_path):
        sb = SpaceBuilder()
        sb.build_from([yaml_tmpl, "--other", "1"])
        assert sb.is_userconfig_an_option is False
        params = [dict(name="/layers/1/type", type="categorical", value="sigmoid"),
                  dict(name="/layers/1/width", type="integer", value=33),
                  dict(name="/training/lr0", type="real", value=0.1),
                  dict(name="/training/mbs", type="integer", value=33)]
        out = str(tmp_path / "x.yaml")
        assert sb.build_to(out, Trial(params=params)) == [out, "--other", "1"]

    def test_json_template(self, tmp_path):
        p = tmp_path / "c.json"
        p.write_text(json.dumps({"a": {"b": "orion~uniform(0, 1)"}, "c": [1, "orion~choices([1, 2])"]}))
        sb = SpaceBuilder()
        s = sb.build_from(["--config=" + str(p)])
        assert set(s) == {"/a/b", "/c/1"}

    def test_conflict(self, tmp_path):
        p = tmp_path / "c.yaml"
        p.write_text(yaml.safe_dump({"x": "orion~uniform(0, 1)"}))
        with pytest.raises(ValueError, match="Conflict"):
            SpaceBuilder().build_from(["-x~uniform(0, 1)", "--config=" + str(p)])

    def test_two_configs(self):
        with pytest.raises(ValueError, match="Already found one configuration file"):
            SpaceBuilder().build_from(["--config=a.yaml", "--config=b.yaml"])

    def test_numpy_values_rendered_plain(self):
        sb = SpaceBuilder()
        sb.build_from(["-x~uniform(0, 1)"])
        t = Trial(params=[dict(name="/x", type="real", value=np.float64(0.25))])
        assert sb.build_to(None, t) == ["-x=0.25"]


def test_template_is_immutable_and_render_is_pure(tmp_path):
    from orion_amd.space.dsl import Hole, ScriptTemplate
    p = tmp_path / "c.yaml"
    p.write_text(yaml.safe_dump({"opt": {"lr": "orion~loguniform(1e-4, 1e-1)"}, "keep": [1, 2]}))
    tmpl = ScriptTemplate.parse(["pos0", "--config=" + str(p), "-x~uniform(0, 1)", "tail"])
    assert tmpl.argv == ("pos0", Hole("/x", "-x"), "tail")
    assert list(tmpl.space) == ["/x", "/opt/lr"]
    with pytest.raises(Exception):
        tmpl.argv = ()
    t = Trial(params=[dict(name="/x", type="real", value=0.5), dict(name="/opt/lr", type="real", value=0.01)])
    a = tmpl.render(t, str(tmp_path / "a.yaml"))
    b = tmpl.render(t, str(tmp_path / "b.yaml"))
    assert a[1:] == b[1:] == ["pos0", "-x=0.5", "tail"]
    assert yaml.safe_load(open(tmp_path / "a.yaml")) == {"opt": {"lr": 0.01}, "keep": [1, 2]}
    # the template document itself is untouched by rendering
    assert tmpl.config_doc["opt"]["lr"].startswith("orion~")
