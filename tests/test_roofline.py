"""scripts/roofline.py: the flagship's kernel plan counts the known ResNet-50
work (4.09 GMAC per 224² image) and its bound is a real lower bound of the
measured step."""
import importlib.util
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mod():
    spec = importlib.util.spec_from_file_location("roofline", os.path.join(REPO, "scripts", "roofline.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_resnet50_flops_at_224():
    r = _mod()
    gflop = sum(k[1] for k in r.plan(1, 224)) / 1e9
    assert abs(gflop - 8.18) < 0.05, gflop


def test_flagship_bound_below_measured(capsys):
    r = _mod()
    r.main(["--json", "--measured-ms", "3.95"])
    import json
    d = json.loads(capsys.readouterr().out)
    assert 0 < d["fraction_of_speed_of_light"] < 1
    assert 5.0 < d["hbm_gb_per_forward"] < 7.0 and 19.5 < d["gflop_per_image"] < 20.5
