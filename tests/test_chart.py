"""Helm chart sanity without helm: every `.Values.x.y` a template references
exists in values.yaml, and the static YAML files parse."""
import os
import re

import yaml

CHART = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "charts", "vgpu-amd")


def _get(d, path):
    for k in path:
        if not isinstance(d, dict) or k not in d:
            return None, False
        d = d[k]
    return d, True


def test_values_references_exist():
    values = yaml.safe_load(open(os.path.join(CHART, "values.yaml")))
    missing = []
    for root, _, files in os.walk(os.path.join(CHART, "templates")):
        for f in files:
            text = open(os.path.join(root, f)).read()
            for m in re.finditer(r"\.Values\.([A-Za-z0-9_.]+)", text):
                path = m.group(1).rstrip(".").split(".")
                _, ok = _get(values, path)
                if not ok:
                    missing.append((f, m.group(1)))
    assert not missing, missing


def test_chart_yaml():
    c = yaml.safe_load(open(os.path.join(CHART, "Chart.yaml")))
    assert c["apiVersion"] == "v2" and c["name"] == "vgpu-amd"


def test_examples_parse():
    ex = os.path.join(os.path.dirname(CHART), "..", "examples")
    for f in os.listdir(ex):
        docs = list(yaml.safe_load_all(open(os.path.join(ex, f))))
        assert docs and all(d["kind"] == "Pod" for d in docs)
