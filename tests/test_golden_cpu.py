"""Oracle vs the committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

Re-runs the fp32 CPU oracle on the fixtures' inputs and compares with the stored outputs.  The
oracle is deterministic, but the CPU thread count changes fp32 summation order, so the bar is
rel-L2 <= 1e-5 (not bitwise); the synthetic weights must reproduce their stored checksums exactly
(to 1e-9 relative), otherwise the fixture no longer describes these weights.
"""
import json
import os

import numpy as np
import pytest
import torch

from tests.golden import make_golden as mg

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL = 1e-5


def load(name):
    return dict(np.load(os.path.join(HERE, f"{name}.npz")))


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def test_golden_manifest():
    meta = json.load(open(os.path.join(HERE, "golden.json")))
    assert set(meta["configs"]) == {"r2", "r4", "f1"}
    for name in meta["configs"]:
        g = load(name)
        assert g["v"].dtype == np.float32 and np.isfinite(g["v"]).all() and np.abs(g["v"]).max() > 0


@pytest.mark.parametrize("name", ["r2", "r4", "f1"])
def test_oracle_reproduces_golden(name):
    g = load(name)
    spec = mg.CONFIGS[name]
    sd = mg.weights(spec["cfg"])
    assert np.allclose(mg.weight_checksum(sd), g["weights_checksum"], rtol=1e-9), "synthetic weights changed"
    inp = mg.inputs(name, spec)
    for k, v in inp.items():  # the seeded inputs are the stored ones
        assert np.array_equal(v.numpy(), g[f"in_{k}"]), k
    out = mg.make(name, spec)
    assert rel(out["v"], g["v"]) < TOL
    for k in g:
        if k.startswith(("feat", "z", "img")):
            assert rel(out[k], g[k]) < TOL, k
