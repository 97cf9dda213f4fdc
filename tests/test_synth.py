"""The native cluster generator (csrc/synth.cpp, ksg_synth_cluster) builds the
same document as the Python generator (ksg/generator.py) for configs 2..5: the
full-size GPU tests and benchmarks use it, the goldens and the smaller tests use
the Python one.  CPU only (libksg.so loads; nothing runs on a device)."""
import json

import pytest

from ksg import generator as g

CASES = [
    (2, dict(n_nodes=300, n_pods=200)),
    (3, dict(n_nodes=200, n_pods=150)),
    (4, dict(n_nodes=120, n_existing=500, n_pods=150, n_zones=6)),
    (4, dict(n_nodes=90, n_existing=200, n_pods=40, n_zones=20)),
    (5, dict(n_nodes=400, n_pods=96)),
]


@pytest.mark.parametrize("c,sizes", CASES, ids=[f"cfg{c}-{i}" for i, (c, _) in enumerate(CASES)])
def test_native_generator_matches_python(c, sizes):
    want = g.generate(c, **sizes)
    got = json.loads(g.generate_native(c, **sizes))
    assert got["profile"] == want["profile"]
    for k in ("nodes", "pods", "queue"):
        assert len(got[k]) == len(want[k]), k
        for i, (a, b) in enumerate(zip(got[k], want[k])):
            assert a == b, (k, i, a, b)


def test_native_generator_defaults_and_seed():
    a = json.loads(g.generate_native(2, n_nodes=50, n_pods=10, seed=12345))
    b = g.generate(2, n_nodes=50, n_pods=10, seed=12345)
    assert a == b
