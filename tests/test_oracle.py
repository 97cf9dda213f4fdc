"""CPU tests of the oracle (oracle/ksg_oracle.cpp) against the reference's own
known answers and the committed golden fixtures; Go math.Log restatement."""
import glob
import json
import math
import os
import struct

import pytest

from _oracle import Oracle, go_log
from ksg import generator as g

HERE = os.path.dirname(os.path.abspath(__file__))
ANN = "kube-scheduler-simulator.sigs.k8s.io/"


def fixture(name):
    with open(os.path.join(HERE, "golden", name + ".json")) as f:
        return json.load(f)


def run(doc):
    o = Oracle(doc)
    o.schedule(record=3)
    return o


def test_readme_known_answer():
    """README.md:63-80 / debuggable-scheduler.md:13-31: Fit 73, BA 76, Taint finalscore 300, raw 0."""
    o = run(fixture("readme_example")["cluster"])
    a = o.annotations(0)
    fin = json.loads(a[ANN + "finalscore-result"])
    raw = json.loads(a[ANN + "score-result"])
    for node in ("node-282x7", "node-gp9t4"):
        assert fin[node]["NodeResourcesFit"] == "73"
        assert fin[node]["NodeResourcesBalancedAllocation"] == "76"
        assert fin[node]["TaintToleration"] == "300"
        assert raw[node]["TaintToleration"] == "0"
    assert a[ANN + "selected-node"] in ("node-282x7", "node-gp9t4")


def test_plugin_extender_known_answer():
    """plugin-extender.md:85-107: node-282x7 (already hosting a {100m, 16Gi} pod) scores
    Fit 47 / BalancedAllocation 52, node-gp9t4 73 / 76, TaintToleration 300 on both,
    and node-gp9t4 is selected — Requested / NonZeroRequested after an assume, BA on a
    loaded node."""
    o = run(fixture("plugin_extender_example")["cluster"])
    a = o.annotations(0)
    fin = json.loads(a[ANN + "finalscore-result"])
    raw = json.loads(a[ANN + "score-result"])
    want = {"node-282x7": ("47", "52"), "node-gp9t4": ("73", "76")}
    for node, (fit, ba) in want.items():
        assert raw[node]["NodeResourcesFit"] == fin[node]["NodeResourcesFit"] == fit
        assert raw[node]["NodeResourcesBalancedAllocation"] == fin[node]["NodeResourcesBalancedAllocation"] == ba
        assert fin[node]["TaintToleration"] == "300"
    assert a[ANN + "selected-node"] == "node-gp9t4"
    assert o.result(0)[0] == 1


def test_store_weight_semantics():
    """store_test.go:284-446 finalscore = score x weight (10 x 2 = "20"); plugins.go:289-304 weight 0 -> 1."""
    a = run(fixture("store_weight_example")["cluster"]).annotations(0)
    fin = json.loads(a[ANN + "finalscore-result"])
    raw = json.loads(a[ANN + "score-result"])
    assert raw["node-0"]["NodeResourcesFit"] == "10" and fin["node-0"]["NodeResourcesFit"] == "20"
    assert raw["node-0"]["NodeResourcesBalancedAllocation"] == fin["node-0"]["NodeResourcesBalancedAllocation"]


def test_empty_maps_render_as_braces():
    """store_test.go:584-833: empty maps are "{}"; one feasible node => no PreScore/Score."""
    a = run(fixture("empty_maps_example")["cluster"]).annotations(0)
    for k in ("score-result", "finalscore-result", "prescore-result", "postfilter-result", "permit-result",
              "permit-result-timeout", "reserve-result", "prebind-result", "bind-result", "prefilter-result"):
        assert a[ANN + k] == "{}", k
    assert a[ANN + "selected-node"] == "node-b"
    f = json.loads(a[ANN + "filter-result"])
    assert f["node-a"]["NodeResourcesFit"] == "Insufficient cpu, Insufficient memory"


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "golden", "*.json"))),
                         ids=lambda p: os.path.basename(p)[:-5])
def test_oracle_reproduces_golden(path):
    d = json.load(open(path))
    o = run(d["cluster"])
    for q, e in enumerate(d["expected"]):
        assert o.result(q) == (e["selected"], e["feasible"], e["status"]), q
        assert o.annotations(q) == e["annotations"], q
        n = e.get("nominated")
        assert o.nominated(q) == ((n["node"], n["victims"]) if n else (-1, [])), q


def test_golden_families_match_generator():
    """The committed cfg fixtures are exactly what the seeded generator produces."""
    for name in ("cfg1_small", "cfg2_small", "cfg3_small", "cfg4_small"):
        d = fixture(name)
        assert g.generate(d["config"], **d["sizes"]) == d["cluster"], name
    from ksg import edge
    for name in ("edge_fit_most_small", "edge_fit_rtc_small", "edge_na_small", "edge_pts_small", "edge_ipa_small",
                 "edge_ipa_ignore_small", "edge_preempt_small", "edge_volumes_small", "edge_queue_small"):
        d = fixture(name)
        assert edge.generate_edge(d["edge"], **d["sizes"]) == d["cluster"], name


def test_queue_entry_semantics():
    """SchedulingGates' PreEnqueue keeps gated pods out of the queue; activeQ pops in
    PrioritySort order (higher spec.priority first, then arrival = document order);
    "queueSort": false models pods arriving one at a time (arrival order).  Hand-worked:
    A(0) B(100, gated) C(100) D(10) -> [C, D, A], gated [B]."""
    gates = [{"name": "example.com/hold"}]
    pods = [g.pod_obj("a", [g.req(100, 64 * g.Mi)], priority=0),
            g.pod_obj("b", [g.req(100, 64 * g.Mi)], priority=100, schedulingGates=gates),
            g.pod_obj("c", [g.req(100, 64 * g.Mi)], priority=100),
            g.pod_obj("d", [g.req(100, 64 * g.Mi)], priority=10)]
    nodes = [g.node_obj("node-0", 4000, 8 * g.Gi)]
    full = g.make_profile(g.DEFAULT_PROFILE, 1)
    o = Oracle({"profile": full, "nodes": nodes, "pods": [], "queue": pods})
    assert o.queue_names() == ["default/c", "default/d", "default/a"]
    assert o.gated_names() == ["default/b"]
    # the ResourcesForSnap form: pending pods among the bound ones
    snap = {"profile": full, "nodes": nodes, "pods": [pods[0], g.pod_obj("x", [], node="node-0")] + pods[1:]}
    assert Oracle(snap).queue_names() == ["default/c", "default/d", "default/a"]
    o = Oracle({"profile": full, "nodes": nodes, "pods": [], "queue": pods, "queueSort": False})
    assert o.queue_names() == ["default/a", "default/c", "default/d"]
    hot = g.make_profile(g.DEFAULT_HOT_PROFILE, 1)  # no SchedulingGates: nothing is held back
    o = Oracle({"profile": hot, "nodes": nodes, "pods": [], "queue": pods})
    assert o.queue_names() == ["default/b", "default/c", "default/d", "default/a"] and o.gated_names() == []
    o.schedule(record=3)
    assert all(o.result(q)[2] == 0 for q in range(4))


def _py_go_log(x):
    """Independent Python restatement of Go's math.Log (src/math/log.go)."""
    L = [6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01,
         2.222219843214978396e-01, 1.818357216161805012e-01, 1.531383769920937332e-01,
         1.479819860511658591e-01]
    f1, ki = math.frexp(x)
    if f1 < math.sqrt(2) / 2:
        f1 *= 2
        ki -= 1
    f = f1 - 1
    k = float(ki)
    s = f / (2 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (L[0] + s4 * (L[2] + s4 * (L[4] + s4 * L[6])))
    t2 = s4 * (L[1] + s4 * (L[3] + s4 * L[5]))
    R = t1 + t2
    hfsq = 0.5 * f * f
    return k * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + k * 1.90821492927058770002e-10)) - f)


def _bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def test_go_log_restatement():
    diffs = 0
    for n in range(2, 20002):
        a, b = go_log(float(n)), _py_go_log(float(n))
        assert _bits(a) == _bits(b), n
        assert abs(_bits(a) - _bits(math.log(n))) <= 1
        diffs += _bits(a) != _bits(math.log(n))
    # Go's algorithm is not libm's: SURVEY.md Appendix C found 9,447 differing integers in [3, 1,000,002]
    assert diffs > 0


def test_tiebreak_hash_matches_generator_twin():
    o = Oracle(fixture("cfg2_small")["cluster"])
    seed = fixture("cfg2_small")["cluster"]["profile"]["seed"]
    from _oracle import lib
    for q, n, total in [(0, 0, 5), (7, 3, 199), (123, 29, 0)]:
        key = lib().ksg_oracle_pack_key(o.h, total, q, n)
        h20 = g.tiebreak_h20(seed, q, n)
        assert key == (total << 40) | ((0xFFFFF - h20) << 20) | n


def test_config_profile_store_weight_quirk():
    """scheduler_test.go:344-407 through the whole recording: a KubeSchedulerConfiguration
    with Score.Enabled NodeResourcesFit weight 3 and MultiPoint weight 2.  The store's
    finalscore is raw x 2 (getScorePluginWeight, plugins.go:289-304) while the framework
    sums raw x 3 (getScoreWeights); same results as the flat profile with those maps."""
    cl = fixture("plugin_extender_example")["cluster"]
    flat = cl["profile"]
    mp = [(n, 2 if n == "NodeResourcesFit" else flat["weights"].get(n, 1)) for n in flat["plugins"]]
    cfg = dict(cl, profile=g.config_profile(mp, flat["seed"], score=[("NodeResourcesFit", 3)]))
    a = run(cfg).annotations(0)
    fin = json.loads(a[ANN + "finalscore-result"])
    assert fin["node-282x7"]["NodeResourcesFit"] == "94" and fin["node-gp9t4"]["NodeResourcesFit"] == "146"
    assert a[ANN + "selected-node"] == "node-gp9t4"
    both = json.loads(json.dumps(cl))
    both["profile"]["weights"]["NodeResourcesFit"], both["profile"]["storeWeights"]["NodeResourcesFit"] = 3, 2
    assert run(both).annotations(0) == a
