"""Regenerate the golden fixtures under tests/golden/ from the CPU oracle.

Fixtures are data: a small cluster (inputs) and the expected per-pod results
(selected node, feasible count, status, and the result-store annotations the
reference's debuggable scheduler would write).  Run:

    python tests/golden/make_golden.py

Cases pinned to the reference's own known answers are listed in KNOWN (README.md:63-80,
simulator/docs/debuggable-scheduler.md:13-31, resultstore/store_test.go:284-833);
the config families are pinned to the restatement itself ("parity unpinned"
against the Go code).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
sys.path.insert(0, os.path.dirname(HERE))

from ksg import edge  # noqa: E402
from ksg import generator as g  # noqa: E402
from _oracle import Oracle  # noqa: E402


def readme_example():
    """README.md:63-80: pod {100m, 16Gi} on two empty {4, 32Gi} nodes (web templates node.yaml/pod.yaml)."""
    prof = g.make_profile(g.DEFAULT_HOT_PROFILE, 1)
    return {"profile": prof,
            "nodes": [g.node_obj("node-282x7", 4000, 32 * g.Gi), g.node_obj("node-gp9t4", 4000, 32 * g.Gi)],
            "pods": [], "queue": [g.pod_obj("hoge-pod", [g.req(100, 16 * g.Gi)])]}


def store_weight_example():
    """resultstore/store_test.go:284-446: finalscore = score x weight (score 10, weight 2 -> "20");
    plugins.go:289-304: a weight of 0 in the store map becomes 1."""
    prof = g.make_profile([("NodeResourcesFit", 2), ("NodeResourcesBalancedAllocation", 1)], 1)
    prof["storeWeights"]["NodeResourcesBalancedAllocation"] = 0
    nodes = [g.node_obj(f"node-{i}", 10000, 10 * g.Gi) for i in range(2)]
    return {"profile": prof, "nodes": nodes, "pods": [],
            "queue": [g.pod_obj("pod1", [g.req(9000, 9 * g.Gi)])]}


def empty_maps_example():
    """resultstore/store_test.go:584-833: maps with no entries render as "{}" — a single
    feasible node is selected without PreScore/Score (schedule_one.go), so the score maps are empty."""
    prof = g.make_profile(g.DEFAULT_HOT_PROFILE, 1)
    nodes = [g.node_obj("node-a", 1000, 1 * g.Gi), g.node_obj("node-b", 8000, 8 * g.Gi)]
    return {"profile": prof, "nodes": nodes, "pods": [],
            "queue": [g.pod_obj("big", [g.req(4000, 2 * g.Gi)])]}


def plugin_extender_example():
    """simulator/docs/plugin-extender.md:85-107: the same {100m, 16Gi} pod, default
    profile; node-282x7 already hosts one {100m, 16Gi} pod.  Documented results:
    node-282x7 Fit 47 / BalancedAllocation 52, node-gp9t4 Fit 73 / BA 76,
    TaintToleration finalscore 300 on both, selected-node node-gp9t4.  (Its
    PodTopologySpread "200" and all-"passed" filter map predate v1.27's PreFilter
    Skip, SURVEY.md §8(c): not asserted.)"""
    prof = g.make_profile(g.DEFAULT_PROFILE, 1)
    return {"profile": prof,
            "nodes": [g.node_obj("node-282x7", 4000, 32 * g.Gi), g.node_obj("node-gp9t4", 4000, 32 * g.Gi)],
            "pods": [g.pod_obj("pod-running", [g.req(100, 16 * g.Gi)], node="node-282x7")],
            "queue": [g.pod_obj("pod-8ldq5", [g.req(100, 16 * g.Gi)])]}


KNOWN = {"readme_example": readme_example, "store_weight_example": store_weight_example,
         "empty_maps_example": empty_maps_example, "plugin_extender_example": plugin_extender_example}
FAMILIES = {
    "cfg1_small": (1, dict(n_nodes=12, n_pods=24)),
    "cfg2_small": (2, dict(n_nodes=30, n_pods=30)),
    "cfg3_small": (3, dict(n_nodes=40, n_pods=25)),
    "cfg4_small": (4, dict(n_nodes=40, n_existing=120, n_pods=25, n_zones=4)),
}


# edge-case family (ksg/edge.py): plugin arguments and pod / node shapes the configs never make
EDGE = {
    "edge_fit_most_small": ("fit_most", dict(n_nodes=12, n_pods=24)),
    "edge_fit_rtc_small": ("fit_rtc", dict(n_nodes=12, n_pods=24)),
    "edge_na_small": ("na", dict(n_nodes=16, n_pods=30)),
    "edge_pts_small": ("pts", dict(n_nodes=16, n_existing=30, n_pods=24)),
    "edge_ipa_small": ("ipa", dict(n_nodes=14, n_existing=30, n_pods=24)),
    "edge_ipa_ignore_small": ("ipa_ignore", dict(n_nodes=14, n_existing=30, n_pods=24)),
    "edge_preempt_small": ("preempt", dict(n_nodes=10, n_existing=40, n_pods=30)),
    "edge_volumes_small": ("volumes", dict(n_nodes=16, n_existing=30, n_pods=40)),
    "edge_queue_small": ("queue", dict(n_nodes=8, n_existing=24, n_pods=30)),
}


def expected(doc):
    o = Oracle(doc)
    o.schedule(record=3)
    pods = []
    for q in range(o.n_queue):
        sel, feas, st = o.result(q)
        e = {"pod": o.queue_names()[q], "selected": sel, "feasible": feas, "status": st,
             "annotations": o.annotations(q)}
        node, victims = o.nominated(q)
        if node >= 0:  # DefaultPreemption dry run (pods of mixed priorities)
            e["nominated"] = {"node": node, "victims": victims}
        pods.append(e)
    return pods


def main():
    for name, fn in KNOWN.items():
        doc = fn()
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump({"cluster": doc, "expected": expected(doc)}, f, indent=1, sort_keys=True)
    for name, (c, kw) in FAMILIES.items():
        doc = g.generate(c, **kw)
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump({"config": c, "sizes": kw, "cluster": doc, "expected": expected(doc)}, f, sort_keys=True)
    for name, (v, kw) in EDGE.items():
        doc = edge.generate_edge(v, **kw)
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump({"edge": v, "sizes": kw, "cluster": doc, "expected": expected(doc)}, f, sort_keys=True)
    print("wrote", len(KNOWN) + len(FAMILIES) + len(EDGE), "fixtures")


if __name__ == "__main__":
    main()
