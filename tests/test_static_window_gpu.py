"""GPU parity of the window path for profiles with TaintToleration / NodeAffinity.

Those plugins' Filter verdicts and raw Scores do not depend on node resources,
so k_static computes them once per (pod, node); the window replay keeps
NormalizeScore's max at the static max while a feasible node reaches it and
re-evaluates a pod exactly when none does.  The bar is the same as everywhere:
selected node, feasible count, status and the rendered annotations equal the
CPU oracle's (which schedules strictly pod by pod).
"""
import os

import pytest

from _oracle import Oracle
from ksg import Scheduler, generator as g

STATIC_PROFILE = [("TaintToleration", 3), ("NodeAffinity", 2), ("NodeResourcesFit", 1),
                  ("NodeResourcesBalancedAllocation", 1)]


def _compare(doc, per_pod=False, every=1, workers=1, record=3):
    o = Oracle(doc)
    o.schedule(workers=workers, record=record)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.set_path(per_pod)
    assert s.batch_path == (not per_pod)
    if record:
        s.keep_outputs(0, s.queue_len)
    s.schedule()
    res = s.results()
    got = [(r.selected, r.feasible, r.status) for r in res]
    want = [o.result(q) for q in range(len(res))]
    bad = [q for q in range(len(got)) if got[q] != want[q]]
    assert not bad, f"{len(bad)} pods differ, first {[(q, got[q], want[q]) for q in bad[:5]]}"
    if record:
        for q in range(0, s.queue_len, every):
            a, b = s.annotations(q), o.annotations(q)
            for k in b:
                assert a.get(k) == b[k], f"pod {q} annotation {k}:\n gpu    {a.get(k)[:300]}\n oracle {b[k][:300]}"
    return o, s


def _tight_cfg3(n_nodes=96, n_pods=900, seed=11):
    """cfg3's node and pod distributions on nodes that hold only a few pods: the
    nodes reaching a pod's static Taint / NodeAffinity max fill up inside a window."""
    doc = g.gen_cfg3(n_nodes=n_nodes, n_pods=n_pods, seed=seed, feasible_check=False)
    r = g.Rng(seed + 1)
    for n in doc["nodes"]:
        cap = str(2 + r.below(5))
        n["status"]["allocatable"]["pods"] = cap
        n["status"]["capacity"]["pods"] = cap
    return doc


@pytest.mark.gpu
@pytest.mark.parametrize("per_pod", [False, True], ids=["window", "per-pod"])
def test_tight_cfg3_both_paths(per_pod):
    o, s = _compare(_tight_cfg3(), per_pod=per_pod, every=5)
    want = [o.result(q) for q in range(s.queue_len)]
    assert sum(1 for w in want if w[2] == 1) > 50, "cluster should saturate"


def _fallback_doc(kind):
    """Pod 0 is pinned (required NodeAffinity) on node X, which then holds no more
    pods; X is the only node at pod 1's static max (the only node with an
    untolerated PreferNoSchedule taint, or the only node its preference matches),
    so pod 1's NormalizeScore max must drop: the exact re-evaluation path."""
    nodes = []
    for i in range(40):
        labels = {"slot": f"s{i}"}
        taints = None
        pods = 8
        if i == 17:
            pods = 1
            labels["special"] = "yes"
            if kind == "taint":
                taints = [{"key": "t", "value": "v", "effect": "PreferNoSchedule"}]
        nodes.append(g.node_obj(f"node-{i:03d}", 4000, 8 * g.Gi, pods=pods, labels=labels, taints=taints))
    pin = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": [{"matchExpressions": [{"key": "special", "operator": "In", "values": ["yes"]}]}]}}}
    pref = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 50, "preference": {"matchExpressions": [{"key": "special", "operator": "Exists"}]}}]}}
    queue = [g.pod_obj("pod-000", [g.req(100, 128 * g.Mi)], affinity=pin)]
    for j in range(1, 70):
        extra = {"affinity": pref} if kind == "na" else {}
        queue.append(g.pod_obj(f"pod-{j:03d}", [g.req(100 + 10 * (j % 7), 128 * g.Mi)], **extra))
    prof = g.make_profile(STATIC_PROFILE, 5)
    return {"profile": prof, "nodes": nodes, "pods": [], "queue": queue}


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["taint", "na"])
def test_normaliser_fallback(kind):
    o, s = _compare(_fallback_doc(kind))
    assert o.result(0)[0] == 17
    import json
    fin = json.loads(s.annotations(1)["kube-scheduler-simulator.sigs.k8s.io/finalscore-result"])
    plugin = "TaintToleration" if kind == "taint" else "NodeAffinity"
    # with node 17 full, every feasible node has the same raw score: the exact max is 0
    assert len({v[plugin] for v in fin.values()}) == 1


@pytest.mark.gpu
def test_cfg3_static_chunk_ring():
    """Static records in a ring of 2 chunks of 64 pods: windows straddle chunk boundaries."""
    os.environ["KSG_STATIC_CHUNK"] = "64"
    try:
        _compare(g.generate(3, n_nodes=500, n_pods=400), every=9)
    finally:
        del os.environ["KSG_STATIC_CHUNK"]


@pytest.mark.gpu
def test_cfg3_full_width_selected_nodes():
    """cfg3's 15,000 nodes, 600 queue pods: every selection equals the oracle's."""
    doc = g.generate(3, n_nodes=15000, n_pods=600)
    _compare(doc, workers=8, record=0)


@pytest.mark.gpu
@pytest.mark.parametrize("dec", ["1", "0"], ids=["decoded", "program-walk"])
def test_static_records_decoded_and_walked(monkeypatch, dec):
    """The static records come from decoded pods (k_static_dec: flattened
    requirements, taint-id sets) wherever a chunk's pods decode, else from the
    program-walking k_static; both against the oracle on a cfg3 cluster and on
    the saturating one, and on the NodeAffinity / TaintToleration fallback cases."""
    monkeypatch.setenv("KSG_STATIC_DEC", dec)
    for doc in (g.generate(3, n_nodes=700, n_pods=300), _tight_cfg3(n_pods=400), _fallback_doc("taint"),
                _fallback_doc("na")):
        _, s = _compare(doc, every=11)
        assert (s.static_dec_chunks() > 0) == (dec == "1")


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"KSG_STATIC_OVERLAP": "0"}, {"KSG_STATIC_RUN_MB": "0"}, {"KSG_WIN_MB": "1"},
                                 {"KSG_WIN_PFIX": "1"}, {"KSG_WIN_SPLIT": "0"}],
                         ids=["persistent", "records-before", "per-window", "merge-blocks", "prior-in-replay",
                              "one-counter"])
def test_static_profiles_persistent_window_loop(monkeypatch, env):
    """Taint / NodeAffinity profiles in the persistent window loop (k_window_run;
    its static records computed by k_static_dec beside the loop, each window's
    evaluation gated on its pods' groups — or, "records-before", all before the
    launch), its variants, and the launch-per-window loop it replaces: a cfg3
    queue, the saturating cluster and both normaliser-fallback cases against the
    oracle."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for i, doc in enumerate((g.generate(3, n_nodes=900, n_pods=500), _tight_cfg3(n_pods=500), _fallback_doc("taint"),
                             _fallback_doc("na"))):
        _, s = _compare(doc, every=13)
        assert (s.window_runs() > 0) == (env.get("KSG_STATIC_RUN_MB") != "0")
        if i == 0:  # (decodable pods: the records beside the loop unless switched off)
            assert (s.static_overlaps() > 0) == (env.get("KSG_STATIC_OVERLAP") != "0" and
                                                 env.get("KSG_STATIC_RUN_MB") != "0")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["1", "2"], ids=["side-late", "side-absent"])
def test_static_side_kernel_late_or_absent(monkeypatch, mode):
    """The static records beside the loop come from a kernel on another stream, and
    HIP only orders launches, not residency.  The
    loop's handshake counts that kernel's blocks in: launched after the loop
    ("side-late") it either becomes resident beside it or the run falls back; never
    resident beside it ("side-absent": launched only after the loop's verdict) the
    loop must take the per-window fallback before any state changes.  Either way
    every pod equals the oracle's and the context stays usable (a second pass)."""
    monkeypatch.setenv("KSG_STATIC_BESIDE_TEST", mode)
    doc = g.generate(3, n_nodes=900, n_pods=500)
    o, s = _compare(doc, every=13)
    if mode == "2":
        assert s.window_runs() == 0, "a loop whose side blocks never started must not go"
    s.reset()
    s.schedule()
    got = [(r.selected, r.feasible, r.status) for r in s.results()]
    assert got == [o.result(q) for q in range(len(got))]
