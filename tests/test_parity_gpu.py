"""GPU parity: libksg.so (HIP) vs the CPU oracle on the same seeded clusters.

Bit-exact bar: every pod's selected node, feasible count and status, and the
rendered result-store annotations (filter-result, score-result,
finalscore-result, prefilter/prescore status, selected-node) byte-for-byte.
"""
import pytest

from _oracle import Oracle
from ksg import KsgError, Scheduler, generator as g

CASES = [
    ("cfg1-default-profile", 1, dict(n_nodes=40, n_pods=120)),
    ("cfg2-fit-ba", 2, dict(n_nodes=300, n_pods=400)),
    ("cfg3-taint-nodeaffinity", 3, dict(n_nodes=300, n_pods=250)),
    ("cfg4-pts-ipa", 4, dict(n_nodes=400, n_existing=1500, n_pods=200, n_zones=8)),
]


def run_both(doc, keep=True):
    o = Oracle(doc)
    o.schedule(record=3 if keep else 0)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    if keep:
        s.keep_outputs(0, s.queue_len)
    s.schedule()
    return o, s


@pytest.mark.gpu
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
def test_selected_and_annotations(name, c, sizes):
    doc = g.generate(c, **sizes)
    o, s = run_both(doc)
    res = s.results()
    mismatches = []
    for q, r in enumerate(res):
        sel, feas, st = o.result(q)
        if (r.selected, r.feasible, r.status) != (sel, feas, st):
            mismatches.append((q, (r.selected, r.feasible, r.status), (sel, feas, st)))
    if mismatches:
        q = mismatches[0][0]
        a, b = s.annotations(q), o.annotations(q)
        diff = {k: (a.get(k, "")[:600], b[k][:600]) for k in b if a.get(k) != b[k]}
        raise AssertionError(f"{name}: {len(mismatches)} pods differ, first {mismatches[:5]}; pod {q} diff {diff}")
    for q in range(s.queue_len):
        a, b = s.annotations(q), o.annotations(q)
        for k in b:
            assert a.get(k) == b[k], f"{name} pod {q} annotation {k}:\n gpu   {a.get(k)[:400]}\n oracle {b[k][:400]}"


@pytest.mark.gpu
def test_assume_delta_matches_oracle_requests():
    doc = g.generate(2, n_nodes=64, n_pods=200)
    o, s = run_both(doc, keep=False)
    req, pc = s.node_requested()
    nzc, nzm = s.node_nonzero()
    # independent recomputation from the oracle's placements: per node, the bound
    # pods' and the placed queue pods' Requested and NonZeroRequested (missing
    # container requests count 100m / 200Mi) and the pod count (NodeInfo.AddPod)
    names = [n["metadata"]["name"] for n in doc["nodes"]]
    N = len(names)
    want = {"cpu": [0] * N, "mem": [0] * N, "nzc": [0] * N, "nzm": [0] * N, "pods": [0] * N}

    def add(pod, i):
        for c in pod["spec"]["containers"]:
            r = c.get("resources", {}).get("requests", {})
            cpu = int(r["cpu"][:-1]) if "cpu" in r else None
            m = r.get("memory")
            mem = None if m is None else (int(m[:-2]) * g.Mi if m.endswith("Mi") else int(m))
            want["cpu"][i] += cpu or 0
            want["mem"][i] += mem or 0
            want["nzc"][i] += 100 if cpu is None else cpu
            want["nzm"][i] += 200 * g.Mi if mem is None else mem
        want["pods"][i] += 1

    for p in doc["pods"]:
        add(p, names.index(p["spec"]["nodeName"]))
    for q in range(o.n_queue):
        if o.result(q)[0] >= 0:
            add(doc["queue"][q], o.result(q)[0])
    assert req[0][:N] == want["cpu"] and req[1][:N] == want["mem"]
    assert nzc == want["nzc"] and nzm == want["nzm"]
    assert pc == want["pods"]


@pytest.mark.gpu
def test_known_answer_readme_example():
    """README.md:63-80 / debuggable-scheduler.md:13-31: Fit 73, BA 76, Taint final 300."""
    prof = g.make_profile(g.DEFAULT_HOT_PROFILE, 1)
    doc = {"profile": prof,
           "nodes": [g.node_obj("node-282x7", 4000, 32 * g.Gi), g.node_obj("node-gp9t4", 4000, 32 * g.Gi)],
           "pods": [], "queue": [g.pod_obj("hoge-pod", [g.req(100, 16 * g.Gi)])]}
    s = Scheduler(prof)
    s.load_cluster(doc)
    s.keep_outputs(0, 1)
    s.schedule()
    import json
    fin = json.loads(s.annotations(0)["kube-scheduler-simulator.sigs.k8s.io/finalscore-result"])
    for node in ("node-282x7", "node-gp9t4"):
        assert fin[node]["NodeResourcesFit"] == "73"
        assert fin[node]["NodeResourcesBalancedAllocation"] == "76"
        assert fin[node]["TaintToleration"] == "300"


@pytest.mark.gpu
def test_known_answer_plugin_extender_example():
    """plugin-extender.md:85-107: Fit 47 / BA 52 on the loaded node-282x7, 73 / 76 on
    node-gp9t4, TaintToleration 300, node-gp9t4 selected (default profile)."""
    import json
    d = _json.load(open(_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "golden",
                                      "plugin_extender_example.json")))
    s = Scheduler(d["cluster"]["profile"])
    s.load_cluster(d["cluster"])
    s.keep_outputs(0, 1)
    s.schedule()
    a = s.annotations(0)
    fin = json.loads(a["kube-scheduler-simulator.sigs.k8s.io/finalscore-result"])
    for node, (fit, ba) in {"node-282x7": ("47", "52"), "node-gp9t4": ("73", "76")}.items():
        assert (fin[node]["NodeResourcesFit"], fin[node]["NodeResourcesBalancedAllocation"]) == (fit, ba)
        assert fin[node]["TaintToleration"] == "300"
    assert a["kube-scheduler-simulator.sigs.k8s.io/selected-node"] == "node-gp9t4"
    assert s.results()[0].selected == 1


def _tight_cluster(n_nodes=24, n_pods=700, seed=7):
    """Few small nodes, many pods: nodes fill up (Too many pods / Insufficient cpu|memory),
    so the speculative batches must re-evaluate modified nodes and drop feasibility."""
    r = g.Rng(seed)
    nodes = [g.node_obj(f"node-{i:07d}", 2000 + 1000 * r.below(4), (4 + 4 * r.below(4)) * g.Gi, pods=10 + r.below(30))
             for i in range(n_nodes)]
    queue = []
    for j in range(n_pods):
        if r.pct() < 15:
            queue.append(g.pod_obj(f"pod-{j:07d}", [{}]))
        else:
            queue.append(g.pod_obj(f"pod-{j:07d}", [g.req(50 * (1 + r.below(8)), 64 * g.Mi * (1 + r.below(8)))]))
    prof = g.make_profile([("NodeResourcesFit", 1), ("NodeResourcesBalancedAllocation", 1)], seed)
    return {"profile": prof, "nodes": nodes, "pods": [], "queue": queue}


@pytest.mark.gpu
@pytest.mark.parametrize("per_pod", [False, True], ids=["batch", "per-pod"])
def test_tight_cluster_both_paths(per_pod):
    doc = _tight_cluster()
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.set_path(per_pod)
    assert s.batch_path == (not per_pod)
    s.keep_outputs(0, s.queue_len)
    s.schedule()
    res = s.results()
    got = [(r.selected, r.feasible, r.status) for r in res]
    want = [o.result(q) for q in range(len(res))]
    assert sum(1 for w in want if w[2] == 1) > 20, "cluster should saturate"
    assert got == want
    for q in range(0, s.queue_len, 7):
        assert s.annotations(q) == o.annotations(q), q


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"KSG_WIN_MB": "1"}, {"KSG_WIN_PFIX": "1"}, {"KSG_WIN_MB": "1", "KSG_WIN_PFIX": "1"},
                                 {"KSG_WIN_RUN": "0"}, {"KSG_WIN_SPLIT": "0"}, {"KSG_WIN_SPLIT": "0", "KSG_WIN_MB": "1"}],
                         ids=["default", "merge-blocks", "prior-in-replay", "both", "launch-per-window", "one-counter",
                              "one-counter-merge-blocks"])
def test_cfg2_large_batch_path_selected_nodes(monkeypatch, env):
    """Full-width cfg2 node count, a queue of 1,000 pods: every selection equals the
    oracle's, for each variant of the window loop (dedicated merge blocks, the
    prior step evaluated by the replay, one launch per window, the hand-over on one
    counter instead of the default split keys / records counters)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    doc = g.generate(2, n_nodes=5000, n_pods=1000)
    o = Oracle(doc)
    o.schedule(workers=8, record=0)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    assert s.batch_path
    s.schedule()
    got = [(r.selected, r.feasible, r.status) for r in s.results()]
    assert got == [o.result(q) for q in range(len(got))]


import glob as _glob
import json as _json
import os as _os

_GOLD = sorted(_glob.glob(_os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "golden", "*.json")))


@pytest.mark.gpu
@pytest.mark.parametrize("path", _GOLD, ids=lambda p: _os.path.basename(p)[:-5])
def test_engine_matches_golden_fixture(path):
    d = _json.load(open(path))
    doc = d["cluster"]
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.keep_outputs(0, s.queue_len)
    s.schedule()
    for q, (r, e) in enumerate(zip(s.results(), d["expected"])):
        assert (r.selected, r.feasible, r.status) == (e["selected"], e["feasible"], e["status"]), q
        assert s.annotations(q) == e["annotations"], q


@pytest.mark.gpu
@pytest.mark.parametrize("c,sizes", [(1, dict(n_nodes=40, n_pods=120)),
                                      (4, dict(n_nodes=600, n_existing=1500, n_pods=150, n_zones=8))],
                         ids=["cfg1", "cfg4"])
def test_one_launch_cycles_match_oracle(monkeypatch, c, sizes):
    """The opt-in one-launch chain (KSG_SOLO=1, k_eval_solo) on pods whose outputs
    are not kept: placements identical to the oracle's, and the cycles really ran
    one-launch (path counter)."""
    monkeypatch.setenv("KSG_SOLO", "1")
    monkeypatch.setenv("KSG_RUN", "0")  # (persistent segments take these pods first)
    doc = g.generate(c, **sizes)
    o, s = run_both(doc, keep=False)
    res = s.results()
    bad = [(q, (r.selected, r.feasible, r.status), o.result(q)) for q, r in enumerate(res)
           if (r.selected, r.feasible, r.status) != o.result(q)]
    assert not bad, f"{len(bad)} pods differ, first {bad[:5]}"
    pc = s.path_counts(solo=True)
    assert pc[2] > 0 or pc[0] == 0, pc  # table-chain pods went one-launch


RUN_CASES = [
    ("cfg4-1block", 4, dict(n_nodes=200, n_existing=600, n_pods=160, n_zones=4), None),
    ("cfg4-3blocks", 4, dict(n_nodes=600, n_existing=1500, n_pods=300, n_zones=8), None),
    ("cfg4-20blocks-kept-middle", 4, dict(n_nodes=5000, n_existing=12000, n_pods=240, n_zones=16), (100, 7)),
    ("cfg4-saturating", 4, dict(n_nodes=64, n_existing=300, n_pods=900, n_zones=4), None),
    ("cfg1-default-profile", 1, dict(n_nodes=300, n_pods=200), None),
]


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"KSG_RUN_MIN": "1"}, {"KSG_RUN_BT": "512"}, {"KSG_RUN_LAG": "4"},
                                 {"KSG_RUN_OVERLAP": "1"}, {"KSG_RUN_DEFER": "0"}],
                         ids=["default", "min1", "bt512", "lag", "overlap", "no-defer"])
@pytest.mark.parametrize("name,c,sizes,keep", RUN_CASES, ids=[c[0] for c in RUN_CASES])
def test_persistent_segments_match_oracle(monkeypatch, env, name, c, sizes, keep):
    """Persistent segments (k_chain_run: the pod loop inside one launch, gates
    between blocks) place every pod exactly as the oracle, with 1, 3 and 20
    blocks (XCD groups of unequal size), around kept pods that split a segment,
    and on a saturating cluster (unschedulable pods in the middle of a segment);
    also with one-pod segments allowed (KSG_RUN_MIN=1), 512-thread blocks, and a
    committer delayed ~14 us per pod (KSG_RUN_LAG=4: longer than a pod's evaluation,
    so the node blocks run a pod ahead of it and rewrite the granules of the pod
    after the one it reads; the parity-slotted granules keep those it reads), and
    with the owner's node-level assume drained at once (KSG_RUN_DEFER=0) instead of
    deferred past an independent next pod's evaluation (the default)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    doc = g.generate(c, **sizes)
    o = Oracle(doc)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    if keep:
        s.keep_outputs(*keep)
        o.schedule(keep[0], record=0)
        o.schedule(keep[1], record=3)
        o.schedule(s.queue_len - keep[0] - keep[1], record=0)
    else:
        o.schedule(record=0)
    s.schedule()
    res = s.results()
    bad = [(q, (r.selected, r.feasible, r.status), o.result(q)) for q, r in enumerate(res)
           if (r.selected, r.feasible, r.status) != o.result(q)]
    assert not bad, f"{name}: {len(bad)} pods differ, first {bad[:5]}"
    if keep:
        for q in range(keep[0], keep[0] + keep[1]):
            a, b = s.annotations(q), o.annotations(q)
            for k in b:
                assert a.get(k) == b[k], f"{name} pod {q} annotation {k}"
    table, _ = s.path_counts()
    run_pods, segs = s.run_counts()
    if table:
        assert run_pods > 0 and segs > 0, (table, run_pods, segs)


@pytest.mark.gpu
def test_persistent_not_resident_falls_back(monkeypatch):
    """A persistent launch whose blocks cannot all be resident (forced: the handshake
    waits for one block more than the grid, KSG_RUN_NORES) leaves before touching any
    state, and its pods run on the two-launch chain: placements identical to the
    oracle's, no pod counted as a persistent-segment pod, the fallback counted."""
    monkeypatch.setenv("KSG_RUN_NORES", "1")
    monkeypatch.setenv("KSG_RUN_WAIT_US", "300")
    doc = g.generate(4, n_nodes=600, n_existing=1500, n_pods=300, n_zones=8)
    o, s = run_both(doc, keep=False)
    res = s.results()
    bad = [(q, (r.selected, r.feasible, r.status), o.result(q)) for q, r in enumerate(res)
           if (r.selected, r.feasible, r.status) != o.result(q)]
    assert not bad, f"{len(bad)} pods differ, first {bad[:5]}"
    assert s.run_fallbacks() >= 1
    assert s.run_counts() == (0, 0)


@pytest.mark.gpu
def test_persistent_abort_marks_context_unusable(monkeypatch):
    """A persistent launch whose poll runs out (forced: one poll per wait and a
    committer delayed ~200 us per pod) raises the sticky abort word: the call fails
    with a device error (later segments of the call leave at their handshake), every
    later call is refused until the cluster is reloaded, and a reload runs again."""
    monkeypatch.setenv("KSG_RUN_SPIN", "1")
    monkeypatch.setenv("KSG_RUN_LAG", "64")
    doc = g.generate(4, n_nodes=600, n_existing=1500, n_pods=120, n_zones=8)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.keep_outputs(40, 2)  # (two segments: pods 0-39 and 42-119)
    with pytest.raises(KsgError, match="gate never completed"):
        s.schedule()
    with pytest.raises(KsgError, match="unusable"):
        s.results()
    s.load_cluster(doc)  # a reload clears the state
    s.results()
    monkeypatch.delenv("KSG_RUN_SPIN")
    monkeypatch.delenv("KSG_RUN_LAG")
    o, s2 = run_both(doc, keep=False)  # a fresh context on the same device, persistent segments on
    assert [(r.selected, r.feasible, r.status) for r in s2.results()] == [o.result(q) for q in range(s2.queue_len)]
    assert s2.run_counts()[0] > 0
