"""GPU parity of the drop-in cycle API (ksg_cycle / ksg_reserve / ksg_unreserve).

The per-pod path a Go plugin would take (PreFilter..NormalizeScore per pod,
Reserve with the framework's choice, Unreserve on a failed binding) must give
exactly the queue-mode / oracle results: same selection, feasible count and
annotations for every pod.
"""
import copy

import pytest

from _oracle import Oracle
from ksg import Scheduler, generator as g

CASES = [
    ("cfg2", 2, dict(n_nodes=200, n_pods=120)),
    ("cfg3", 3, dict(n_nodes=200, n_pods=80)),
    ("cfg4", 4, dict(n_nodes=160, n_existing=600, n_pods=60, n_zones=6)),
]


def _empty_queue(doc):
    d = dict(doc)
    d["queue"] = []
    return d


@pytest.mark.gpu
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
def test_cycle_matches_oracle(name, c, sizes):
    doc = g.generate(c, **sizes)
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    s.load_cluster(_empty_queue(doc))
    for i, pod in enumerate(doc["queue"]):
        q, r = s.cycle(pod, commit=True)
        assert q == i
        assert (r.selected, r.feasible, r.status) == o.result(i), (name, i)
        if i % 7 == 0:
            a, b = s.annotations(q), o.annotations(i)
            for k in b:
                assert a.get(k) == b[k], (name, i, k)


@pytest.mark.gpu
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
def test_reserve_with_framework_choice(name, c, sizes):
    """commit=0 then Reserve on the engine's own choice == commit=1."""
    doc = g.generate(c, **sizes)
    o = Oracle(doc)
    o.schedule(record=0)
    s = Scheduler(doc["profile"])
    s.load_cluster(_empty_queue(doc))
    for i, pod in enumerate(doc["queue"]):
        q, r = s.cycle(pod, commit=False)
        assert (r.selected, r.feasible, r.status) == o.result(i), (name, i)
        if r.selected >= 0:
            s.reserve(q, r.selected)


def _blocker(pod):
    """A copy of `pod` no node can hold: its cycle assumes nothing in the oracle."""
    p = copy.deepcopy(pod)
    p["metadata"]["name"] = p["metadata"]["name"] + "-blocked"
    p["spec"]["containers"] = [{"name": "c0", "image": "registry.k8s.io/pause:3.5",
                                "resources": {"requests": {"cpu": "100000", "memory": "1Gi"}}}]
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
def test_unreserve_restores_state(name, c, sizes):
    """Every 5th pod is assumed then unreserved; the others must match an oracle
    run in which those pods were unschedulable (same queue indices)."""
    doc = g.generate(c, **sizes)
    ref = copy.deepcopy(doc)
    ref["queue"] = [(_blocker(p) if i % 5 == 2 else p) for i, p in enumerate(doc["queue"])]
    o = Oracle(ref)
    o.schedule(record=0)
    s = Scheduler(doc["profile"])
    s.load_cluster(_empty_queue(doc))
    for i, pod in enumerate(doc["queue"]):
        q, r = s.cycle(pod, commit=True)
        if i % 5 == 2:
            if r.selected >= 0:
                s.unreserve(q)
            continue
        assert (r.selected, r.feasible, r.status) == o.result(i), (name, i)


@pytest.mark.gpu
def test_cycle_new_vocabulary_rebuilds():
    """Pods bringing label keys/values and namespaces the snapshot never saw grow the
    vocabulary in place (new label keys widen the device's label columns); a pod
    bringing a new topology key re-encodes (placements kept).  Selectors naming
    values no pod carries yet (an assumed pod's required anti-affinity on a fresh
    value, carried by a later pod) stay exact.  Results stay equal to the oracle's;
    an Unreserve of an early pod then takes exactly its requests off its node."""
    doc = g.generate(4, n_nodes=120, n_existing=400, n_pods=40, n_zones=4)
    for i, p in enumerate(doc["queue"]):
        if i % 6 == 3:
            p["metadata"]["labels"] = dict(p["metadata"]["labels"], **{f"fresh-{i}": f"v{i}"})
        if i % 11 == 5:
            p["metadata"]["namespace"] = f"ns-new-{i}"
        if i % 7 == 2 and i + 3 < len(doc["queue"]):  # anti-affinity on a value only pod i+3 will carry
            aff = p["spec"].setdefault("affinity", {})
            aff.setdefault("podAntiAffinity", {}).setdefault("requiredDuringSchedulingIgnoredDuringExecution", []).append(
                {"labelSelector": {"matchLabels": {"fresh-sel": f"x{i}"}}, "topologyKey": "kubernetes.io/hostname"})
            q3 = doc["queue"][i + 3]["metadata"]
            q3["labels"] = dict(q3.get("labels", {}), **{"fresh-sel": f"x{i}"})
        if i == 30:  # a topology key no node or pod named yet: re-encode
            p["spec"]["topologySpreadConstraints"] = [{"maxSkew": 1, "topologyKey": "example.com/rack",
                                                      "whenUnsatisfiable": "ScheduleAnyway",
                                                      "labelSelector": {"matchLabels": {"app": "x"}}}]
    o = Oracle(doc)
    o.schedule(record=0)
    s = Scheduler(doc["profile"])
    s.load_cluster(_empty_queue(doc))
    for i, pod in enumerate(doc["queue"]):
        q, r = s.cycle(pod, commit=True)
        assert (r.selected, r.feasible, r.status) == o.result(i), i
    sel1 = s.results(1, 1)[0].selected
    assert sel1 >= 0
    req0, pc0 = s.node_requested()
    s.unreserve(1)
    req1, pc1 = s.node_requested()
    assert pc0[sel1] - pc1[sel1] == 1
    assert sum(pc0) - sum(pc1) == 1
    assert req0[0][sel1] - req1[0][sel1] > 0 or req0[1][sel1] - req1[1][sel1] > 0


@pytest.mark.gpu
def test_cycle_table_grows_in_place():
    """More assumed pods than the existing-pod table's slack (1,024 rows): the table
    grows in place (rows, terms, reqs, vals re-laid, contents kept) and every
    cycle still equals the oracle."""
    doc = g.generate(4, n_nodes=60, n_existing=120, n_pods=1300, n_zones=3)
    o = Oracle(doc)
    o.schedule(record=0)
    s = Scheduler(doc["profile"])
    s.load_cluster(_empty_queue(doc))
    for i, pod in enumerate(doc["queue"]):
        q, r = s.cycle(pod, commit=True)
        assert (r.selected, r.feasible, r.status) == o.result(i), i


@pytest.mark.gpu
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("keep", [0, 2], ids=["keep0", "keep2"])
def test_compact_bounds_the_queue(name, c, sizes, keep):
    """ksg_compact (plugin mode's memory bound): after K cycles, all but the last
    `keep` pods leave the queue (placed ones become bound pods); the kept pods keep
    their results, and every later cycle equals the oracle's run of the whole
    queue without any compaction (the tie-break hash keeps each pod's position in
    the sequence of queued pods: ADVICE r02)."""
    doc = g.generate(c, **sizes)
    pods = doc["queue"]
    k = len(pods) // 2
    s = Scheduler(doc["profile"])
    s.load_cluster(_empty_queue(doc))
    names = [n["metadata"]["name"] for n in doc["nodes"]]
    first = [s.cycle(p, commit=True)[1] for p in pods[:k]]
    s.compact(k - keep)
    assert s.queue_len == keep
    assert [(r.selected, r.feasible, r.status) for r in s.results()] == \
        [(r.selected, r.feasible, r.status) for r in first[k - keep:]]
    o = Oracle(doc)
    o.schedule(record=3)
    assert [(r.selected, r.feasible, r.status) for r in first] == [o.result(i) for i in range(k)]
    for j, p in enumerate(pods[k:]):
        q, r = s.cycle(p, commit=True)
        assert q == keep + j
        assert (r.selected, r.feasible, r.status) == o.result(k + j), (name, j)
        if j % 5 == 0:
            assert s.annotations(q) == o.annotations(k + j), (name, j)
    s.compact()
    assert s.queue_len == 0


@pytest.mark.gpu
def test_retried_pod_then_events():
    """kube-scheduler retries an unschedulable pod by running a new cycle for the same
    (namespace, name).  After the retry places it, a removePod event releases that
    placement (the first placed cycle of the name), and events keep using the name
    index (a duplicate name no longer switches lookups to a scan)."""
    doc = g.generate(2, n_nodes=40, n_pods=30)
    s = Scheduler(doc["profile"])
    s.load_cluster(_empty_queue(doc))
    for pod in doc["queue"][:10]:
        s.cycle(pod, commit=True)
    big = copy.deepcopy(doc["queue"][10])
    big["metadata"]["name"] = "retry-me"
    big["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "200", "memory": "1Gi"}}
    q1, r1 = s.cycle(big, commit=True)
    assert r1.status == 1 and r1.selected < 0  # 200 cores fit nowhere
    before = s.node_requested(3)
    node = g.node_obj("node-huge", 512000, 2048 * g.Gi)
    s.apply_events([{"op": "addNode", "node": node}])
    q2, r2 = s.cycle(big, commit=True)  # the retry
    assert q2 == q1 + 1 and r2.status == 0
    assert r2.selected == s.node_index("node-huge")
    s.apply_events([{"op": "removePod", "name": "retry-me", "namespace": big["metadata"].get("namespace", "default")}])
    after = s.node_requested(3)
    n = len(before[1])
    assert [row[:n] for row in after[0]] == before[0] and after[1][:n] == before[1]
    assert after[1][n] == 0 and all(row[n] == 0 for row in after[0])  # released from the new node
    for pod in doc["queue"][11:20]:  # later cycles still run
        _, r = s.cycle(pod, commit=True)
        assert r.status in (0, 1)
