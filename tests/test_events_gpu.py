"""GPU parity of scheduler-cache events between cycles (ksg_apply_events).

Upstream the scheduler cache follows informer events (v1.30.4
pkg/scheduler/internal/cache/cache.go AddNode/UpdateNode/RemoveNode/AddPod/
UpdatePod/RemovePod, via eventhandlers.go).  A queue is scheduled half-way, a
batch of events mutates the cluster (node resources/labels updated, a node
added, a drained node removed, bound pods added and removed, a scheduled queue
pod deleted), and the second half is scheduled.  The oracle sees the equivalent
fresh cluster: the mutated nodes, the mutated bound pods plus the first half's
placements as bound pods, and a queue whose first half is replaced by pods
that fit nowhere (so the second half keeps its queue indices, which the
tie-break hash uses, and nothing else changes).
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


def _nowhere(i):
    return g.pod_obj(f"zz-dummy-{i:05d}", [g.req(10 ** 9, 1 << 50)])


def _events(doc, placed, k):
    """Event batch + the oracle's equivalent document."""
    nodes = copy.deepcopy(doc["nodes"])
    bound = copy.deepcopy(doc.get("pods", []))
    names = [n["metadata"]["name"] for n in nodes]
    ev = []
    # updateNode: more cpu, a relabel (new key = new vocabulary)
    upd = copy.deepcopy(nodes[3])
    upd["status"]["allocatable"]["cpu"] = "96"
    upd["metadata"]["labels"]["evt"] = "updated"
    ev.append({"op": "updateNode", "node": upd})
    nodes[3] = upd
    # addNode: a copy of node 0 under a new name
    new = copy.deepcopy(nodes[0])
    new["metadata"]["name"] = "node-9999999"
    new["metadata"]["labels"]["kubernetes.io/hostname"] = "node-9999999"
    ev.append({"op": "addNode", "node": new})
    nodes.append(new)
    # addPod: a bound pod (copy of an existing one when there is any: labels count for PTS/IPA)
    src = copy.deepcopy(bound[0]) if bound else g.filler_pod("x", names[5], 500, 1 << 30)
    src["metadata"]["name"] = "evt-added"
    src["spec"]["nodeName"] = names[5]
    ev.append({"op": "addPod", "pod": src})
    bound.append(src)
    # removePod: a bound pod of the snapshot
    if len(bound) > 2:
        gone = bound[1]["metadata"]
        ev.append({"op": "removePod", "name": gone["name"], "namespace": gone.get("namespace", "default")})
        del bound[1]
    # removePod: a queue pod scheduled in the first half
    first = [i for i in range(k) if placed[i] >= 0]
    deleted = first[0] if first else None
    if deleted is not None:
        ev.append({"op": "removePod", "name": doc["queue"][deleted]["metadata"]["name"], "namespace": "default"})
    # removeNode: drain the node with the fewest bound pods and no placement, then remove it
    on = {}
    for p in bound:
        on.setdefault(p["spec"]["nodeName"], []).append(p)
    taken = {names[placed[i]] for i in range(k) if placed[i] >= 0 and i != deleted}
    cand = [n for n in names[10:] if n not in taken]
    victim = min(cand, key=lambda n: len(on.get(n, [])))
    for p in on.get(victim, []):
        ev.append({"op": "removePod", "name": p["metadata"]["name"], "namespace": p["metadata"].get("namespace", "default")})
        bound.remove(p)
    ev.append({"op": "removeNode", "name": victim})
    nodes = [n for n in nodes if n["metadata"]["name"] != victim]
    # the oracle's equivalent document
    for i in range(k):
        if placed[i] >= 0 and i != deleted:
            p = copy.deepcopy(doc["queue"][i])
            p["spec"]["nodeName"] = names[placed[i]]
            bound.append(p)
    eq = dict(doc)
    eq["nodes"], eq["pods"] = nodes, bound
    eq["queue"] = [_nowhere(i) for i in range(k)] + doc["queue"][k:]
    return ev, eq


@pytest.mark.gpu
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
def test_events_between_cycles(name, c, sizes):
    doc = g.generate(c, **sizes)
    n, k = len(doc["queue"]), len(doc["queue"]) // 2
    s = Scheduler(doc["profile"])
    s.load_cluster(dict(doc, queue=[]))
    placed = []
    for pod in doc["queue"][:k]:
        _, r = s.cycle(pod, commit=True)
        placed.append(r.selected if r.status == 0 else -1)
    ev, eq = _events(doc, placed, k)
    s.apply_events(ev)
    assert s.n_nodes == len(eq["nodes"])
    o = Oracle(eq)
    o.schedule(record=3)
    for i in range(k, n):
        q, r = s.cycle(doc["queue"][i], commit=True)
        assert q == i
        assert (r.selected, r.feasible, r.status) == o.result(i), (name, i)
        if i % 5 == 0:
            a, b = s.annotations(q), o.annotations(i)
            for key in b:
                assert a.get(key) == b[key], (name, i, key)


@pytest.mark.gpu
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
def test_events_between_queue_runs(name, c, sizes):
    """Queue mode (window path for cfg2/cfg3): schedule [0, k), events, schedule [k, n)."""
    doc = g.generate(c, **sizes)
    n, k = len(doc["queue"]), len(doc["queue"]) // 2
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.schedule(0, k)
    placed = [r.selected if r.status == 0 else -1 for r in s.results(0, k)]
    ev, eq = _events(doc, placed, k)
    s.apply_events(ev)
    o = Oracle(eq)
    o.schedule(record=0)
    s.schedule(k, n - k)
    got = s.results(k, n - k)
    for i in range(k, n):
        r = got[i - k]
        assert (r.selected, r.feasible, r.status) == o.result(i), (name, i)


@pytest.mark.gpu
def test_event_batch_is_all_or_nothing():
    doc = g.generate(2, n_nodes=64, n_pods=40)
    s = Scheduler(doc["profile"])
    s.load_cluster(dict(doc, queue=[]))
    bad = [{"op": "addNode", "node": g.node_obj("node-8888888", 8000, 32 << 30)},
           {"op": "removeNode", "name": "no-such-node"}]
    with pytest.raises(Exception, match="removeNode"):
        s.apply_events(bad)
    assert s.n_nodes == 64
    with pytest.raises(Exception, match="unknown node"):
        s.apply_events([{"op": "addPod", "pod": g.filler_pod("p", "nowhere", 100, 1 << 20)}])
    o = Oracle(doc)
    o.schedule(record=0)
    for i, pod in enumerate(doc["queue"]):
        _, r = s.cycle(pod, commit=True)
        assert (r.selected, r.feasible, r.status) == o.result(i)


def _pod_events(doc, placed, k):
    """Bound-pod additions/removals and allocatable-only node updates (the in-place
    path) + the oracle's document."""
    names = [n["metadata"]["name"] for n in doc["nodes"]]
    nodes = copy.deepcopy(doc["nodes"])
    bound = copy.deepcopy(doc.get("pods", []))
    ev = []
    for j, (cpu, pods) in ((1, ("48", "60")), (4, ("3", "110")), (1, ("40", "50"))):
        x = copy.deepcopy(nodes[j])
        x["status"]["allocatable"]["cpu"], x["status"]["allocatable"]["pods"] = cpu, pods
        ev.append({"op": "updateNode", "node": x})
        nodes[j] = x
    src = [p for p in bound[:40]] or [g.filler_pod("x", names[0], 300, 1 << 29)]
    for j in range(12):  # copies of existing pods (labels, terms, ports) on other nodes
        p = copy.deepcopy(src[j % len(src)])
        p["metadata"]["name"] = f"evt-add-{j:03d}"
        p["spec"]["nodeName"] = names[(7 * j + 3) % len(names)]
        ev.append({"op": "addPod", "pod": p})
        bound.append(p)
    for p in list(bound[2:30:3]):  # snapshot pods and some of the pods just added
        ev.append({"op": "removePod", "name": p["metadata"]["name"], "namespace": p["metadata"].get("namespace", "default")})
        bound.remove(p)
    late = next(p for p in bound if p["metadata"]["name"] == "evt-add-010")  # added by this same batch
    ev.append({"op": "removePod", "name": "evt-add-010", "namespace": late["metadata"].get("namespace", "default")})
    bound.remove(late)
    # a queue pod scheduled in the first half is deleted (Unreserve's delta in place)
    deleted = next((i for i in range(k) if placed[i] >= 0), None)
    if deleted is not None:
        ev.append({"op": "removePod", "name": doc["queue"][deleted]["metadata"]["name"], "namespace": "default"})
    for i in range(k):
        if placed[i] >= 0 and i != deleted:
            p = copy.deepcopy(doc["queue"][i])
            p["spec"]["nodeName"] = names[placed[i]]
            bound.append(p)
    eq = dict(doc)
    eq["nodes"], eq["pods"] = nodes, bound
    eq["queue"] = [_nowhere(i) for i in range(k)] + doc["queue"][k:]
    return ev, eq


@pytest.mark.gpu
@pytest.mark.parametrize("reencode", [False, True], ids=["inplace", "reencode"])
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
def test_bound_pod_events_in_place(name, c, sizes, reencode):
    """Bound-pod batches go through the device assume delta (no re-encode); both
    paths must agree with the oracle, in cycle mode and then in queue mode."""
    doc = g.generate(c, **sizes)
    n, k = len(doc["queue"]), len(doc["queue"]) // 2
    s = Scheduler(doc["profile"])
    s.load_cluster(dict(doc, queue=[]))
    placed = []
    for pod in doc["queue"][:k]:
        _, r = s.cycle(pod, commit=True)
        placed.append(r.selected if r.status == 0 else -1)
    ev, eq = _pod_events(doc, placed, k)
    s.apply_events(ev, reencode=reencode)
    if not reencode and doc.get("pods"):  # the batch took the in-place path (no re-encode)
        assert s.n_nodes == len(doc["nodes"])
        with pytest.raises(Exception, match="reset after in-place"):
            s.reset()
    o = Oracle(eq)
    o.schedule(record=3)
    for i in range(k, n):
        q, r = s.cycle(doc["queue"][i], commit=True)
        assert (r.selected, r.feasible, r.status) == o.result(i), (name, reencode, i)
        if i % 5 == 0:
            a, b = s.annotations(q), o.annotations(i)
            for key in b:
                assert a.get(key) == b[key], (name, i, key)


def _random_batch(rng, nodes, bound, tag):
    """A random mix of events over the python mirror (nodes, bound, placements)."""
    ev = []
    for _ in range(rng.randint(1, 6)):
        kind = rng.choice(["addPod", "removePod", "allocNode", "relabelNode", "addNode"])
        if kind == "addPod" and bound:
            p = copy.deepcopy(rng.choice(bound))
            p["metadata"]["name"] = f"rnd-{tag}-{len(ev)}-{rng.randint(0, 10**6)}"
            p["spec"]["nodeName"] = rng.choice(nodes)["metadata"]["name"]
            ev.append({"op": "addPod", "pod": p})
            bound.append(p)
        elif kind == "removePod" and len(bound) > 2:
            p = rng.choice(bound)
            ev.append({"op": "removePod", "name": p["metadata"]["name"],
                       "namespace": p["metadata"].get("namespace", "default")})
            bound.remove(p)
        elif kind == "allocNode":
            j = rng.randrange(len(nodes))
            x = copy.deepcopy(nodes[j])
            x["status"]["allocatable"]["cpu"] = str(rng.choice([4, 8, 32, 96]))
            ev.append({"op": "updateNode", "node": x})
            nodes[j] = x
        elif kind == "relabelNode":
            j = rng.randrange(len(nodes))
            x = copy.deepcopy(nodes[j])
            x["metadata"]["labels"][f"rnd-{rng.randint(0, 3)}"] = f"v{rng.randint(0, 2)}"
            ev.append({"op": "updateNode", "node": x})
            nodes[j] = x
        elif kind == "addNode":
            x = copy.deepcopy(rng.choice(nodes))
            nm = f"node-{9000000 + rng.randint(0, 999999):07d}"
            if any(n["metadata"]["name"] == nm for n in nodes):
                continue
            x["metadata"]["name"] = nm
            x["metadata"]["labels"]["kubernetes.io/hostname"] = nm
            ev.append({"op": "addNode", "node": x})
            nodes.append(x)
    return ev


@pytest.mark.gpu
@pytest.mark.parametrize("name,c,sizes", CASES, ids=[c[0] for c in CASES])
def test_random_event_rounds(name, c, sizes):
    """Eight rounds of (cycles, random event batch: in-place or re-encoded); after
    every batch the next round's pods match the oracle on the equivalent fresh
    cluster."""
    import random
    rng = random.Random(20250131 + c)
    doc = g.generate(c, **sizes)
    n = len(doc["queue"])
    s = Scheduler(doc["profile"])
    s.load_cluster(dict(doc, queue=[]))
    nodes = copy.deepcopy(doc["nodes"])
    bound = copy.deepcopy(doc.get("pods", [])) or [g.filler_pod("seed-pod", nodes[0]["metadata"]["name"], 100, 1 << 28)]
    if not doc.get("pods"):
        s.apply_events([{"op": "addPod", "pod": bound[0]}])
    R = 8
    cuts = [n * j // R for j in range(R + 1)]
    for rnd in range(R):
        eq = dict(doc)
        eq["nodes"], eq["pods"] = nodes, list(bound)
        eq["queue"] = [_nowhere(i) for i in range(cuts[rnd])] + doc["queue"][cuts[rnd]:]
        o = Oracle(eq)
        o.schedule(cuts[rnd + 1], record=0)
        for i in range(cuts[rnd], cuts[rnd + 1]):
            q, r = s.cycle(doc["queue"][i], commit=True)
            assert (r.selected, r.feasible, r.status) == o.result(i), (name, rnd, i)
            if r.status == 0:  # from now on a bound pod of the mirror
                p = copy.deepcopy(doc["queue"][i])
                p["spec"]["nodeName"] = nodes[r.selected]["metadata"]["name"]
                bound.append(p)
        s.apply_events(_random_batch(rng, nodes, bound, rnd))
        assert s.n_nodes == len(nodes)


@pytest.mark.gpu
def test_inplace_adds_beyond_table_slack_then_queue():
    """bound-pod additions that use up the existing-pod table's
    slack before the queue runs.  The device table must still hold every queue
    pod the run assumes (the in-place path checks the room it needs, else the
    batch is re-encoded), so PTS/IPA results after the batch match the oracle."""
    doc = g.generate(4, n_nodes=120, n_existing=400, n_pods=80, n_zones=6)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    names = [n["metadata"]["name"] for n in doc["nodes"]]
    bound = copy.deepcopy(doc["pods"])
    ev = []
    for j in range(1400):  # > the 1,024 rows of slack beyond the loaded pods + queue
        p = copy.deepcopy(doc["pods"][j % len(doc["pods"])])
        p["metadata"]["name"] = f"slack-{j:05d}"
        p["spec"]["nodeName"] = names[(11 * j + 5) % len(names)]
        ev.append({"op": "addPod", "pod": p})
        bound.append(p)
    s.apply_events(ev)
    s.schedule()
    o = Oracle(dict(doc, pods=bound))
    o.schedule(record=0)
    got = [(r.selected, r.feasible, r.status) for r in s.results()]
    assert got == [o.result(q) for q in range(len(got))]


def _static_events(doc, rng, fresh=False):
    """updateNode events that rewrite labels (non-topology keys, values some node
    already carries), taint lists (taints some node already carries: added,
    removed, replaced, reordered) and spec.unschedulable — the in-place path.
    fresh=True also brings a label value no node carries (the re-encode path)."""
    nodes = copy.deepcopy(doc["nodes"])
    topo = {"kubernetes.io/hostname", "topology.kubernetes.io/zone"}
    vals = {}
    taints = []
    for n in nodes:
        for k, v in n["metadata"].get("labels", {}).items():
            if k not in topo:
                vals.setdefault(k, set()).add(v)
        for t in (n.get("spec") or {}).get("taints") or []:
            if t not in taints:
                taints.append(t)
    vals = {k: sorted(v) for k, v in sorted(vals.items())}
    ev = []
    for j in rng.sample(range(len(nodes)), min(40, len(nodes))):
        x = copy.deepcopy(nodes[j])
        lab = x["metadata"].setdefault("labels", {})
        spec = x.setdefault("spec", {})
        for _ in range(rng.randint(1, 3)):
            kind = rng.choice(["set", "drop", "taint+", "taint-", "taint~", "unsched"] if taints else ["set", "drop", "unsched"])
            keys = list(vals)
            if kind == "set" and keys:
                k = rng.choice(keys)
                lab[k] = rng.choice(vals[k])
            elif kind == "drop":
                droppable = [k for k in lab if k not in topo]
                if droppable:
                    del lab[rng.choice(droppable)]
            elif kind == "taint+":
                t = rng.choice(taints)
                spec.setdefault("taints", []).insert(rng.randint(0, len(spec.get("taints") or [])), copy.deepcopy(t))
            elif kind == "taint-" and spec.get("taints"):
                spec["taints"].pop(rng.randrange(len(spec["taints"])))
            elif kind == "taint~" and spec.get("taints"):
                spec["taints"][rng.randrange(len(spec["taints"]))] = copy.deepcopy(rng.choice(taints))
                rng.shuffle(spec["taints"])
            elif kind == "unsched":
                spec["unschedulable"] = not spec.get("unschedulable", False)
        ev.append({"op": "updateNode", "node": x})
        nodes[j] = x
    if fresh:
        x = copy.deepcopy(nodes[0])
        x["metadata"].setdefault("labels", {})["tier"] = "never-seen-before"
        ev.append({"op": "updateNode", "node": x})
        nodes[0] = x
    return ev, nodes


STATIC_CASES = [
    ("cfg3", 3, dict(n_nodes=200, n_pods=80)),
    ("cfg2", 2, dict(n_nodes=200, n_pods=120)),
    ("cfg4", 4, dict(n_nodes=160, n_existing=600, n_pods=60, n_zones=6)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["inplace", "reencode", "fresh"])
@pytest.mark.parametrize("name,c,sizes", STATIC_CASES, ids=[c[0] for c in STATIC_CASES])
def test_node_label_taint_events_in_place(name, c, sizes, path):
    """Node label / taint / unschedulable rewrites between cycles go to the device
    columns in place (no re-encode) when the vocabularies hold their values and no
    topology key changes; a batch with a value no node carried is re-encoded.
    Cycle mode for the first half, events, then queue mode for the second half —
    every result matches the oracle on the equivalent fresh cluster."""
    import random
    rng = random.Random(7100 + c)
    doc = g.generate(c, **sizes)
    n, k = len(doc["queue"]), len(doc["queue"]) // 2
    s = Scheduler(doc["profile"])
    s.load_cluster(dict(doc, queue=[]))
    placed = []
    for pod in doc["queue"][:k]:
        _, r = s.cycle(pod, commit=True)
        placed.append(r.selected if r.status == 0 else -1)
    ev, nodes = _static_events(doc, rng, fresh=path == "fresh")
    s.apply_events(ev, reencode=path == "reencode")
    if path == "inplace":
        with pytest.raises(Exception, match="reset after in-place"):
            s.reset()
    bound = copy.deepcopy(doc.get("pods", []))
    names = [x["metadata"]["name"] for x in doc["nodes"]]
    for i in range(k):
        if placed[i] >= 0:
            p = copy.deepcopy(doc["queue"][i])
            p["spec"]["nodeName"] = names[placed[i]]
            bound.append(p)
    eq = dict(doc, nodes=nodes, pods=bound, queue=[_nowhere(i) for i in range(k)] + doc["queue"][k:])
    o = Oracle(eq)
    o.schedule(record=3)
    h = (n - k) // 2
    for i in range(k, k + h):  # cycle mode
        q, r = s.cycle(doc["queue"][i], commit=True)
        assert (r.selected, r.feasible, r.status) == o.result(i), (name, path, i)
        if i % 7 == 0:
            a, b = s.annotations(q), o.annotations(i)
            for key in b:
                assert a.get(key) == b[key], (name, path, i, key)
    # the rest through a second batch (queue mode): the context's own queue
    s2 = Scheduler(doc["profile"])
    s2.load_cluster(dict(doc, pods=copy.deepcopy(bound), queue=[_nowhere(i) for i in range(k)] + doc["queue"][k:]))
    s2.schedule(0, k)
    ev2, nodes2 = _static_events(doc, random.Random(7200 + c), fresh=path == "fresh")
    s2.apply_events(ev2, reencode=path == "reencode")
    if path == "inplace":
        with pytest.raises(Exception, match="reset after in-place"):
            s2.reset()
    o2 = Oracle(dict(eq, nodes=nodes2))
    o2.schedule(record=0)
    s2.schedule(k, n - k)
    got = s2.results(k, n - k)
    for i in range(k, n):
        assert (got[i - k].selected, got[i - k].feasible, got[i - k].status) == o2.result(i), (name, path, "queue", i)
