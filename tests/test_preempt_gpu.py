"""GPU parity of DefaultPreemption's dry run (PostFilter of unschedulable pods;
upstream v1.30.4 default_preemption.go / preemption.go as oracle/ksg_oracle.cpp
preempt() restates it; the result store's postfilter-result entry, store.go:442).

The edge family's ``preempt`` cluster (ksg/edge.py): bound pods and queue pods
at mixed priorities, start times, preemptionPolicy Never, host ports, pod-count
limits, spread constraints, anti-affinity, taints.  Per pod the nominated node
and the victims (most important first) equal the oracle's, in queue mode and
through the drop-in cycle API; the dry run leaves the device state exactly as
it was (the same cluster without DefaultPreemption schedules identically and
ends with the same node rows); ksg_reset + a second run reproduces the first."""
import pytest

from _oracle import Oracle
from ksg import Scheduler, edge


def _doc(**sizes):
    return edge.generate_edge("preempt", **sizes)


def _oracle(doc):
    o = Oracle(doc)
    o.schedule(record=3)
    return o


@pytest.mark.gpu
@pytest.mark.parametrize("batch", ["1", "store", "0"], ids=["batched", "victim-store", "per-node"])
@pytest.mark.parametrize("sizes", [{}, dict(n_nodes=10, n_existing=40, n_pods=30),
                                   dict(n_existing=70, n_pods=120, queue_sort=False)],
                         ids=["default", "small", "queue-victims"])
def test_preempt_queue_matches_oracle(monkeypatch, sizes, batch):
    """Both victim searches — batched over every potential node (pods whose
    PreFilter state no removal changes) and the per-node probes — nominate the
    oracle's node and victims; "victim-store": the batched search staging its
    candidates by reference into the device-resident store of every bound pod's
    program (what searches with thousands of victims use) from the first search."""
    monkeypatch.setenv("KSG_PREEMPT_BATCH", "0" if batch == "0" else "1")
    if batch == "store":
        monkeypatch.setenv("KSG_VICTIM_STORE_MIN", "0")
    doc = _doc(**sizes)
    o = _oracle(doc)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.keep_outputs(0, s.queue_len)
    s.schedule()
    res = s.results()
    nominated = 0
    for q, r in enumerate(res):
        assert (r.selected, r.feasible, r.status) == o.result(q), q
        assert s.postfilter_result(q) == o.nominated(q), q
        nominated += s.postfilter_result(q)[0] >= 0
        assert s.annotations(q) == o.annotations(q), q
    assert nominated >= 5  # the family exercises the dry run
    if batch != "0":
        assert s.preempt_batched() > 0
    else:
        assert s.preempt_batched() == 0


@pytest.mark.gpu
def test_preempt_cycle_api_matches_oracle():
    # pods arriving one at a time (arrival order): earlier queue pods can be victims
    doc = _doc(n_pods=50, queue_sort=False)
    o = _oracle(doc)
    s = Scheduler(doc["profile"])
    d = dict(doc)
    d["queue"] = []
    d.pop("queueSort")
    s.load_cluster(d)
    for i, pod in enumerate(doc["queue"]):
        q, r = s.cycle(pod, commit=True)
        assert (r.selected, r.feasible, r.status) == o.result(i), i
        assert s.postfilter_result(q) == o.nominated(i), i
        if i % 5 == 0:
            assert s.annotations(q) == o.annotations(i), i


@pytest.mark.gpu
def test_preempt_dry_run_leaves_state():
    doc = _doc()
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.schedule()
    res = [(r.selected, r.feasible, r.status) for r in s.results()]
    req, cnt = s.node_requested()
    prof = dict(doc["profile"])
    prof["plugins"] = [p for p in prof["plugins"] if p != "DefaultPreemption"]
    t = Scheduler(prof)
    t.load_cluster(doc)
    t.schedule()
    assert [(r.selected, r.feasible, r.status) for r in t.results()] == res
    req2, cnt2 = t.node_requested()
    assert req == req2 and cnt == cnt2
    # a second run after ksg_reset: same placements and nominations
    noms = [s.postfilter_result(q) for q in range(s.queue_len)]
    s.reset()
    s.schedule()
    assert [(r.selected, r.feasible, r.status) for r in s.results()] == res
    assert [s.postfilter_result(q) for q in range(s.queue_len)] == noms


@pytest.mark.gpu
def test_victim_store_refreshed_after_events_and_compaction(monkeypatch):
    """The device-resident victim store (every bound pod's program, KSG_VICTIM_STORE_MIN=0:
    from the first search) stays valid only while the bound pods do not change
    (ADVICE r05).  Drop-in cycles run searches, then an event batch removes a bound
    pod and adds another and a compaction turns the placed queue pods into bound
    pods; every later search must see the new set.  The oracle schedules the
    equivalent cluster: the mutated bound pods, the first half's placements as bound
    pods, and pods that fit nowhere in the first half's queue slots (the tie-break
    hash keeps each later pod's queue index)."""
    import copy
    from ksg import generator as g
    monkeypatch.setenv("KSG_PREEMPT_BATCH", "1")
    monkeypatch.setenv("KSG_VICTIM_STORE_MIN", "0")
    doc = _doc(n_pods=80, queue_sort=False)
    queue = doc["queue"]
    s = Scheduler(doc["profile"])
    d = dict(doc)
    d["queue"] = []
    d.pop("queueSort")
    s.load_cluster(d)
    placed = []
    for pod in queue:  # (until a batched search has built the store)
        _, r = s.cycle(pod, commit=True)
        placed.append(r.selected)
        if s.preempt_batched() > 0 and len(placed) >= 8:
            break
    k = len(placed)
    assert s.preempt_batched() > 0 and k + 16 <= len(queue), "no search ran before the events"
    bound = copy.deepcopy(doc["pods"])
    gone = bound[0]["metadata"]
    added = copy.deepcopy(bound[1])
    added["metadata"]["name"] = "evt-added"
    s.apply_events([{"op": "removePod", "name": gone["name"], "namespace": gone.get("namespace", "default")},
                    {"op": "addPod", "pod": added}])
    del bound[0]
    bound.append(added)
    s.compact()
    names = [n["metadata"]["name"] for n in doc["nodes"]]
    for i in range(k):
        if placed[i] >= 0:
            p = copy.deepcopy(queue[i])
            p["spec"]["nodeName"] = names[placed[i]]
            bound.append(p)
    eq = dict(doc)  # (arrival order, like the cycles: queueSort kept off)
    eq["pods"] = bound
    eq["queue"] = [g.pod_obj(f"zz-dummy-{i:05d}", [g.req(10 ** 9, 1 << 50)]) for i in range(k)] + queue[k:]
    o = _oracle(eq)
    b0 = s.preempt_batched()
    nominated = 0
    for i in range(k, len(queue)):
        q, r = s.cycle(queue[i], commit=True)
        assert (r.selected, r.feasible, r.status) == o.result(i), i
        assert s.postfilter_result(q) == o.nominated(i), i
        nominated += s.postfilter_result(q)[0] >= 0
    assert s.preempt_batched() > b0 and nominated > 0, "no search ran after the events"


@pytest.mark.gpu
def test_preempt_batched_with_schedule_anyway_constraints(monkeypatch):
    """A preemptor whose spread constraints are all ScheduleAnyway takes the batched
    search (upstream podtopologyspread's PreFilter state holds only DoNotSchedule
    constraints, so no removal changes what its filters read): every queue pod of the
    preempt family gets a ScheduleAnyway zone constraint instead of its DoNotSchedule
    one; its required anti-affinity terms (kubernetes.io/hostname: one node per value,
    so a node's removals change only its own domain) stay batched as well.
    Nominations and victims equal the oracle's and the batched search ran for them."""
    monkeypatch.setenv("KSG_PREEMPT_BATCH", "1")
    doc = _doc()
    for p in doc["queue"]:
        p["spec"]["topologySpreadConstraints"] = [{
            "maxSkew": 1, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "ScheduleAnyway",
            "labelSelector": {"matchLabels": dict(list(p["metadata"].get("labels", {}).items())[:1])}}]
    assert sum(1 for p in doc["queue"] if "affinity" in p["spec"]) >= 5
    o = _oracle(doc)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.keep_outputs(0, s.queue_len)
    s.schedule()
    nominated = 0
    for q, r in enumerate(s.results()):
        assert (r.selected, r.feasible, r.status) == o.result(q), q
        assert s.postfilter_result(q) == o.nominated(q), q
        nominated += s.postfilter_result(q)[0] >= 0
    assert nominated >= 5
    assert s.preempt_batched() >= nominated // 2
