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
