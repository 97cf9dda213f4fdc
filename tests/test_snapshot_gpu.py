"""The simulator's snapshot document as input (ResourcesForSnap,
simulator/snapshot/snapshot.go:33-42): bound pods and pending pods mixed in
"pods" (pending = no spec.nodeName, scheduled in document order), plus keys the
path does not read.  Results equal the oracle's on the equivalent
{"pods": bound, "queue": pending} document."""
import pytest

from _oracle import Oracle
from ksg import Scheduler, generator as g


@pytest.mark.gpu
def test_resources_for_snap_document():
    doc = g.generate(4, n_nodes=200, n_existing=600, n_pods=80, n_zones=5)
    snap = {
        "nodes": doc["nodes"],
        "pods": doc["pods"][:300] + doc["queue"] + doc["pods"][300:],  # pending pods anywhere in the list
        "pvs": [], "pvcs": [], "storageClasses": [], "priorityClasses": [], "namespaces": [],
        "schedulerConfig": {"profiles": [{"schedulerName": "default-scheduler"}]},
    }
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    s.load_cluster(snap)
    assert s.queue_len == len(doc["queue"])
    s.keep_outputs(0, s.queue_len)
    s.schedule()
    got = [(r.selected, r.feasible, r.status) for r in s.results()]
    assert got == [o.result(q) for q in range(len(got))]
    for q in range(0, s.queue_len, 9):
        assert s.annotations(q) == o.annotations(q), q
