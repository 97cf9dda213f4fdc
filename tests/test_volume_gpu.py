"""GPU parity of the volume plugins (VolumeRestrictions, EBS/GCE/Azure/NodeVolumeLimits,
VolumeBinding, VolumeZone as one KP_VOLUMES device position): the hand-worked
clusters of tests/test_volume_oracle.py and the ``volumes`` edge cluster under
profiles with and without VolumeZone (whose PreFilter otherwise rejects missing
PVs before VolumeBinding's PVNotExist reason shows), every pod and annotation
equal to the oracle's; queue mode and the drop-in cycle path."""
import pytest

import test_volume_oracle as kv
from _oracle import Oracle
from ksg import Scheduler, edge
from ksg.generator import DEFAULT_PROFILE, make_profile
from test_plugin_api_gpu import rebuild


def _known_clusters():
    E = edge
    docs = []
    pv = E._pv("pv-1", "wffc", claim=("default", "c1"), affinity={"nodeSelectorTerms": [
        {"matchExpressions": [{"key": kv.HOSTNAME, "operator": "In", "values": ["n1"]}]}]})
    docs.append(kv.cluster(kv.with_claims("p", "c1"), [E._pvc("c1", "default", volume="pv-1", cls="wffc", bound=True)],
                           [pv], [kv.WFFC]))
    pv = E._pv("pv-z", "wffc", claim=("default", "cz"), labels={kv.ZONE: "zone-a"})
    docs.append(kv.cluster(kv.with_claims("p", "cz"), [E._pvc("cz", "default", volume="pv-z", cls="wffc", bound=True)],
                           [pv], [kv.WFFC]))
    rw = E._pvc("rw", "default", volume="pv-rw", cls="wffc", bound=True, modes=("ReadWriteOncePod",))
    docs.append(kv.cluster(kv.with_claims("p", "rw"), [rw], [E._pv("pv-rw", "wffc", claim=("default", "rw"))], [kv.WFFC],
                           bound=[kv.with_claims("b", "rw", node="n2")]))
    cls = dict(kv.WFFC, metadata={"name": "zb"}, allowedTopologies=[{"matchLabelExpressions": [
        {"key": kv.ZONE, "values": ["zone-b"]}]}])
    docs.append(kv.cluster(kv.with_claims("p", "new"), [E._pvc("new", "default", cls="zb")], [], [cls]))
    d = kv.cluster(kv.with_claims("p", "c"), [E._pvc("c", "default", volume="pv-gone", cls="wffc", bound=True)], [],
                   [kv.WFFC])
    d["profile"] = make_profile(kv.PROFILE[:-1], 7)
    docs.append(d)
    drv = "csi.example.com"  # NodeVolumeLimits (test_csi_attach_limits)
    pvs = [E._pv("pv-a", "wffc", claim=("default", "a")), E._pv("pv-b", "wffc", claim=("default", "b"))]
    pvcs = [E._pvc("a", "default", volume="pv-a", cls="wffc", bound=True),
            E._pvc("b", "default", volume="pv-b", cls="wffc", bound=True)]
    d = kv.cluster(kv.with_claims("p", "a"), pvcs, pvs, [kv.WFFC], bound=[kv.with_claims("h0", "b", node="n0"),
                                                                          kv.with_claims("h1", "b", node="n1")])
    d["csiNodes"] = [{"metadata": {"name": "n0"}, "spec": {"drivers": [{"name": drv, "allocatable": {"count": 1}}]}}]
    d["nodes"][1]["status"]["allocatable"]["attachable-volumes-csi-" + drv] = "2"
    docs.append(d)
    return docs


def _queue_parity(doc, tag):
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.keep_outputs(0, s.queue_len)
    s.schedule()
    for q, r in enumerate(s.results()):
        assert (r.selected, r.feasible, r.status) == o.result(q), (tag, q)
        assert s.annotations(q) == o.annotations(q), (tag, q)


@pytest.mark.gpu
def test_known_volume_clusters():
    for i, doc in enumerate(_known_clusters()):
        _queue_parity(doc, i)


@pytest.mark.gpu
@pytest.mark.parametrize("zone", [True, False], ids=["default-profile", "without-VolumeZone"])
def test_volume_edge_cluster(zone):
    doc = edge.generate_edge("volumes")
    if not zone:
        doc["profile"] = make_profile([p for p in DEFAULT_PROFILE if p[0] != "VolumeZone"], doc["profile"]["seed"])
    _queue_parity(doc, zone)
    # drop-in cycle path, with the per-extension-point ABI rebuilding the annotations
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    d = dict(doc)
    d["queue"] = []
    s.load_cluster(d)
    names = [n["metadata"]["name"] for n in doc["nodes"]]
    for i, pod in enumerate(doc["queue"][:60]):
        q, r = s.cycle(pod, commit=True)
        assert (r.selected, r.feasible, r.status) == o.result(i), i
        if i % 3 == 0:
            got, ora = rebuild(s, q, doc["profile"], names, r.status), o.annotations(i)
            for k, v in got.items():
                assert v == ora[k], (i, k)


@pytest.mark.gpu
def test_rwop_conflict_preemption():
    doc = kv.rwop_preemption_cluster()
    _queue_parity(doc, "rwop")
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.schedule()
    assert s.postfilter_result(0) == o.nominated(0) == (2, ["default/holder"])
