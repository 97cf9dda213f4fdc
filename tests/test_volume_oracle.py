"""Known answers of the volume plugins on the CPU oracle, worked by hand from
upstream v1.30.4 (plugins/volumerestrictions, volumebinding, volumezone,
nodevolumelimits) — the reference holds no vectors for them (parity unpinned
against Go; these pin the restatement to the upstream code paths)."""
import json

import pytest

from _oracle import Oracle
from ksg import edge
from ksg.generator import Gi, Mi, ZONE, HOSTNAME, make_profile, node_obj, pod_obj, req

P = "kube-scheduler-simulator.sigs.k8s.io/"
PROFILE = [("NodeResourcesFit", 1), ("VolumeRestrictions", 1), ("NodeVolumeLimits", 1), ("VolumeBinding", 1),
           ("VolumeZone", 1)]


def cluster(queue_pod, pvcs, pvs=(), classes=(), bound=()):
    nodes = [node_obj("n0", 8000, 32 * Gi, labels={ZONE: "zone-a"}), node_obj("n1", 8000, 32 * Gi, labels={ZONE: "zone-b"}),
             node_obj("n2", 8000, 32 * Gi)]
    return {"profile": make_profile(PROFILE, 7), "nodes": nodes, "pods": list(bound), "queue": [queue_pod],
            "pvcs": list(pvcs), "pvs": list(pvs), "storageClasses": list(classes)}


def with_claims(name, *claims, node=None, ns="default"):
    return pod_obj(name, [req(100, 128 * Mi)], node=node, ns=ns,
                   volumes=[{"name": f"v{i}", "persistentVolumeClaim": {"claimName": c}} for i, c in enumerate(claims)])


WFFC = {"metadata": {"name": "wffc"}, "provisioner": "csi.example.com", "volumeBindingMode": "WaitForFirstConsumer"}


def run(doc):
    o = Oracle(doc)
    o.schedule(record=3)
    a = o.annotations(0)
    return o.result(0), {k[len(P):]: json.loads(v) if v.startswith("{") else v for k, v in a.items()}


def test_local_pv_prefilter_result():
    """GetEligibleNodes: a claim bound to a PV with hostname In [n1] restricts the cycle to n1."""
    pv = edge._pv("pv-1", "wffc", claim=("default", "c1"), affinity={"nodeSelectorTerms": [
        {"matchExpressions": [{"key": HOSTNAME, "operator": "In", "values": ["n1"]}]}]})
    (sel, feas, st), a = run(cluster(with_claims("p", "c1"), [edge._pvc("c1", "default", volume="pv-1", cls="wffc",
                                                                        bound=True)], [pv], [WFFC]))
    assert a["prefilter-result"] == {"VolumeBinding": ["n1"]}
    assert set(a["filter-result"]) == {"n1"} and (sel, feas, st) == (1, 1, 0)
    assert a["prefilter-result-status"]["VolumeZone"] == ""  # no zone labels on the PV: Skip
    assert a["filter-result"]["n1"] == {"NodeResourcesFit": "passed", "VolumeRestrictions": "passed",
                                        "NodeVolumeLimits": "passed", "VolumeBinding": "passed"}


def test_volume_zone_labels():
    """VolumeZone: n0 matches the PV's zone, n1 does not, n2 carries no zone label and passes."""
    pv = edge._pv("pv-z", "wffc", claim=("default", "cz"), labels={ZONE: "zone-a"})
    (sel, feas, st), a = run(cluster(with_claims("p", "cz"), [edge._pvc("cz", "default", volume="pv-z", cls="wffc",
                                                                        bound=True)], [pv], [WFFC]))
    f = a["filter-result"]
    assert f["n0"]["VolumeZone"] == "passed" and f["n2"]["VolumeZone"] == "passed"
    assert f["n1"]["VolumeZone"] == "node(s) had no available volume zone"
    assert feas == 2 and st == 0


def test_read_write_once_pod_conflict():
    """VolumeRestrictions: a ReadWriteOncePod claim already used by a bound pod fails every node (Unschedulable)."""
    pvc = edge._pvc("rw", "default", volume="pv-rw", cls="wffc", bound=True, modes=("ReadWriteOncePod",))
    pv = edge._pv("pv-rw", "wffc", claim=("default", "rw"))
    (sel, feas, st), a = run(cluster(with_claims("p", "rw"), [pvc], [pv], [WFFC], bound=[with_claims("b", "rw", node="n2")]))
    msg = "node has pod using PersistentVolumeClaim with the same name and ReadWriteOncePod access mode"
    assert all(row["VolumeRestrictions"] == msg for row in a["filter-result"].values())
    assert (sel, feas, st) == (-1, 0, 1)


def test_provisioning_topology_and_selected_node():
    """A WaitForFirstConsumer claim is provisioned where the class's allowedTopologies allow;
    a selected-node annotation pins it to that node (checkVolumeProvisions / FindPodVolumes)."""
    cls = dict(WFFC, metadata={"name": "zb"}, allowedTopologies=[{"matchLabelExpressions": [
        {"key": ZONE, "values": ["zone-b"]}]}])
    (sel, feas, st), a = run(cluster(with_claims("p", "new"), [edge._pvc("new", "default", cls="zb")], [], [cls]))
    bind = "node(s) didn't find available persistent volumes to bind"
    f = a["filter-result"]
    assert f["n0"]["VolumeBinding"] == bind and f["n2"]["VolumeBinding"] == bind
    assert f["n1"]["VolumeBinding"] == "passed" and (sel, feas) == (1, 1)
    pinned = edge._pvc("new", "default", cls="wffc", ann={"volume.kubernetes.io/selected-node": "n2"})
    (sel, feas, st), a = run(cluster(with_claims("p", "new"), [pinned], [], [WFFC]))
    assert (sel, feas) == (2, 1) and a["filter-result"]["n0"]["VolumeBinding"] == bind


def test_prefilter_rejections():
    """Unbound immediate claims (VolumeBinding) and missing claims (VolumeRestrictions, first in
    profile order) reject the pod at PreFilter: no Filter runs."""
    imm = {"metadata": {"name": "imm"}, "provisioner": "csi.example.com", "volumeBindingMode": "Immediate"}
    (_, _, st), a = run(cluster(with_claims("p", "c"), [edge._pvc("c", "default", cls="imm")], [], [imm]))
    assert a["prefilter-result-status"]["VolumeBinding"] == "pod has unbound immediate PersistentVolumeClaims"
    assert a["filter-result"] == {} and st == 1
    (_, _, st), a = run(cluster(with_claims("p", "nope"), []))
    assert a["prefilter-result-status"] == {"NodeResourcesFit": "success",
                                            "VolumeRestrictions": 'persistentvolumeclaim "nope" not found'}
    assert st == 1


def test_bound_claim_reasons():
    """checkBoundClaims: a PV whose affinity no node matches -> node conflict everywhere; a missing PV ->
    the PVNotExist reason (without VolumeZone in the profile, whose PreFilter would reject first)."""
    pv = edge._pv("pv-x", "wffc", claim=("default", "c"), affinity={"nodeSelectorTerms": []})
    (_, feas, _), a = run(cluster(with_claims("p", "c"), [edge._pvc("c", "default", volume="pv-x", cls="wffc", bound=True)],
                                  [pv], [WFFC]))
    assert feas == 0 and all(r["VolumeBinding"] == "node(s) had volume node affinity conflict"
                             for r in a["filter-result"].values())
    doc = cluster(with_claims("p", "c"), [edge._pvc("c", "default", volume="pv-gone", cls="wffc", bound=True)], [], [WFFC])
    doc["profile"] = make_profile(PROFILE[:-1], 7)
    (_, feas, _), a = run(doc)
    assert feas == 0 and all(r["VolumeBinding"] == "node(s) unavailable due to one or more pvc(s) bound to "
                             "non-existent pv(s)" for r in a["filter-result"].values())


def test_no_volumes_skip():
    (_, feas, _), a = run(cluster(pod_obj("p", [req(100, 128 * Mi)]), []))
    assert feas == 3
    assert all(a["prefilter-result-status"][n] == "" for n in ("VolumeRestrictions", "NodeVolumeLimits", "VolumeBinding",
                                                                "VolumeZone"))
    assert all(set(r) == {"NodeResourcesFit"} for r in a["filter-result"].values())


@pytest.mark.parametrize("bad", ["shared_wffc", "static_pv", "inline"])
def test_unmodelled_inputs_refused(bad):
    doc = cluster(with_claims("p", "c"), [edge._pvc("c", "default", cls="wffc")], [], [WFFC])
    if bad == "shared_wffc":
        doc["queue"].append(with_claims("q", "c"))
    elif bad == "static_pv":
        doc["pvs"] = [edge._pv("free", "wffc")]
    else:
        doc["queue"][0]["spec"]["volumes"].append({"name": "x", "gcePersistentDisk": {"pdName": "d"}})
    with pytest.raises(Exception):
        Oracle(doc)


def rwop_preemption_cluster():
    """A ReadWriteOncePod claim held by a low-priority pod on n2: the high-priority pod that
    wants it fails VolumeRestrictions (Unschedulable) everywhere, so preemption may help;
    evicting the holder clears the conflict (RemovePod) on n2 only."""
    pvc = edge._pvc("rw", "default", volume="pv-rw", cls="wffc", bound=True, modes=("ReadWriteOncePod",))
    holder = with_claims("holder", "rw", node="n2")
    holder["spec"]["priority"] = 10
    other = pod_obj("other", [req(100, 128 * Mi)], node="n0")
    other["spec"]["priority"] = 10
    pod = with_claims("p", "rw")
    pod["spec"]["priority"] = 1000
    doc = cluster(pod, [pvc], [edge._pv("pv-rw", "wffc", claim=("default", "rw"))], [WFFC], bound=[holder, other])
    doc["profile"] = make_profile(PROFILE + [("DefaultPreemption", 1)], 7)
    return doc


def test_rwop_conflict_preemption():
    o = Oracle(rwop_preemption_cluster())
    o.schedule(record=3)
    assert o.result(0) == (-1, 0, 1)
    assert o.nominated(0) == (2, ["default/holder"])


def test_csi_attach_limits():
    """NodeVolumeLimits (csi.go): n0 allows 1 volume of the driver (CSINode count) and already
    holds one of another claim -> "node(s) exceed max volume count" (Unschedulable); n1's
    limit 2 comes from the legacy allocatable key; a volume already attached on a node is
    not counted twice; n2 declares no limit."""
    drv = "csi.example.com"
    pvs = [edge._pv("pv-a", "wffc", claim=("default", "a")), edge._pv("pv-b", "wffc", claim=("default", "b"))]
    pvcs = [edge._pvc("a", "default", volume="pv-a", cls="wffc", bound=True),
            edge._pvc("b", "default", volume="pv-b", cls="wffc", bound=True)]
    doc = cluster(with_claims("p", "a"), pvcs, pvs, [WFFC], bound=[with_claims("h0", "b", node="n0"),
                                                                   with_claims("h1", "b", node="n1")])
    doc["csiNodes"] = [{"metadata": {"name": "n0"}, "spec": {"drivers": [{"name": drv, "allocatable": {"count": 1}}]}}]
    doc["nodes"][1]["status"]["allocatable"]["attachable-volumes-csi-" + drv] = "2"
    (sel, feas, st), a = run(doc)
    f = a["filter-result"]
    assert f["n0"]["NodeVolumeLimits"] == "node(s) exceed max volume count"
    assert f["n1"]["NodeVolumeLimits"] == "passed" and f["n2"]["NodeVolumeLimits"] == "passed"
    assert feas == 2
    # the pod's volume already attached on n0 (a holder of "a" there): nothing new, n0 passes
    doc["pods"].append(with_claims("h2", "a", node="n0"))
    (sel, feas, st), a = run(doc)
    assert a["filter-result"]["n0"]["NodeVolumeLimits"] == "passed" and feas == 3
