"""GPU parity of the whole default profile (scheduler_test.go:531-557): the
hot-path plugins plus NodeUnschedulable, NodeName, NodePorts, ImageLocality,
the volume plugins' Skip records and the binding-cycle records.

Each case runs the HIP engine and the CPU oracle on the same cluster and
compares every pod's selection and every annotation byte-for-byte.  The cases
push the new plugins to their edges: host ports saturating nodes (NodePorts
failures, unschedulable pods), wildcard vs specific host IPs, pods naming a
node (and one naming no node), cordoned nodes with and without the toleration,
images listed under several names, a pod with no containers' images on any
node, and Reserve/Unreserve of host-port pods through the drop-in cycle API.
"""
import copy
import json

import pytest

from _oracle import Oracle
from ksg import Scheduler, generator as g

P = "kube-scheduler-simulator.sigs.k8s.io/"


def _compare(doc, s=None, keep=True):
    o = Oracle(doc)
    o.schedule(record=3)
    if s is None:
        s = Scheduler(doc["profile"])
        s.load_cluster(doc)
        s.keep_outputs(0, s.queue_len)
        s.schedule()
    for q, r in enumerate(s.results()):
        assert (r.selected, r.feasible, r.status) == o.result(q), (q, r, o.result(q))
        a, b = s.annotations(q), o.annotations(q)
        for k in b:
            assert a.get(k) == b[k], f"pod {q} {k}:\n gpu    {a.get(k, '')[:500]}\n oracle {b[k][:500]}"
    return o, s


def _port(hp, proto=None, ip=None):
    d = {"containerPort": hp, "hostPort": hp}
    if proto:
        d["protocol"] = proto
    if ip:
        d["hostIP"] = ip
    return d


def edge_cluster():
    """12 nodes, half cordoned or image-rich; a queue that exhausts host port 8080."""
    doc = g.generate(1, n_nodes=12, n_pods=0)
    nodes = doc["nodes"]
    for i in (1, 4, 7):
        nodes[i]["spec"]["unschedulable"] = True
    nodes[2]["status"]["images"] = [{"names": ["registry.k8s.io/app-3:1.3", "app3-alias:v1"], "sizeBytes": 900 << 20}]
    nodes[3]["status"]["images"] = [{"names": ["quay.io/big/model:latest"], "sizeBytes": 1800 << 20}]
    q = []
    for j in range(16):  # 16 pods wanting 8080 on 0.0.0.0: 9 uncordoned nodes, then NodePorts fails everywhere
        q.append(g.pod_obj(f"web-{j:03d}", [g.req(100, 64 * g.Mi)], images={0: "registry.k8s.io/app-3:1.3"},
                           ports={0: [_port(8080)]}))
    tol = [{"key": "node.kubernetes.io/unschedulable", "operator": "Exists", "effect": "NoSchedule"}]
    q.append(g.pod_obj("tolerant", [g.req(100, 64 * g.Mi)], ports={0: [_port(8080)]}, tolerations=tol))
    q.append(g.pod_obj("udp-8080", [g.req(100, 64 * g.Mi)], ports={0: [_port(8080, "UDP")]}))
    q.append(g.pod_obj("ip-9100", [g.req(100, 64 * g.Mi)], ports={0: [_port(9100, ip="10.0.0.9")]}))
    q.append(g.pod_obj("ip-5353", [g.req(100, 64 * g.Mi)], ports={0: [_port(5353, "UDP", "10.0.0.1")]}))
    q.append(g.pod_obj("wild-5353", [g.req(100, 64 * g.Mi)], ports={0: [_port(5353, "UDP")]}))
    q.append(g.pod_obj("named", [g.req(100, 64 * g.Mi)], nodeName="node-0000005"))
    q.append(g.pod_obj("named-cordoned", [g.req(100, 64 * g.Mi)], nodeName="node-0000004"))
    q.append(g.pod_obj("named-nowhere", [g.req(100, 64 * g.Mi)], nodeName="node-9999999"))
    q.append(g.pod_obj("alias-image", [g.req(100, 64 * g.Mi), g.req(100, 64 * g.Mi)],
                       images={0: "app3-alias:v1", 1: "quay.io/big/model"}))
    q.append(g.pod_obj("big-only", [g.req(100, 64 * g.Mi)], images={0: "quay.io/big/model"}))
    q.append(g.pod_obj("init", [g.req(100, 64 * g.Mi)], images={0: "busybox"},
                       initContainers=[{"name": "i", "image": "registry.k8s.io/app-3:1.3"}]))
    doc["queue"] = q
    return doc


@pytest.mark.gpu
def test_default_profile_cfg1_matches_oracle():
    """BASELINE configs[0] at its full size: 100 nodes, all 1,000 queue pods of the
    default profile, every selection and every annotation byte for byte."""
    _compare(g.generate(1, n_nodes=100, n_pods=1000))


@pytest.mark.gpu
def test_default_profile_edges_match_oracle():
    o, s = _compare(edge_cluster())
    res = s.results()
    assert sum(1 for r in res[:16] if r.status == 1) >= 6  # 8080 exhausted on the schedulable nodes
    names = [p["metadata"]["name"] for p in edge_cluster()["queue"]]
    assert res[names.index("named")].selected == 5
    assert res[names.index("named-nowhere")].status == 1
    f = json.loads(s.annotations(names.index("named-cordoned"))[P + "filter-result"])
    assert f["node-0000004"]["NodeUnschedulable"] == "node(s) were unschedulable"


@pytest.mark.gpu
def test_default_profile_cycles_reserve_unreserve():
    """Cycle API: host-port pods assumed / unassumed (UsedPorts delta and its reversal)."""
    doc = edge_cluster()
    queue = doc["queue"]
    base = copy.deepcopy(doc)
    base["queue"] = []
    s = Scheduler(doc["profile"])
    s.load_cluster(base)
    placed = []
    for i, pod in enumerate(queue[:12]):
        q, r = s.cycle(pod, commit=True)
        placed.append((q, r.selected))
    # release every 8080 pod, then the next cycles see the ports free again
    for q, sel in placed:
        if sel >= 0:
            s.unreserve(q)
    # oracle: the same queue indices (tie-break hash input), the released pods
    # replaced by pods no node fits (they leave the snapshot unchanged)
    ref = copy.deepcopy(doc)
    ref["queue"] = [g.pod_obj(f"void-{k}", [g.req(10 ** 9, 64 * g.Mi)]) for k in range(12)] + queue[12:]
    o = Oracle(ref)
    o.schedule(record=3)
    for i, pod in enumerate(queue[12:], start=12):
        q, r = s.cycle(pod, commit=True)
        assert q == i
        assert (r.selected, r.feasible, r.status) == o.result(i), (i, pod["metadata"]["name"])
        a, b = s.annotations(q), o.annotations(i)
        for k in b:
            assert a.get(k) == b[k], (i, k)


@pytest.mark.gpu
def test_image_locality_scores_abi():
    """ksg_scores at ImageLocality's profile position == the oracle's score-result."""
    doc = edge_cluster()
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.keep_outputs(0, s.queue_len)
    s.schedule()
    pos = doc["profile"]["plugins"].index("ImageLocality")
    o = Oracle(doc)
    o.schedule(record=3)
    names = [p["metadata"]["name"] for p in doc["queue"]]
    for name in ("alias-image", "big-only", "init"):
        q = names.index(name)
        sc = json.loads(o.annotations(q)[P + "score-result"])
        codes = s.filter_codes(q)
        got = s.scores(q, pos)
        for i, nd in enumerate(doc["nodes"]):
            nm = nd["metadata"]["name"]
            if nm in sc:
                assert codes[i] == 0xFFFFFFFF
                assert str(got[i]) == sc[nm]["ImageLocality"], (name, nm)


@pytest.mark.gpu
def test_unmodelled_volumes_refused():
    """PersistentVolumeClaims run on the device (tests/test_volume_gpu.py); inline cloud
    disks, and claims on a sharded context, are refused instead of approximated."""
    doc = g.generate(1, n_nodes=4, n_pods=2)
    doc["queue"][1]["spec"]["volumes"] = [{"name": "d", "gcePersistentDisk": {"pdName": "disk"}}]
    with pytest.raises(Exception):
        Scheduler(doc["profile"]).load_cluster(doc)
    doc["queue"][1]["spec"]["volumes"] = [{"name": "d", "persistentVolumeClaim": {"claimName": "c"}}]
    Scheduler(doc["profile"]).load_cluster(doc)  # a missing claim: VolumeRestrictions' PreFilter rejects the pod
    with pytest.raises(Exception):
        Scheduler(doc["profile"], shard_rank=0, shard_count=2).load_cluster(doc)


@pytest.mark.gpu
def test_mixed_priorities_sharded_refused():
    """DefaultPreemption's dry run runs on unsharded contexts (test_preempt_gpu.py);
    a sharded context refuses a cluster of mixed priorities instead of approximating."""
    doc = g.generate(1, n_nodes=4, n_pods=2)
    doc["queue"][1]["spec"]["priority"] = 1000
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    t = Scheduler(doc["profile"], shard_rank=0, shard_count=2)
    with pytest.raises(Exception):
        t.load_cluster(doc)
