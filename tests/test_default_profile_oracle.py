"""CPU checks of the oracle's restatement of the rest of the default profile
(no GPU).  Known answers worked out by hand from the upstream v1.30 formulas:

* ImageLocality (image_locality.go): scaledImageScore = int64(size x numNodes/totalNodes),
  score = 100 x (clamp(sum, 23Mi, 1000Mi x containers) - 23Mi) / (1000Mi x containers - 23Mi);
* NodePorts (HostPortInfo.CheckConflict): 0.0.0.0 conflicts with every IP of the
  same (protocol, port); a specific IP with itself and 0.0.0.0; protocol defaults to TCP;
* NodeUnschedulable / NodeName messages; VolumeBinding / volume plugins recorded as
  Skip ("") for pods without volumes; DefaultBinder / VolumeBinding binding records.
"""
import json

from _oracle import Oracle
from ksg import generator as g

P = "kube-scheduler-simulator.sigs.k8s.io/"
Mi = g.Mi


def _doc(nodes, queue, pods=()):
    return {"profile": g.make_profile(g.DEFAULT_PROFILE, 7), "nodes": nodes, "pods": list(pods), "queue": queue}


def _ann(o, q, key):
    return json.loads(o.annotations(q)[P + key])


def test_image_locality_known_answer():
    img = [(("example.com/app:1",), 500 * Mi)]
    nodes = [g.node_obj("n0", 4000, 8 * g.Gi, images=img), g.node_obj("n1", 4000, 8 * g.Gi)]
    o = Oracle(_doc(nodes, [g.pod_obj("p", [g.req(100, 64 * Mi)], images={0: "example.com/app:1"})]))
    o.schedule(record=3)
    sc = _ann(o, 0, "score-result")
    # spread 1/2: 250Mi; 100 * (250 - 23) / (1000 - 23) = 23
    assert sc["n0"]["ImageLocality"] == "23"
    assert sc["n1"]["ImageLocality"] == "0"


def test_image_locality_tagless_name_and_cap():
    img = [(("docker.io/library/big:latest",), 3000 * Mi)]
    nodes = [g.node_obj(f"n{i}", 4000, 8 * g.Gi, images=img) for i in range(2)]
    pod = g.pod_obj("p", [g.req(100, 64 * Mi), g.req(100, 64 * Mi)],
                    images={0: "docker.io/library/big", 1: "docker.io/library/big"})
    o = Oracle(_doc(nodes, [pod]))
    o.schedule(record=3)
    # two containers: 6000Mi capped at 2000Mi -> 100
    assert _ann(o, 0, "score-result")["n0"]["ImageLocality"] == "100"


def test_node_ports_conflicts():
    def port(hp, proto=None, ip=None):
        d = {"containerPort": hp, "hostPort": hp}
        if proto:
            d["protocol"] = proto
        if ip:
            d["hostIP"] = ip
        return d

    nodes = [g.node_obj(f"n{i}", 4000, 8 * g.Gi) for i in range(4)]
    bound = [g.pod_obj("b0", [g.req(100, Mi)], node="n0", ports={0: [port(80)]}),
             g.pod_obj("b1", [g.req(100, Mi)], node="n1", ports={0: [port(80, ip="10.0.0.1")]}),
             g.pod_obj("b2", [g.req(100, Mi)], node="n2", ports={0: [port(80, "UDP")]})]
    q = [g.pod_obj("wild", [g.req(100, Mi)], ports={0: [port(80)]}),
         g.pod_obj("ip1", [g.req(100, Mi)], ports={0: [port(80, ip="10.0.0.1")]}),
         g.pod_obj("ip2", [g.req(100, Mi)], ports={0: [port(80, "TCP", "10.0.0.2")]})]
    o = Oracle(_doc(nodes, q, bound))
    o.schedule(record=3)
    bad = "node(s) didn't have free ports for the requested pod ports"
    f = _ann(o, 0, "filter-result")  # 0.0.0.0:80/TCP: n0 (wildcard) and n1 (any IP) conflict
    assert f["n0"]["NodePorts"] == bad and f["n1"]["NodePorts"] == bad and f["n2"]["NodePorts"] == "passed"
    # "wild" landed on n2 or n3; 10.0.0.1 conflicts with n0 (0.0.0.0), n1 (same IP), wherever "wild" went
    f1 = _ann(o, 1, "filter-result")
    assert f1["n0"]["NodePorts"] == bad and f1["n1"]["NodePorts"] == bad
    f2 = _ann(o, 2, "filter-result")
    assert f2["n1"]["NodePorts"] == "passed"  # 10.0.0.2 vs 10.0.0.1: no conflict
    assert _ann(o, 0, "prefilter-result-status")["NodePorts"] == "success"


def test_unschedulable_nodename_and_skip_records():
    nodes = [g.node_obj("n0", 4000, 8 * g.Gi, unschedulable=True), g.node_obj("n1", 4000, 8 * g.Gi)]
    q = [g.pod_obj("a", [g.req(100, Mi)]), g.pod_obj("b", [g.req(100, Mi)], nodeName="n0")]
    o = Oracle(_doc(nodes, q))
    o.schedule(record=3)
    f = _ann(o, 0, "filter-result")
    assert f["n0"] == {"NodeUnschedulable": "node(s) were unschedulable"}
    assert o.result(0)[0] == 1
    pre = _ann(o, 0, "prefilter-result-status")
    for name in ("VolumeRestrictions", "EBSLimits", "GCEPDLimits", "NodeVolumeLimits", "AzureDiskLimits",
                 "VolumeBinding", "VolumeZone", "NodePorts"):
        assert pre[name] == ""
    assert _ann(o, 0, "bind-result") == {"DefaultBinder": "success"}
    assert _ann(o, 0, "reserve-result") == {"VolumeBinding": "success"}
    # "b" names the cordoned node: unschedulable on n0, NodeName on n1; DefaultPreemption records both
    assert o.result(1)[2] == 1
    fb = _ann(o, 1, "filter-result")
    assert fb["n1"]["NodeName"] == "node(s) didn't match the requested node name"
    assert _ann(o, 1, "postfilter-result") == {"n0": {}, "n1": {}}
    assert _ann(o, 1, "bind-result") == {}


def test_preemption_known_answers():
    """DefaultPreemption dry run by hand (default_preemption.go / preemption.go v1.30.4):
    SelectVictimsOnNode removes every lower-priority pod, then reprieves the most
    important first; pickOneNodeForPreemption prefers the node whose highest
    victim priority is lowest; preemptionPolicy Never and requests above the
    allocatable (UnschedulableAndUnresolvable) nominate nothing."""
    nodes = [g.node_obj("a", 4000, 8 * g.Gi), g.node_obj("b", 4000, 8 * g.Gi)]
    bound = [g.pod_obj("low", [g.req(3000, Mi)], node="a", priority=0),
             g.pod_obj("mid", [g.req(500, Mi)], node="a", priority=100),
             g.pod_obj("b-mid", [g.req(3500, Mi)], node="b", priority=100)]
    bound[0]["status"] = {"startTime": "2025-01-02T00:00:00Z"}
    q = [g.pod_obj("hi", [g.req(2000, Mi)], priority=1000),
         g.pod_obj("never", [g.req(2000, Mi)], priority=1000, preemptionPolicy="Never"),
         g.pod_obj("huge", [g.req(5000, Mi)], priority=1000)]
    prof = g.make_profile([("NodeResourcesFit", 1), ("DefaultPreemption", 1)], 7)
    o = Oracle({"profile": prof, "nodes": nodes, "pods": bound, "queue": q})
    o.schedule(record=3)
    assert [o.result(i)[2] for i in range(3)] == [1, 1, 1]
    # node a: remove low+mid, fits; reprieve mid (2.5 <= 4 cpu), low stays a victim (5.5 > 4)
    # node b: victim b-mid (priority 100) -> a wins on the lowest highest victim priority
    assert o.nominated(0) == (0, ["default/low"])
    assert _ann(o, 0, "postfilter-result") == {"a": {"DefaultPreemption": "preemption victim"}, "b": {}}
    assert o.nominated(1) == (-1, [])  # preemptionPolicy Never
    assert o.nominated(2) == (-1, [])  # 5 cpu > allocatable 4: UnschedulableAndUnresolvable everywhere
    assert _ann(o, 2, "postfilter-result") == {"a": {}, "b": {}}
