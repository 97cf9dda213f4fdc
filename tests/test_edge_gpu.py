"""GPU parity on the edge-case family (ksg/edge.py): MostAllocated and
RequestedToCapacityRatio over four resources, BalancedAllocation beyond cpu /
memory, ephemeral-storage and scalar requests, init / sidecar containers, pod
overhead, matchFields, DoesNotExist, Gt / Lt on non-numeric values, tolerations
of every form, minDomains, node inclusion policies, matchLabelKeys, terminating
bound pods, namespaces lists and selectors, hardPodAffinityWeight 0 / 3 and
ignorePreferredTermsOfExistingPods.  Every pod's selection, feasible count and
status equal the oracle's; annotations byte-identical on a sample; the drop-in
cycle path and the per-extension-point ABI agree too."""
import pytest

from _oracle import Oracle
from ksg import Scheduler, edge
from test_plugin_api_gpu import rebuild


def without_queue(doc):
    """The document with no pending pods (the drop-in cycle API receives them one by one)."""
    d = dict(doc)
    if "queue" in d:
        d["queue"] = []
    else:
        d["pods"] = [p for p in d["pods"] if p["spec"].get("nodeName")]
    return d

VARIANTS = list(edge.EDGE_VARIANTS)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_edge_queue_matches_oracle(variant):
    doc = edge.generate_edge(variant)
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.keep_outputs(0, s.queue_len)
    s.schedule()
    res = s.results()
    assert [s.queue_pod(q) for q in range(s.queue_len)] == o.queue_names(), variant
    assert s.gated_pods() == o.gated_names(), variant
    for q, r in enumerate(res):
        assert (r.selected, r.feasible, r.status) == o.result(q), (variant, q)
    for q in range(0, len(res), 3):
        assert s.annotations(q) == o.annotations(q), (variant, q)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_edge_cycle_and_extension_points(variant):
    doc = edge.generate_edge(variant, n_pods=60)
    o = Oracle(doc)
    o.schedule(record=3)
    s = Scheduler(doc["profile"])
    s.load_cluster(without_queue(doc))
    names = [n["metadata"]["name"] for n in doc["nodes"]]
    for i, pod in enumerate(o.ordered_queue(doc)):  # the framework runs them in its queue order
        q, r = s.cycle(pod, commit=True)
        assert (r.selected, r.feasible, r.status) == o.result(i), (variant, i)
        if i % 4 == 0:
            got, ora = rebuild(s, q, doc["profile"], names, r.status), o.annotations(i)
            for k, v in got.items():
                assert v == ora[k], (variant, i, k)
