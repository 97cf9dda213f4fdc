"""Parity at the BASELINE.json workload sizes (VERDICT r01 "configs untested").

cfg4: 50,000 nodes in 20 zones, 200,000 existing pods, PodTopologySpread +
InterPodAffinity (+ Fit / BalancedAllocation); 300 queue pods scheduled back to
back, every selection / feasible count / status equal to the oracle's, and the
rendered annotations (filter-result, score-result, finalscore-result, ...)
byte-equal for 10 sampled pods.

cfg5: 1,000,000 nodes, one what-if step of 4,096 pods against the frozen
snapshot; pods inside a step are independent, so the oracle scores a sampled
subset (the first 64 pods of the step) and the first pod's annotations.

Clusters come from the native generator twin (ksg_synth_cluster; tests/test_synth.py
pins it to the Python generator).
"""
import json
import os
import time

import pytest

from _oracle import Oracle
from ksg import Scheduler, generator as g

WORKERS = 16  # oracle parallelize.Until workers (the box's CPU share)


def _progress(msg):
    """Long steps report to $KSG_PROGRESS (a file the GPU runner watches for liveness)."""
    p = os.environ.get("KSG_PROGRESS")
    if p:
        with open(p, "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_cfg4_full_size_matches_oracle():
    n_pods, keep0, nkeep = 300, 120, 10
    blob = g.generate_native(4, n_nodes=50000, n_existing=200000, n_pods=n_pods, n_zones=20)
    prof = json.loads(blob[:blob.index(b',"nodes"')] + b"}")["profile"]
    s = Scheduler(prof)
    _progress("cfg4 generated")
    s.load_cluster(blob)
    _progress("cfg4 loaded")
    assert s.n_nodes == 50000
    s.keep_outputs(keep0, nkeep)
    s.schedule()
    res = s.results()
    _progress("cfg4 scheduled on the GPU")
    o = Oracle(blob)
    o.schedule(keep0, workers=WORKERS, record=0)
    o.schedule(nkeep, workers=WORKERS, record=3)
    o.schedule(n_pods - keep0 - nkeep, workers=WORKERS, record=0)
    bad = [(q, (r.selected, r.feasible, r.status), o.result(q)) for q, r in enumerate(res)
           if (r.selected, r.feasible, r.status) != o.result(q)]
    assert not bad, f"{len(bad)} of {n_pods} pods differ, first {bad[:5]}"
    assert sum(1 for r in res if r.status == 0) > n_pods // 2
    for q in range(keep0, keep0 + nkeep):
        a, b = s.annotations(q), o.annotations(q)
        for k in b:
            assert a.get(k) == b[k], (q, k)


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_cfg5_full_size_whatif_step_matches_oracle():
    step, sample = 4096, 64
    blob = g.generate_native(5, n_nodes=1_000_000, n_pods=step)
    prof = json.loads(blob[:blob.index(b',"nodes"')] + b"}")["profile"]
    s = Scheduler(prof)
    _progress("cfg5 generated")
    s.load_cluster(blob)
    _progress("cfg5 loaded")
    assert s.n_nodes == 1_000_000
    s.keep_outputs(0, 1)
    s.whatif(0, step)
    res = s.results(0, step)
    assert sum(1 for r in res if r.status == 0) > step // 2
    _progress("cfg5 what-if step done")
    o = Oracle(blob)
    _progress("cfg5 oracle loaded")
    o.whatif(sample, workers=WORKERS, record=0)
    got = [(r.selected, r.feasible, r.status) for r in res[:sample]]
    assert got == [o.result(q) for q in range(sample)]
    del o
    o1 = Oracle(blob)  # pod 0 rendered: its result in a one-pod step equals its result in the 4,096-pod step
    o1.whatif(1, workers=WORKERS, record=3)
    _progress("cfg5 oracle pod 0 rendered")
    a, b = s.annotations(0), o1.annotations(0)
    for k in b:
        assert a.get(k) == b[k], k
