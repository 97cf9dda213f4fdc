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


def _cfg5_shard_worker(rank, world, port, step, sample, out):
    """One rank of a node-sharded cfg5 step (host exchange over gloo: the ranks
    share the box's one MI355X); every rank generates the same cluster itself."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "kube-scheduler-simulator-p9_amd"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ksg import Scheduler as S, generator as gen
    blob = gen.generate_native(5, n_nodes=1_000_000, n_pods=step)
    prof = json.loads(blob[:blob.index(b',"nodes"')] + b"}")["profile"]
    s = S(prof, device=0, shard_rank=rank, shard_count=world)
    s.set_exchange_host(world)
    s.load_cluster(blob)
    del blob
    _progress(f"cfg5 sharded rank {rank} loaded")
    s.whatif(0, step)
    out[rank] = [(r.selected, r.feasible, r.status) for r in s.results(0, sample)]
    out[f"sched{rank}"] = sum(1 for r in s.results(0, step) if r.status == 0)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_cfg5_full_size_sharded_2rank_matches_oracle():
    """BASELINE cfg5 node-sharded: 1,000,000 nodes over 2 ranks (500,000 each), one
    4,096-pod what-if step; per-pod normalisers and argmax keys merged across the
    ranks (k_whatif_merge after each pass); the first 64 pods of the step equal the
    oracle's on both ranks."""
    import socket
    import torch.multiprocessing as mp
    step, sample = 4096, 64
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_cfg5_shard_worker, args=(2, port, step, sample, out), nprocs=2, join=True)
        got = {r: out[r] for r in range(2)}
        sched = [out["sched0"], out["sched1"]]
    assert sched[0] == sched[1] and sched[0] > step // 2
    blob = g.generate_native(5, n_nodes=1_000_000, n_pods=step)
    o = Oracle(blob)
    del blob
    _progress("cfg5 sharded: oracle loaded")
    o.whatif(sample, workers=WORKERS, record=0)
    want = [o.result(q) for q in range(sample)]
    for r in range(2):
        assert got[r] == want, f"rank {r} differs"
