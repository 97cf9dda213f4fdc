"""Every pod of the queues bench.py times, against the oracle (VERDICT r05 "next" 1).

bench.py times whole 10,000-pod queues (cfg2, cfg3, cfg4) and 4,096-pod what-if
steps with binds between them (cfg5).  The other parity tests stop at a queue
prefix; these run the exact benched path -- the context bench.py builds
(`sharded_scheduler`, default env), a warm-up step, `reset()`, then the timed
step's `schedule(0, n, wait=False)` + `wait()` (`ksg_schedule_queue`) or two
consecutive `whatif` steps (`ksg_whatif`) -- and compare (selected node,
feasible count, status) of every pod with the fixtures
`tests/golden/fullqueue/cfg*.json`, which the CPU oracle wrote
(`tests/golden/make_fullqueue.py`, run in the build container).

Reference: the per-pod Filter -> Score -> NormalizeScore -> Reserve sequence,
simulator/scheduler/plugin/wrappedplugin.go:523 -> :420 -> :388 -> :616.
"""
import hashlib
import json
import os
import sys
import time

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.dirname(HERE))

import make_fullqueue as mf  # noqa: E402


def _progress(msg):
    p = os.environ.get("KSG_PROGRESS")
    if p:
        with open(p, "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


def _fixture(c):
    with open(mf.path(c)) as f:
        d = json.load(f)
    return d, mf.unpack(d["results_i32_zlib_b64"])


def _profile(blob):
    return json.loads(blob[:blob.index(b',"nodes"')] + b"}")["profile"]


def _diff(got, want):
    bad = [(q, tuple(g), tuple(int(x) for x in w)) for q, (g, w) in enumerate(zip(got, want)) if tuple(g) != tuple(w)]
    return bad


@pytest.mark.parametrize("c", [2, 3])
def test_fullqueue_fixture_matches_generator(c):
    """CPU: the fixture's cluster hash is the generator's, so the GPU test compares
    against the queue the bench actually builds (cfg2 / cfg3; cfg4 / cfg5 are
    hashed on the GPU box where they are generated anyway)."""
    d, rows = _fixture(c)
    assert rows.shape == (d["pods"], 3)
    assert hashlib.sha256(mf.cluster_blob(c)).hexdigest() == d["cluster_sha256"]
    assert int((rows[:, 2] == 0).sum()) == d["scheduled"]


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("c", [2, 3, 4])
def test_benched_queue_matches_oracle_every_pod(c):
    import torch
    from ksg.distributed import sharded_scheduler
    d, want = _fixture(c)
    blob = mf.cluster_blob(c)
    assert hashlib.sha256(blob).hexdigest() == d["cluster_sha256"], "generator changed: regenerate the fixture"
    _progress(f"cfg{c} generated")
    s = sharded_scheduler(_profile(blob), torch, 0, 1, 0)
    s.load_cluster(blob)
    del blob
    n = s.queue_len
    assert n == d["pods"]
    wr0, rc0 = s.window_runs(), s.run_counts()
    for _ in range(2):  # bench.py time_queue(): warm-up step, then a timed step from the same snapshot
        s.reset()
        s.schedule(0, n, wait=False)
        s.wait()
    _progress(f"cfg{c} scheduled on the GPU")
    if c in (2, 3):
        assert s.batch_path and s.window_runs() >= wr0 + 2, "the persistent window loop did not run"
    else:
        assert s.run_counts()[1] > rc0[1], "the persistent chain (k_chain_run) did not run"
    got = [(r.selected, r.feasible, r.status) for r in s.results()]
    bad = _diff(got, want)
    assert not bad, f"cfg{c}: {len(bad)} of {n} pods differ, first {bad[:5]}"


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_benched_whatif_steps_match_oracle_every_pod():
    """cfg5: two consecutive 4,096-pod what-if steps at 1,000,000 nodes (the second
    scored after the first step's placements are bound), every pod compared."""
    import torch
    from ksg.distributed import sharded_scheduler
    d, want = _fixture(5)
    blob = mf.cluster_blob(5)
    assert hashlib.sha256(blob).hexdigest() == d["cluster_sha256"], "generator changed: regenerate the fixture"
    _progress("cfg5 generated")
    s = sharded_scheduler(_profile(blob), torch, 0, 1, 0)
    s.load_cluster(blob)
    del blob
    _progress("cfg5 loaded")
    P = mf.WHATIF_STEP
    assert s.queue_len == d["pods"] == 2 * P
    for k in range(2):
        s.whatif(k * P, P, wait=False)
        s.wait()
    _progress("cfg5 two steps done")
    assert s.whatif_class_chunks() > 0, "the class path bench_whatif times did not run"
    got = [(r.selected, r.feasible, r.status) for r in s.results(0, 2 * P)]
    bad = _diff(got, want)
    assert not bad, f"cfg5: {len(bad)} of {2 * P} pods differ, first {bad[:5]}"
