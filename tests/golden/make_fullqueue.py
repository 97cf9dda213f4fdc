"""Full-length placement fixtures for the queues bench.py times (VERDICT r05 "next" 1).

The bench times whole queues: cfg2 (5,000 nodes x 10,000 pods), cfg3 (15,000 x
10,000), cfg4 (50,000 nodes, 200,000 bound pods, 10,000 pods) and cfg5's what-if
steps (1,000,000 nodes, 4,096 pods per step, binds between steps).  These
fixtures hold the CPU oracle's (selected node, feasible count, status) for every
pod of those queues -- 12 bytes a pod, zlib + base64 -- with the SHA-256 of the
generated cluster document so a generator change is caught before the
comparison.  tests/test_fullqueue_gpu.py runs the benched path against them.

The oracle is test infrastructure (tests/_oracle.py); this script runs here, in
the build container, not on the GPU box.  Run:

    python tests/golden/make_fullqueue.py [cfg ...]      # default: 2 3 4 5
"""
import base64
import hashlib
import json
import os
import sys
import time
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
sys.path.insert(0, os.path.dirname(HERE))

WORKERS = int(os.environ.get("KSG_FIXTURE_WORKERS", os.cpu_count() or 8))

# the sizes bench.py / bench_whatif.py time (BASELINE.json configs[1..4])
CASES = {
    2: dict(n_nodes=5000, n_pods=10000),
    3: dict(n_nodes=15000, n_pods=10000),
    4: dict(n_nodes=50000, n_existing=200000, n_pods=10000, n_zones=20),
    5: dict(n_nodes=1_000_000, n_pods=2 * 4096),   # two what-if steps, binds between them
}
WHATIF_STEP = 4096


def cluster_blob(c):
    """The cluster document exactly as the bench builds it: the Python generator for
    cfg2 (bench.py run()), the native twin for the others (extra_config, bench_whatif)."""
    from ksg import generator as g
    if c == 2:
        return g.dumps(g.generate(2, **CASES[2])).encode()
    return g.generate_native(c, **CASES[c])


def pack(rows):
    a = np.asarray(rows, dtype="<i4").reshape(-1)
    return base64.b64encode(zlib.compress(a.tobytes(), 9)).decode()


def unpack(s):
    return np.frombuffer(zlib.decompress(base64.b64decode(s)), dtype="<i4").reshape(-1, 3)


def path(c):
    return os.path.join(HERE, "fullqueue", f"cfg{c}.json")


def make(c):
    from _oracle import Oracle
    t0 = time.time()
    blob = cluster_blob(c)
    sha = hashlib.sha256(blob).hexdigest()
    o = Oracle(blob)
    n = o.n_queue
    steps = []
    if c == 5:
        for k in range(0, n, WHATIF_STEP):
            o.whatif(min(WHATIF_STEP, n - k), workers=WORKERS, record=0)
            steps.append(min(WHATIF_STEP, n - k))
            print(f"cfg5 step {len(steps)} done, {time.time() - t0:.0f} s", flush=True)
    else:
        done = 0
        while done < n:
            done += o.schedule(n=min(1000, n - done), workers=WORKERS, record=0)
            print(f"cfg{c}: {done}/{n} pods, {time.time() - t0:.0f} s", flush=True)
    rows = [o.result(q) for q in range(n)]
    doc = {"config": c, "sizes": CASES[c], "cluster_sha256": sha, "pods": n,
           "whatif_steps": steps or None,
           "scheduled": sum(1 for r in rows if r[2] == 0),
           "results_i32_zlib_b64": pack(rows),
           "note": "(selected node index, feasible count, status) per queue pod, from the CPU oracle"}
    with open(path(c), "w") as f:
        json.dump(doc, f, indent=1)
    print(f"cfg{c}: wrote {path(c)} ({n} pods, {doc['scheduled']} scheduled) in {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    for c in (int(x) for x in (sys.argv[1:] or ["2", "3", "4", "5"])):
        make(c)
