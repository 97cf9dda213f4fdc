"""Drop-in cycle latency breakdown at cfg4 size (run under rocprofv3 --kernel-trace
--memory-copy-trace --stats for the device side): the queue's first pods are
scheduled (tables warm), then n copies of queue pods go through ksg_cycle
(commit=0), ksg_cycle_view_acquire and ksg_reserve, each timed on the host; the
view is acquired twice per pod (the second time: no cycle in between).

usage: python tools/dropin_probe.py [--nodes 50000] [--existing 200000] [--n 100]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50000)
    ap.add_argument("--existing", type=int, default=200000)
    ap.add_argument("--pods", type=int, default=400)
    ap.add_argument("--n", type=int, default=100)
    a = ap.parse_args()
    import torch  # noqa: F401  (device init as in bench.py)
    from ksg import Scheduler, generator as g
    blob = g.generate_native(4, n_nodes=a.nodes, n_pods=a.pods, n_existing=a.existing, n_zones=20)
    doc = json.loads(blob)
    s = Scheduler(doc["profile"])
    s.load_cluster(blob)
    s.schedule(0, 200)
    t = {"cycle": 0.0, "view": 0.0, "view2": 0.0, "release": 0.0, "reserve": 0.0}
    for i, p in enumerate(doc["queue"][200:200 + a.n]):
        p = json.loads(json.dumps(p))
        p["metadata"]["name"] = f"dropin-{i:05d}"
        t0 = time.perf_counter()
        q, r = s.cycle(p, commit=False)
        t1 = time.perf_counter()
        v = s.cycle_view(q)
        t2 = time.perf_counter()
        v.release()
        t3 = time.perf_counter()
        v2 = s.cycle_view(q)
        t4 = time.perf_counter()
        v2.release()
        t5 = time.perf_counter()
        if r.selected >= 0:
            s.reserve(q, r.selected)
        t6 = time.perf_counter()
        t["cycle"] += t1 - t0
        t["view"] += t2 - t1
        t["release"] += t3 - t2
        t["view2"] += t4 - t3
        t["reserve"] += t6 - t5
    print(json.dumps({k: v * 1e6 / a.n for k, v in t.items()} | {"nodes": a.nodes, "n": a.n}), flush=True)


if __name__ == "__main__":
    main()
