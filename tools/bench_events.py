"""Latency of cluster-event batches (ksg_apply_events): in-place device delta vs
snapshot re-encode, on a generated cluster (cfg2 / cfg4 node and pod mix: bound-pod
additions; cfg3: node label / taint rewrites).

    python tools/bench_events.py [--cfg 4] [--nodes 20000] [--existing 80000]
Prints one JSON line per (path, batch size).
"""
import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
from ksg import Scheduler, generator as g  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=4)
    ap.add_argument("--nodes", type=int, default=20000)
    ap.add_argument("--existing", type=int, default=80000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    t0 = time.time()
    if a.cfg == 4:
        doc = g.generate(4, n_nodes=a.nodes, n_existing=a.existing, n_pods=256, n_zones=20)
    elif a.cfg == 3:
        doc = g.generate(3, n_nodes=a.nodes, n_pods=256)
    else:
        doc = g.generate(2, n_nodes=a.nodes, n_pods=256)
    print(f"generated in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)
    s.schedule()
    names = [n["metadata"]["name"] for n in doc["nodes"]]
    src = doc.get("pods", [])[:64]
    seq = [0]

    nodes = copy.deepcopy(doc["nodes"])
    tiers = sorted({n["metadata"]["labels"].get("tier", "") for n in nodes} - {""})
    taints = []
    for n in nodes:
        for t in (n.get("spec") or {}).get("taints") or []:
            if t not in taints:
                taints.append(t)

    def node_batch(b):  # label + taint rewrites with known values (the in-place path)
        ev = []
        for j in range(b):
            i = (seq[0] * 7919) % len(nodes)
            x = nodes[i]
            x["metadata"]["labels"]["tier"] = tiers[seq[0] % len(tiers)]
            spec = x.setdefault("spec", {})
            spec["taints"] = [taints[seq[0] % len(taints)]] if not spec.get("taints") else []
            seq[0] += 1
            ev.append({"op": "updateNode", "node": copy.deepcopy(x)})
        return ev

    def batch(b):
        if a.cfg == 3:
            return node_batch(b)
        ev = []
        for j in range(b):
            p = copy.deepcopy(src[j % len(src)])
            p["metadata"]["name"] = f"evt-{seq[0]:07d}"
            p["spec"]["nodeName"] = names[(seq[0] * 7919) % len(names)]
            seq[0] += 1
            ev.append({"op": "addPod", "pod": p})
        return ev

    for reencode in (False, True):
        for b in (1, 64):
            ts = []
            for _ in range(a.reps):
                ev = batch(b)
                t = time.perf_counter()
                s.apply_events(ev, reencode=reencode)
                ts.append(time.perf_counter() - t)
            ts.sort()
            print(json.dumps({"cfg": a.cfg, "nodes": len(names), "bound_pods": len(doc.get("pods", [])),
                              "events": "updateNode labels+taints" if a.cfg == 3 else "addPod",
                              "path": "reencode" if reencode else "in-place", "batch": b,
                              "ms_median": 1e3 * ts[len(ts) // 2], "ms_min": 1e3 * ts[0]}), flush=True)


if __name__ == "__main__":
    main()
