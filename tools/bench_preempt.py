"""DefaultPreemption dry-run latency at scale: pods that fit nowhere without
preempting, on a cluster of N nodes full of lower-priority bound pods
(ksg/edge.py's preempt family, queue pods made large and high-priority).  Each
queue run stops after every pod that may preempt and runs its dry run on the
device state of its own cycle (host.cpp Cluster::preempt), so the wall time per
pod is the cycle plus the victim search.  The batched search (every potential
node in one dry run, the reprieve in lockstep) and the per-node probes run in
separate processes (KSG_PREEMPT_BATCH); their nominations must agree.

usage: python tools/bench_preempt.py [--nodes 50000] [--pods 8] [--per-node-pods 2] [--per-node-nodes 2000]"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))


def make_doc(nodes, pods, spread=0):
    """The preempt family at `nodes` nodes, 4 random bound pods per node plus one
    lowest-priority 4-core filler on every node (no node has 6 free cores), and
    `pods` queue pods of priority 5000 asking 6 cores: every node is a potential
    node (Unschedulable: insufficient cpu), the 8-core ones fit once their
    lower-priority pods are gone, so every pod runs a full victim search.  The bound
    pods carry no anti-affinity terms (one applying to the incoming pod takes the
    per-node search: ksg's preempt_batched).  spread=1: every queue pod also carries a
    ScheduleAnyway zone spread constraint and a required hostname anti-affinity term
    on its own first label (both batched since round 6)."""
    from ksg import edge
    from ksg.generator import pod_obj, req
    doc = edge.gen_preempt(n_nodes=nodes, n_existing=4 * nodes, n_pods=pods)
    low = min(edge.PRIORITIES)
    for b in doc["pods"]:  # (an existing pod's anti-affinity term would apply to the incoming pods: per-node search)
        b["spec"].pop("affinity", None)
    for i, n in enumerate(doc["nodes"]):
        doc["pods"].append(pod_obj(f"fill-{i:07d}", [req(4000, 1024 * 1024 * 1024)], node=n["metadata"]["name"],
                                   priority=low))
    for p in doc["queue"]:
        sp = p["spec"]
        sp["priority"] = 5000
        for k in ("preemptionPolicy", "topologySpreadConstraints", "affinity", "nodeSelector", "tolerations"):
            sp.pop(k, None)
        for c in sp["containers"]:
            c["resources"] = {"requests": {"cpu": "6000m", "memory": "2Gi"}}
            c.pop("ports", None)
        if spread:
            sel = {"matchLabels": dict(list(p["metadata"].get("labels", {}).items())[:1])}
            sp["topologySpreadConstraints"] = [{"maxSkew": 1, "topologyKey": edge.ZONE,
                                                "whenUnsatisfiable": "ScheduleAnyway", "labelSelector": sel}]
            sp["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": sel, "topologyKey": edge.HOSTNAME}]}}
    return doc


def one(batch, nodes, pods, warm=0, spread=0):
    env = dict(os.environ, KSG_PREEMPT_BATCH=str(batch))
    code = f"""
import json, sys, time
sys.path.insert(0, {os.path.join(ROOT, 'tools')!r})
sys.path.insert(0, {os.path.join(ROOT, 'kube-scheduler-simulator-p9_amd')!r})
import torch
from bench_preempt import make_doc
from ksg import Scheduler
doc = make_doc({nodes}, {pods}, {spread})
print("[child] document built", file=sys.stderr, flush=True)
s = Scheduler(doc["profile"])
s.load_cluster(doc)
print("[child] cluster loaded", file=sys.stderr, flush=True)
import ctypes
# the victim store's warm-up after the load (host.cpp Cluster::warm_step, a thread of
# the context): WARM=1 waits for it before the first pod, 0 starts right after the load
s.L.ksg_debug_victim_warm.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
wms = ctypes.c_double(-1)
if {warm}:
    while s.L.ksg_debug_victim_warm(s.h, ctypes.byref(wms)) == 0:
        time.sleep(0.005)
s.L.ksg_debug_preempt_times.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
def split():
    pt = (ctypes.c_double * 4)()
    s.L.ksg_debug_preempt_times(s.h, pt, 1)
    k = 1e-3 / max(pt[3], 1)
    return {{"potential_nodes": pt[0] * k, "victims_programs": pt[1] * k, "search": pt[2] * k, "searches": pt[3]}}
s.L.ksg_debug_preempt_times(s.h, None, 1)
t = time.perf_counter()
s.schedule(0, 1)  # (the first search compiles the bound pods' programs and uploads the victim store)
t1 = time.perf_counter()
first = split()
if s.queue_len > 1:
    s.schedule(1)
dt = time.perf_counter() - t
rest = split() if s.queue_len > 1 else None
noms = [s.postfilter_result(q) for q in range(s.queue_len)]
warm = s.L.ksg_debug_victim_warm(s.h, ctypes.byref(wms))
print(json.dumps({{"ms_per_pod": dt * 1e3 / s.queue_len, "nominated": sum(1 for n in noms if n[0] >= 0),
                  "victim_store_warm": {{"waited": bool({warm}), "state": warm, "load_to_store_ms": wms.value}},
                  "first_pod_ms": (t1 - t) * 1e3,
                  "ms_per_pod_after_first": (dt - (t1 - t)) * 1e3 / max(s.queue_len - 1, 1),
                  "host_split_ms_per_search": {{"first": first, "after_first": rest}},
                  "batched": s.preempt_batched(), "noms": noms,
                  "res": [(r.selected, r.feasible, r.status) for r in s.results()]}}))
"""
    print(f"[bench_preempt] batch={batch} nodes={nodes} pods={pods}", file=sys.stderr, flush=True)
    out = subprocess.run([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, text=True, timeout=900)
    if out.returncode != 0:
        raise RuntimeError(f"exit {out.returncode}")
    return json.loads(out.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50000)
    ap.add_argument("--pods", type=int, default=8)
    ap.add_argument("--per-node-pods", type=int, default=2)
    ap.add_argument("--spread", type=int, default=0, help="1: preemptors with a ScheduleAnyway spread constraint "
                    "and hostname anti-affinity (make_doc)")
    ap.add_argument("--per-node-nodes", type=int, default=2000,
                    help="cluster size of the batched vs per-node comparison (a per-node search is one dry run per node)")
    a = ap.parse_args()
    b = one(1, a.nodes, a.pods, spread=a.spread)
    bw = one(1, a.nodes, a.pods, warm=1, spread=a.spread)
    k = a.per_node_pods
    bs = one(1, a.per_node_nodes, k, spread=a.spread)
    p = one(0, a.per_node_nodes, k, spread=a.spread)
    print(json.dumps({"nodes": a.nodes, "bound_pods": 5 * a.nodes, "spread": a.spread,
                      "batched": {"pods": a.pods, "ms_per_pod": b["ms_per_pod"], "nominated": b["nominated"],
                                  "first_pod_ms": b["first_pod_ms"], "ms_per_pod_after_first": b["ms_per_pod_after_first"],
                                  "batched_searches": b["batched"], "split": b["host_split_ms_per_search"],
                                  "victim_store_warm": b["victim_store_warm"]},
                      "batched_after_warmup": {"pods": a.pods, "ms_per_pod": bw["ms_per_pod"], "nominated": bw["nominated"],
                                               "first_pod_ms": bw["first_pod_ms"],
                                               "ms_per_pod_after_first": bw["ms_per_pod_after_first"],
                                               "split": bw["host_split_ms_per_search"],
                                               "victim_store_warm": bw["victim_store_warm"],
                                               "same_nominations": bw["noms"] == b["noms"] and bw["res"] == b["res"]},
                      "compare": {"nodes": a.per_node_nodes, "pods": k,
                                  "batched_ms_per_pod": bs["ms_per_pod"], "per_node_ms_per_pod": p["ms_per_pod"],
                                  "nominated": p["nominated"], "batched_searches": bs["batched"],
                                  "same_nominations": bs["noms"] == p["noms"] and bs["res"] == p["res"]}}, indent=1))


if __name__ == "__main__":
    main()
