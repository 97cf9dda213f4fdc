"""cfg4 A/B: us per pod of the table chain with an engine switch off and on
(--var: KSG_RUN persistent segments by default, KSG_SOLO one-launch cycles), same
cluster, results checked equal (and against the oracle on the first pods).
usage: python tools/cfg4_ab.py [--var KSG_RUN] [--nodes N] [--pods P] [--check C]"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def one(var, val, nodes, pods, existing, steps):
    env = dict(os.environ, **{var: str(val)})
    code = f"""
import json, sys, time
sys.path.insert(0, {os.path.join(ROOT, 'kube-scheduler-simulator-p9_amd')!r})
import torch
from ksg import Scheduler, generator as g
blob = g.generate_native(4, n_nodes={nodes}, n_pods={pods}, n_existing={existing}, n_zones=20)
prof = json.loads(blob[:blob.index(b',"nodes"')] + b"}}")["profile"]
s = Scheduler(prof)
s.load_cluster(blob)
s.schedule(); s.reset()
t = time.perf_counter()
for _ in range({steps}):
    s.reset(); s.schedule()
dt = (time.perf_counter() - t) / {steps}
print(json.dumps({{"us_per_pod": dt * 1e6 / {pods}, "paths": s.path_counts(True) + s.run_counts(),
                  "res": [(r.selected, r.feasible, r.status) for r in s.results()]}}))
"""
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        raise RuntimeError(out.stderr[-3000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--var", default="KSG_RUN")
    ap.add_argument("--vals", default="0,1", help="the variable's off,on values")
    ap.add_argument("--nodes", type=int, default=50000)
    ap.add_argument("--existing", type=int, default=200000)
    ap.add_argument("--pods", type=int, default=2000)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--check", type=int, default=200, help="pods checked against the oracle")
    a = ap.parse_args()
    v0, v1 = a.vals.split(",")
    r0 = one(a.var, v0, a.nodes, a.pods, a.existing, a.steps)
    r1 = one(a.var, v1, a.nodes, a.pods, a.existing, a.steps)
    same = r0["res"] == r1["res"]
    from _oracle import Oracle
    from ksg import generator as g
    o = Oracle(g.generate_native(4, n_nodes=a.nodes, n_pods=a.pods, n_existing=a.existing, n_zones=20))
    o.schedule(a.check, workers=16, record=0)
    ora = [o.result(q) for q in range(a.check)]
    print(json.dumps({"nodes": a.nodes, "pods": a.pods,
                      "var": a.var,
                      "off": {"us_per_pod": r0["us_per_pod"], "paths": r0["paths"]},
                      "on": {"us_per_pod": r1["us_per_pod"], "paths": r1["paths"]},
                      "results_equal": same,
                      "oracle_ok_off": [tuple(x) for x in r0["res"][:a.check]] == ora,
                      "oracle_ok_on": [tuple(x) for x in r1["res"][:a.check]] == ora}, indent=1))


if __name__ == "__main__":
    main()
