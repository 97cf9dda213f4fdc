"""Host split of bench.py's cfg2 step (reset, schedule(wait=False), wait) on one
context, after two warm-up steps: where the step's time goes outside the
persistent window loop (k_window_run is ~6.42 ms of a ~6.6 ms step).

usage: python tools/step_probe.py
"""
import sys, time, json
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))), "kube-scheduler-simulator-p9_amd"))
import torch
from ksg import generator as g
from ksg.distributed import sharded_scheduler
blob = g.dumps(g.generate(2, n_nodes=5000, n_pods=10000)).encode()
prof = json.loads(blob[:blob.index(b',"nodes"')] + b"}")["profile"]
s = sharded_scheduler(prof, torch, 0, 1, 0)
s.load_cluster(blob)
n = s.queue_len
for _ in range(2):
    s.reset(); s.schedule(0, n, wait=False); s.wait()
torch.cuda.synchronize()
rows = []
for _ in range(6):
    t0 = time.perf_counter(); s.reset(); t1 = time.perf_counter()
    s.schedule(0, n, wait=False); t2 = time.perf_counter(); s.wait(); t3 = time.perf_counter()
    rows.append(((t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6, (t3 - t0) * 1e6))
for r in rows: print("reset %.0f us  schedule %.0f us  wait %.0f us  total %.0f us" % r)
