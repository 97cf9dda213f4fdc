"""Short run for PMC passes: 64 batches of the cfg2 batch path (no CPU baseline)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
from ksg import Scheduler, generator as g  # noqa: E402

doc = g.generate(2, n_nodes=5000, n_pods=2048)
s = Scheduler(doc["profile"])
s.load_cluster(doc)
s.schedule()
print("ok", s.queue_len)
