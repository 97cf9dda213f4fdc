"""Diagnostic: per-phase cycle breakdown of the batch fixup loop (s_memtime stamps)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
from ksg import Scheduler, generator as g  # noqa: E402

doc = g.generate(2, n_nodes=5000, n_pods=640)
s = Scheduler(doc["profile"])
s.load_cluster(doc)
L = s.L
L.ksg_debug_fixup_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
n = s.queue_len
s.schedule()  # warm
s.reset()
L.ksg_debug_fixup_stamps(s.h, n, None)
s.schedule()
buf = (ctypes.c_uint64 * (8 * n))()
L.ksg_debug_fixup_stamps(s.h, n, buf)
# per batch: [0] start [1] staged [2] guess+prep [3] converged [4] iterations [5] flushed
bs = [buf[j * 8:(j + 1) * 8] for j in range(32, n, 32)]
names = ["stage", "guess+prep", "iterations", "flush"]
for k, (i0, i1) in enumerate([(0, 1), (1, 2), (2, 3), (3, 5)]):
    v = sorted(x[i1] - x[i0] for x in bs)
    print(f"fixup {names[k]:12s} median {v[len(v)//2]:6d} mean {sum(v)/len(v):8.1f} cycles")
it = [x[4] for x in bs]
print("fixup iterations: mean", sum(it) / len(it), "max", max(it), "hist", {k: it.count(k) for k in sorted(set(it))})
tot = sorted(x[5] - x[0] for x in bs)
print("per batch total median", tot[len(tot) // 2], "cycles")

# k_batch_eval per-wave phases (last batch of a run)
L.ksg_debug_eval_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
s.reset()
L.ksg_debug_eval_stamps(s.h, 1, None, None)
s.schedule()
T = (s.n_nodes + 255) // 256
m = T * 32 * 4 * 8
eb = (ctypes.c_uint64 * m)()
L.ksg_debug_eval_stamps(s.h, 1, eb, None)
waves = [eb[i * 8:(i + 1) * 8] for i in range(T * 32 * 4)]
waves = [w for w in waves if w[0] and w[5]]
names = ["load row", "eval", "store+key", "sort", "merge+write"]
for k in range(5):
    v = sorted(w[k + 1] - w[k] for w in waves)
    print(f"eval {names[k]:12s} median {v[len(v)//2]:6d} cycles")
t0 = min(w[0] for w in waves)
t1 = max(w[5] for w in waves)
print("eval kernel span (s_memtime ticks)", t1 - t0, "waves", len(waves))
starts = sorted(w[0] - t0 for w in waves)
print("wave start spread: median", starts[len(starts)//2], "max", starts[-1])
