"""Diagnostic: timeline of k_window per window (s_memtime / s_memrealtime stamps).

Per window W, 24 slots at [W*24]: fixup block (shader clock) 0 start, 1 staged,
2 prior-node evaluations, 3 starting guess, 4 Jacobi converged, 5 flushed,
7 Jacobi iterations; realtime (100 MHz): 8 ~first eval-block start of window W
(evaluated one launch earlier), 9 last tile eval done, 10 last merge done,
11 fixup start, 12 fixup end.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
from ksg import Scheduler, generator as g  # noqa: E402

n_nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
n_pods = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 2
doc = g.generate(cfg, n_nodes=n_nodes, n_pods=n_pods)
s = Scheduler(doc["profile"])
s.load_cluster(doc)
L = s.L
L.ksg_debug_fixup_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
n = s.queue_len
nw = (n + 31) // 32
s.schedule()  # warm
s.reset()
L.ksg_debug_fixup_stamps(s.h, n, None)
s.schedule()
buf = (ctypes.c_uint64 * (8 * n))()
L.ksg_debug_fixup_stamps(s.h, n, buf)
bs = [buf[j * 32:(j + 1) * 32] for j in range(nw)]
lt = [buf[nw * 32 + j * 4:nw * 32 + (j + 1) * 4] for j in range(nw)]  # persistent loop: loop top, ready, after wait


def med(v):
    v = sorted(v)
    return v[len(v) // 2]


names = ["stage", "prior eval", "guess", "jacobi", "flush"]
for k in range(5):
    v = [x[k + 1] - x[k] for x in bs[1:]]
    print(f"fixup {names[k]:12s} median {med(v):6d} mean {sum(v)/len(v):8.1f} cycles")
it = [x[7] for x in bs[1:]]
print("jacobi iterations: mean", sum(it) / len(it), "max", max(it), "hist", {k: it.count(k) for k in sorted(set(it))})
print("fixup block total median", med([x[5] - x[0] for x in bs[1:]]), "cycles")
ns = 10.0  # s_memrealtime: 100 MHz
ev = [((~x[8]) & 0xFFFFFFFFFFFFFFFF) for x in bs]
print("realtime (us): eval start->last tile eval", med([(bs[j][9] - ev[j]) / 100 for j in range(1, nw)]))
print("realtime (us): eval block duration max", med([bs[j][28] / 100 for j in range(1, nw)]),
      "mean", med([bs[j][29] / max(bs[j][31], 1) / 100 for j in range(1, nw)]), "blocks", bs[1][31])
nb_ = [max(bs[j][31], 1) for j in range(1, nw)]
print("eval wave-0 cycles per block: eval", med([bs[j][13] / nb_[j - 1] for j in range(1, nw)]),
      "sort+merge", med([bs[j][14] / nb_[j - 1] for j in range(1, nw)]),
      "LDS merge+tile store+arrive", med([bs[j][15] / nb_[j - 1] for j in range(1, nw)]),
      "(of eval: load wait", med([bs[j][18] / nb_[j - 1] for j in range(1, nw)]), ")")
print("realtime (us): first -> last eval block start", med([(bs[j][30] - ev[j]) / 100 for j in range(1, nw)]))
print("realtime (us): eval start->last merge", med([(bs[j][10] - ev[j]) / 100 for j in range(1, nw)]))
# window j's eval runs in the same launch as window j-1's fixup
print("realtime (us): fixup W-1 start -> eval W start", med([(ev[j] - bs[j - 1][11]) / 100 for j in range(2, nw)]))
print("realtime (us): fixup duration", med([(x[12] - x[11]) / 100 for x in bs[1:]]))
print("realtime (us): fixup W-1 end -> fixup W start", med([(bs[j][11] - bs[j - 1][12]) / 100 for j in range(2, nw)]))
print("realtime (us): last merge of W -> fixup W start", med([(bs[j][11] - bs[j][10]) / 100 for j in range(2, nw)]))
print("realtime (us): window period", med([(bs[j][11] - bs[j - 1][11]) / 100 for j in range(2, nw)]))
for lab, i0, i1 in [("prior eval", 1, 16), ("keys->LDS+sync", 16, 17), ("pmask+sync", 17, 2),
                     ("iteration 1", 3, 19), ("it1 phase A", 3, 21), ("it1 barrier A", 21, 22), ("it1 phase B", 22, 23),
                     ("it1 barrier B", 23, 19), ("A: start->find", 3, 24), ("A: find/chain", 24, 25),
                     ("A: find/chain->phase A end", 25, 21),
                     ("flush: P_W+publish", 4, 6), ("flush: patches", 6, 5),
                     ("flush: P_W built (wave 0)", 4, 26), ("flush: P_W acks", 26, 27), ("flush: barrier+publish", 27, 6)]:
    print(f"fixup {lab:14s} median {med([x[i1] - x[i0] for x in bs[1:]]):6d}")
if any(x[0] for x in lt):
    print("loop top: windows ready at the flush", sum(1 for x in lt[1:] if x[1]), "of", nw - 1)
    print("realtime (us): fixup W-1 end -> loop top", med([(lt[j][0] - bs[j - 1][12]) / 100 for j in range(2, nw)]))
    print("realtime (us): loop-top wait", med([(lt[j][2] - lt[j][0]) / 100 for j in range(2, nw)]),
          "(not ready only:", med([(lt[j][2] - lt[j][0]) / 100 for j in range(2, nw) if not lt[j][1]] or [0]), ")")
    print("realtime (us): after wait -> fixup start", med([(bs[j][11] - lt[j][2]) / 100 for j in range(2, nw)]))
two = [x for x in bs[1:] if x[7] >= 2]
if two:
    print("iteration 2 median", med([x[20] - x[19] for x in two]), "windows", len(two))
