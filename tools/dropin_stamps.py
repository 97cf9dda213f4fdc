"""Where a drop-in cycle's k_eval spends its time (cfg2 by default): block 0's
s_memrealtime deltas per k_eval point (table_chain.hip CS_*), averaged over n
ksg_cycle(commit=0) + ksg_cycle_view + ksg_reserve cycles on an empty-queue
context, with the cycle's host split beside them.

usage: python tools/dropin_stamps.py [--cfg 2] [--n 200] [--warmup 20]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from chain_stamps import NAMES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=2)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    import torch
    assert torch.cuda.is_available()
    from ksg import Scheduler, generator as g
    doc = json.loads(g.generate_native(a.cfg))
    pods = doc["queue"][:a.warmup + a.n]
    doc["queue"] = []
    s = Scheduler(doc["profile"])
    s.load_cluster(doc)

    def run(ps, tag):
        for i, p in enumerate(ps):
            p["metadata"]["name"] = f"{tag}-{i:05d}"
            q, r = s.cycle(p, commit=False)
            v = s.cycle_view(q)
            v.release()
            if r.selected >= 0:
                s.reserve(q, r.selected)
    run(pods[:a.warmup], "warm")
    s.L.ksg_debug_eval_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    s.L.ksg_debug_eval_stamps(s.h, 1, None, None)
    run(pods[a.warmup:], "pod")
    out = (ctypes.c_uint64 * 64)()
    n = ctypes.c_size_t()
    s.L.ksg_debug_eval_stamps(s.h, 1, out, ctypes.byref(n))
    last = out[63] or 1
    res = {NAMES.get(k, str(k)): round(out[k] / (last if 24 <= k <= 27 else a.n) * 0.01, 3)
           for k in range(64) if out[k] and k not in (48, 49, 63)}
    print(json.dumps({"cfg": a.cfg, "cycles": a.n, "select_samples_block0_last": out[63],
                      "views_fused": s.views_fused(), "us_avg_block0_since_entry": res}, indent=1))


if __name__ == "__main__":
    main()
