"""Where a table-chain cycle spends its time (cfg4): block 0's s_memrealtime
deltas per kernel point, averaged over the pods of a run (table_chain.hip CS_*).

usage: python tools/chain_stamps.py [--nodes N] [--existing E] [--pods P]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))

NAMES = {13: "k_eval: entry + gap stamp", 14: "k_eval (run): row-only Fit/BA done", 15: "k_eval (run): flag wait done", 7: "k_eval: inputs issued (vids, row, setup)", 11: "k_eval: +1 stamp", 12: "k_eval: +2 stamps", 8: "k_eval: slot vids in LDS", 9: "k_eval: lookups issued",
         10: "k_eval: setup (minMatchNum, IPA bits)",
         3: "k_eval: filter done",
         4: "k_eval: scores done", 5: "k_eval: block reduce", 6: "k_eval: partials written",
         16: "k_final: raw loads issued", 17: "k_final: partials folded", 18: "k_final: ipa bits",
         19: "k_final: normalized + key", 20: "k_final: block key written",
         24: "select (last block): partials loaded", 25: "select (last block): block reduce", 26: "select (last block): summary + row atomics",
         27: "select (last block): class tables", 40: "gap k_eval->k_final entry",
         42: "gap k_final->next k_eval entry"}

RUN_NAMES = {30: "eval + partial granules stored", 31: "every partial seen", 39: "partials block-reduced",
             32: "partials folded", 47: "normalised + keyed", 33: "key granules stored", 34: "every key seen, argmax",
             50: "pod done (owner commit, next wait set)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50000)
    ap.add_argument("--existing", type=int, default=200000)
    ap.add_argument("--pods", type=int, default=600)
    a = ap.parse_args()
    import torch
    assert torch.cuda.is_available()
    from ksg import Scheduler, generator as g
    blob = g.generate_native(4, n_nodes=a.nodes, n_pods=a.pods, n_existing=a.existing)
    doc = json.loads(blob)
    s = Scheduler(doc["profile"])
    s.load_cluster(blob)
    s.schedule(0, 64)
    s.L.ksg_debug_eval_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    s.L.ksg_debug_eval_stamps(s.h, 1, None, None)
    s.schedule(64, s.queue_len - 64)
    out = (ctypes.c_uint64 * 64)()
    n = ctypes.c_size_t()
    s.L.ksg_debug_eval_stamps(s.h, 1, out, ctypes.byref(n))
    pods = s.queue_len - 64  # every cycle's block 0 stamps; the select's only when block 0 arrives last
    last = out[63] or 1
    res = {NAMES.get(k, str(k)): round(out[k] / (last if 24 <= k <= 27 else pods) * 0.01, 3)
           for k in sorted(NAMES, key=lambda k: (k not in (13, 14, 15, 7, 11, 12, 8, 9, 10), k)) if out[k]}
    rep = {"pods": pods, "select_samples": last, "us_avg_block0": res}
    if out[35]:  # persistent segments (k_chain_run)
        rep["k_chain_run_us_since_pod_start_block0"] = {RUN_NAMES[k]: round(out[k] / out[35] * 0.01, 3) for k in (30, 31, 39, 32, 47, 33, 34, 50)}
        rep["k_chain_run_pods_block0"] = out[35]
        rep["k_chain_run_pods_read_ahead_block0"] = out[40]
        rep["k_chain_run_flag_wait_us_block0"] = round(out[38] / out[35] * 0.01, 3)
        rep["k_chain_run_latest_block_partial_us"] = round(out[51] / out[35] * 0.01, 3)
        rep["k_chain_run_latest_block_key_us"] = round(out[53] / out[35] * 0.01, 3)
        rep["rec_block_eval_us: folds, lds record, barrier, end"] = [round(out[i] / out[35] * 0.01, 3) for i in (0, 1, 2, 61)]
        rep["k_eval_block0_wave_scores_done_us"] = [round((out[56 + w] - out[60]) / out[35] * 0.01, 3) for w in range(4)]
        if out[37]:
            rep["k_chain_run_owner_commit_us"] = round(out[36] / out[37] * 0.01, 3)
            rep["k_chain_run_owner_atomics_issued_us"] = round(out[44] / out[37] * 0.01, 3)
            rep["k_chain_run_owner_atomics_drained_us"] = round(out[45] / out[37] * 0.01, 3)
            rep["k_chain_run_assume_items_avg"] = round(out[46] / out[37], 2)
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
