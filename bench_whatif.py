#!/usr/bin/env python3
"""Secondary benchmark: BASELINE.json configs[4] (cfg5), the what-if batch.

1,000,000 nodes (cfg3 node distribution: taints, labels), steps of 4,096 pods,
profile TaintToleration + NodeAffinity + NodeResourcesFit + BalancedAllocation.
One step = every pod of the step filtered and scored against the same frozen
snapshot (NormalizeScore, weights, seeded selectHost), then the step's
placements bound (ksg_whatif).  value = pod x node pairs per second over the
timed steps; W warm-up steps run first on the same queue.  Multi-GPU: one
process per GPU (torch.distributed.run), nodes sharded, per-pod normalisers and
argmax keys exchanged over RCCL after each pass.

--variant pts-ipa: the same step shape with PodTopologySpread + InterPodAffinity
on frozen domain tables (SURVEY §8(d) cfg5 "+PTS/IPA"): 1,000,000 nodes of the
cfg4 distribution (20 zones, unique hostnames) with existing pods, profile
Fit + PodTopologySpread + InterPodAffinity + BalancedAllocation; every pod of a
step runs the table chain without assume, then the step is bound in pod order.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
HBM_PEAK_GBS = 8000.0
CUS = 256  # MI355X compute units (MI355X_MICROARCH.md)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--step-pods", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-pods", type=int, default=48, help="pods in the CPU oracle sample (0: skip)")
    ap.add_argument("--cpu-workers", type=int, default=16)
    ap.add_argument("--variant", choices=["cfg5", "pts-ipa"], default="cfg5")
    ap.add_argument("--existing", type=int, default=1_000_000, help="existing pods (pts-ipa variant)")
    return ap.parse_args(argv)


def pmc_step_traffic(kernels):
    """HBM bytes of one step from the newest committed PMC pass holding every one of
    `kernels` (profiles/*cfg5_pmc_traffic.json: FETCH_SIZE x 2 per the gfx950
    correction + WRITE_SIZE, per dispatch), summed; None when none is committed."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*cfg5_pmc_traffic.json")), reverse=True):
        ks = json.load(open(f)).get("kernels", {})
        if all(k in ks for k in kernels):
            return sum(ks[k]["hbm_bytes_per_dispatch"] for k in kernels)
    return None


def pmc_issue(kernel, kernel_ms):
    """Issue utilisation of `kernel` from the newest committed SQ pass holding it
    (profiles/*cfg5_pmc_sq.csv, per-dispatch means): SALU instructions over one
    scalar issue slot per CU per cycle, VALU wave-instructions over one per SIMD
    per 2 cycles (wave64 on SIMD-32), cycles = GRBM_GUI_ACTIVE / 8 XCDs when the
    pass has it, else the kernel time at the 2.4 GHz peak clock."""
    import csv
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*cfg5_pmc_sq.csv")), reverse=True):
        for row in csv.DictReader(open(f)):
            if row["kernel"].split("::")[-1].split("<")[0] != kernel:  # (template arguments dropped)
                continue
            salu = float(row["SQ_INSTS_SALU_per_dispatch"])
            valu = float(row["SQ_INSTS_VALU_per_dispatch"])
            gui = float(row.get("GRBM_GUI_ACTIVE_per_dispatch") or 0.0)
            cyc = gui / 8 if gui else kernel_ms * 1e-3 * 2.4e9
            return {"kernel": kernel, "source": os.path.basename(f), "salu_per_dispatch": salu,
                    "valu_per_dispatch": valu, "cycles": cyc, "cycles_from": "GRBM_GUI_ACTIVE/8" if gui else "2.4 GHz",
                    "salu_util": salu / (CUS * cyc), "valu_util": 2 * valu / (4 * CUS * cyc)}
    return None


def main():
    a = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    out = run(a, torch, rank, world, local, dist)
    if out is not None:
        print(json.dumps(out), flush=True)


def run(a, torch, rank=0, world=1, local=0, dist=None):
    """One what-if benchmark (args as parse()); the result line on rank 0, else None
    (bench.py reports cfg5 through this at N=1)."""
    from ksg import generator as g
    from ksg.distributed import sharded_scheduler
    t0 = time.time()
    n_pods = a.step_pods * (a.warmup + a.steps + 1)  # (+1: one untimed step with kernel sampling)
    if a.variant == "pts-ipa":
        blob = g.generate_native(4, n_nodes=a.nodes, n_pods=n_pods, n_existing=a.existing, n_zones=20)
    else:
        blob = g.generate_native(5, n_nodes=a.nodes, n_pods=n_pods)  # native twin of the generator (tests/test_synth.py)
    prof = json.loads(blob[blob.index(b'"profile"') + 10:].split(b',"nodes"', 1)[0]) if blob.startswith(b'{"profile"') \
        else json.loads(blob)["profile"]
    print(f"[rank {rank}] generated {a.nodes} nodes / {n_pods} pods in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    s = sharded_scheduler(prof, torch, rank, world, local)
    t0 = time.time()
    s.load_cluster(blob)
    print(f"[rank {rank}] loaded in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    P = a.step_pods
    for k in range(a.warmup):
        s.whatif(k * P, P)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    s.sample_kernel(0)  # no events inside the timed steps
    t0 = time.perf_counter()
    for k in range(a.warmup, a.warmup + a.steps):
        s.whatif(k * P, P, wait=False)
        s.wait()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:  # the slowest rank's time (gloo in the CPU test of the multi-rank path)
        t = torch.tensor([elapsed], device="cpu" if dist.get_backend() == "gloo" else "cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = s.results(a.warmup * P, a.steps * P)
    # one more (untimed) step with HIP events on the engine stream around the passes
    s.sample_kernel(1 if a.variant == "cfg5" else 64)  # (pts-ipa: one k_eval in 64 pods)
    s.whatif((a.warmup + a.steps) * P, P)
    avg_ms, nsamp = s.kernel_time()  # cfg5: the average of the step's two passes
    s.sample_kernel(0)
    classes = s.whatif_class_chunks() > 0
    del s
    if rank != 0:
        return None
    pairs = float(a.nodes) * P * a.steps
    shard = a.nodes // world
    # algorithmic bytes per step, SURVEY.md §8(d) basis: cfg5 ~7 B per (pod, node)
    # pair (the node row amortised over a 64-pod tile ~2 B + filter 1 B + total 4 B);
    # the kernel time is one step's two passes (HIP events around each, summed).
    bytes_per_launch = 7.0 * shard * P
    kernel_ms = 2 * avg_ms
    issue = None
    if classes:  # class path: per-class best keys, nothing per pair in memory
        kernel = "k_whatif_cls1 + k_whatif_cls2 (one step)"
        traffic = pmc_step_traffic(["cfg5:k_whatif_cls1", "cfg5:k_whatif_cls2"])
        note = ("issue-bound: pass 1 (k_whatif_cls1) runs at its occupancy limit (4 waves/SIMD, LDS) with "
                "VALU / SALU / SMEM issue and their latencies as the limit (`issue`: utilisation from "
                "profiles/*cfg5_pmc_sq.csv), not HBM: its measured traffic is far below the §8(d) bytes, "
                "so `frac` prices the step against bytes it never moves")
        issue = pmc_issue("k_whatif_cls1", kernel_ms)
    else:  # record path: pass 1's 4-byte per-pair record, written and read back by pass 2
        kernel = "k_whatif_rec1 + k_whatif_rec2 (one step)"
        traffic = pmc_step_traffic(["cfg5:k_whatif_rec1", "cfg5:k_whatif_rec2"])
        note = ("pass 1 (k_whatif_rec1) program decode per (pod, node tile): SALU issue, "
                "profiles/*cfg5_pmc_sq.csv; traffic = both passes' HBM bytes (PMC) incl. the record round trip")
    workload = f"cfg5: {a.nodes} nodes, {P} pods/step, TaintToleration+NodeAffinity+Fit+BA"
    if a.variant == "pts-ipa":  # table chain: k_eval reads 68 B per node (row 56, zone id 4, class count 8)
        bytes_per_launch = 88.0 * shard  # + the per-pair filter code and four raw scores it writes
        kernel_ms = avg_ms
        traffic = None
        kernel = "k_eval (table chain, sampled pods)"
        note = "per-pod table chain over frozen class tables; sequence of dependent memory round trips per pod"
        workload = (f"cfg5+PTS/IPA: {a.nodes} nodes (cfg4 distribution, {a.existing} existing pods, 20 zones), "
                    f"{P} pods/step, Fit+PodTopologySpread+InterPodAffinity+BA on frozen domain tables")
    out = {
        "metric": "what-if filter+score pod x node pairs/sec (1M nodes, 4,096 pods/step)"
                  + (", PTS/IPA" if a.variant == "pts-ipa" else ""),
        "value": pairs / elapsed, "unit": "pairs/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": elapsed * 1e3 / a.steps, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "int64+f64", "data": "synthetic (seeded generator, SURVEY.md §8(d) cfg5)",
        "config": {"workload": workload,
                   "nodes_total": a.nodes, "nodes_per_gpu": shard, "pods_per_step": P,
                   "parallelism": f"node-shard x{world}" if world > 1 else "1 GPU"},
        "scheduled_per_step": sum(1 for r in res if r.status == 0) / a.steps,
        "roofline": {"bound": "issue" if issue else "hbm", "achieved": bytes_per_launch / (kernel_ms * 1e-3) / 1e9 if kernel_ms else 0.0,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": kernel,
                     "kernel_avg_ms": kernel_ms, "kernel_samples": nsamp, "bytes_per_launch": bytes_per_launch,
                     "traffic": traffic, "note": note},
    }
    if issue:
        out["roofline"]["issue"] = issue
    out["roofline"]["frac"] = out["roofline"]["achieved"] / HBM_PEAK_GBS
    if a.cpu_pods and world == 1:  # the oracle's what-if step on a bounded sample of the same cluster
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from _oracle import Oracle
        o = Oracle(blob)
        t = time.perf_counter()
        done = o.whatif(a.cpu_pods, workers=a.cpu_workers)
        dt = time.perf_counter() - t
        out["cpu_baseline"] = {"value": done * a.nodes / dt, "unit": "pairs/s", "cores": a.cpu_workers, "kind": "port",
                               "sample": f"what-if step of the first {a.cpu_pods} pods x {a.nodes} nodes, oracle "
                                         f"plugin-only path, {a.cpu_workers} parallelize.Until workers, {dt:.1f} s"}
    return out


if __name__ == "__main__":
    main()
