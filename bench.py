#!/usr/bin/env python3
"""Headline benchmark: filter+score pod x node pairs/sec (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 5,000 nodes x 10,000
pods, profile NodeResourcesFit + NodeResourcesBalancedAllocation, synthetic
cluster from the seeded generator.  One *step* = one pass of the hot path over
the whole queue: every pod is filtered and scored against every node, the best
node is selected and the pod is assumed on it on the device (so pod k sees the
placements of pods < k), starting from the same snapshot each step.

value = pairs evaluated by all ranks / max-over-ranks wall time of the K timed
steps.  Multi-GPU: one process per GPU (torch.distributed.run); each rank owns
its own shard of nodes of a weak-scaled cluster (5,000 nodes per GPU) —
see DESIGN.md "Multi-GPU".
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=10000)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on a bounded sample (rank 0, N=1)")
    ap.add_argument("--cpu-pods", type=int, default=0, help="pods in the CPU sample (0 = auto, ~15 s)")
    ap.add_argument("--cpu-workers", type=int, default=16, help="parallelize.Until workers (upstream default 16)")
    return ap.parse_args()


def algorithmic_bytes_per_node_fit_ba(n_res=3):
    """Per (pod, node) pair, Fit+BA profile (DESIGN.md roofline table):
    reads  alloc cpu/mem 16 + allowed pods 4 + requested cpu/mem 16 + nonzero cpu/mem 16 + pod count 4 = 56 B
    writes filter code 4 + raw Fit 4 + raw BA 4 + total 4 = 16 B."""
    return 56 + 16


WINDOW = 32          # pods per k_window launch (KSG_BATCH)
TILE = 1024          # nodes per eval block (KSG_TILE)
REC_BYTES = 128 + WINDOW * 64 * 96  # candidate record of one window (KSG_XHDR + 32 x 64 CandRow)


def window_bytes_per_launch(shard):
    """k_window, one launch = eval of one window (WINDOW pods x shard nodes) + the
    replay of the previous one: per-pair row reads and outputs, the tile top-64
    lists (written and read back), the candidate record (written by the eval
    part, read by the next launch's replay)."""
    tiles = (shard + TILE - 1) // TILE
    return WINDOW * shard * algorithmic_bytes_per_node_fit_ba() + 2 * tiles * WINDOW * 64 * 8 + 2 * REC_BYTES


def pmc_traffic(kernel):
    """HBM bytes per dispatch of `kernel` from the committed PMC pass
    (profiles/*pmc_traffic.json, tools/pmc_pass.sh): FETCH_SIZE x 2 (gfx950
    tallies 128-B requests at 64 B, MI355X_MICROARCH.md HBM section) + WRITE_SIZE,
    both in KB per dispatch.  None when no pass is committed."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    k = d.get("kernels", {}).get(kernel)
    return None if k is None else k["hbm_bytes_per_dispatch"]


def cpu_baseline(doc, n_pods, workers):
    """Time the oracle (the CPU restatement, test infrastructure) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _oracle import Oracle
    res, secs = {}, 0.0
    for w in sorted({1, workers}):
        o = Oracle(doc)
        t = time.perf_counter()
        done = o.schedule(n=n_pods, workers=w, record=0)
        dt = time.perf_counter() - t
        secs += dt
        res[w] = done * len(doc["nodes"]) / dt
    best_w = max(res, key=res.get)
    return best_w, res, secs


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
    from ksg import Scheduler, generator as g

    # weak scaling: a cluster of nodes x world nodes, node-sharded (each rank owns
    # `nodes`); every pod is scheduled over the whole cluster (RCCL exchange per batch)
    doc = g.generate(2, n_nodes=a.nodes * world, n_pods=a.pods)
    stream = torch.cuda.current_stream().cuda_stream if world > 1 else None
    s = Scheduler(doc["profile"], device=local, stream=stream, shard_rank=rank, shard_count=world)
    if world > 1:
        from ksg.distributed import rccl_unique_id_broadcast
        s.set_exchange_rccl(rccl_unique_id_broadcast(s.L, rank))
    s.load_cluster(doc)
    n_nodes, n_pods = s.n_nodes, s.queue_len  # n_nodes: whole cluster
    sample_every = 64

    def step(timed):
        s.reset()
        s.sample_kernel(sample_every if timed else 0)
        s.schedule(0, n_pods, wait=False)
        s.wait()

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    ksum, kcount = 0.0, 0
    for _ in range(a.steps):
        step(True)
        ms, n = s.kernel_time()
        ksum += ms * n
        kcount += n
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = s.results()
    scheduled = sum(1 for r in res if r.status == 0)
    pairs = float(n_nodes) * n_pods * a.steps  # n_nodes already spans all ranks
    value = pairs / elapsed
    ms_per_step = elapsed * 1e3 / a.steps
    kernel_ms = ksum / max(kcount, 1)
    shard = n_nodes // world
    if s.batch_path:
        kname = "k_window"
        bytes_per_launch = window_bytes_per_launch(shard)
    else:
        kname = "k_filter_score"
        bytes_per_launch = shard * algorithmic_bytes_per_node_fit_ba()
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    if rank != 0:
        return
    out = {
        "metric": "filter+score pod x node pairs/sec (5k nodes, Fit+BalancedAllocation)",
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64+f64",
        "data": "synthetic (seeded generator, SURVEY.md §8(d) cfg2)",
        "config": {"workload": "cfg2: 5,000 nodes x 10,000 pods, NodeResourcesFit+NodeResourcesBalancedAllocation",
                   "nodes_per_gpu": shard, "nodes_total": n_nodes, "pods": n_pods, "parallelism": f"node-shard x{world} (RCCL all-gather per 32-pod batch)" if world > 1 else "1 GPU"},
        "scheduled_pods_per_s": scheduled * a.steps / elapsed,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(kname),
                     "kernel": kname, "kernel_avg_us": kernel_ms * 1e3, "kernel_samples": kcount,
                     "bytes_per_launch": bytes_per_launch},
    }
    if a.cpu_baseline and world == 1:
        n_cpu = a.cpu_pods or n_pods
        w, rates, secs = cpu_baseline(doc, n_cpu, a.cpu_workers)
        out["cpu_baseline"] = {"value": rates[w], "unit": "pairs/s", "cores": w, "kind": "port",
                               "sample": f"first {n_cpu} of {n_pods} pods x {n_nodes} nodes (same cfg2 cluster), "
                                         f"oracle plugin-only path (parallelize.Until chunking), "
                                         f"{secs:.1f} s of CPU runs; rates by workers: "
                                         + ", ".join(f"{k}: {v:.3g}" for k, v in sorted(rates.items()))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
