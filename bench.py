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

The same JSON line also carries the other BASELINE configs as extra keys
(--extra): cfg3 and cfg4 queues at full size, and cfg5 — one what-if step of
4,096 pods x 1,000,000 nodes per timed step (bench_whatif.py) — each with its own
roofline (and, at N=1, its CPU baseline).  At N>1 they run node-sharded over the
N ranks at their BASELINE sizes (strong scaling: the cluster is fixed, every rank
holds 1/N of its nodes; RCCL all-gathers on the engine stream, "transport"),
which is what BASELINE.json quotes for cfg3 ("1 and 8 MI355X"), cfg4 ("8x
sharded") and cfg5 ("node-sharded over 8x with RCCL argmax").
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
    ap.add_argument("--cpu-seconds", type=float, default=4.0, help="CPU time per oracle variant")
    ap.add_argument("--extra", default="3,4,5", help="other BASELINE configs reported beside cfg2 (node-sharded "
                    "at N>1; 5 = the cfg5 what-if step of bench_whatif.py)")
    ap.add_argument("--extra-sizes", default="", help="tests only: c:nodes:pods[:existing],... overriding the "
                    "BASELINE sizes of the extra configs (e.g. 3:300:64,4:400:64:800,5:2000:64)")
    ap.add_argument("--extra-steps", type=int, default=2)
    ap.add_argument("--whatif-steps", type=int, default=16, help="cfg5 timed what-if steps (SURVEY.md §8(d): 16, "
                    "binds between them)")
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
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json")), reverse=True):
        k = json.load(open(f)).get("kernels", {}).get(kernel)  # newest pass that holds the kernel
        if k is not None:  # (persistent segments: per pod cycle, like the roofline's "launch")
            return k.get("hbm_bytes_per_pod", k["hbm_bytes_per_dispatch"])
    return None


def cpu_info():
    """Host CPU facts for cpu_baseline: nproc, the CPUs this process may run on,
    the cgroup CPU quota (the box's share), the CPU model."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    info["cgroup_cpus"] = quota
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    info["model"] = model
    info["all_core_workers"] = min(x for x in (info["affinity"], quota) if x)
    return info


def _timed_oracle(src, n_nodes, workers, record, seconds):
    """Oracle pairs/s over the first pods of the queue, run until ~`seconds` of wall time."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _oracle import Oracle
    o = Oracle(src)
    pods, dt, chunk = 0, 0.0, 2
    while dt < seconds:
        t = time.perf_counter()
        done = o.schedule(n=chunk, workers=workers, record=record)
        dt += time.perf_counter() - t
        pods += done
        if done < chunk:  # queue exhausted
            break
        chunk = max(1, min(4096, int(pods / max(dt, 1e-6) * 0.5)))
    return pods * n_nodes / max(dt, 1e-9), pods, dt


def cpu_baseline(src, n_nodes, workers, seconds, label):
    """The oracle (the CPU restatement, test infrastructure; never the product) timed on
    this host: plugin-only at 1 worker, at upstream's 16 parallelize.Until workers and at
    all cores, and the "debuggable" result-store emulation (record=1) at 16 workers
    (BASELINE.md CPU-baseline plan).  value = plugin-only at all cores."""
    ci = cpu_info()
    allw = ci["all_core_workers"]
    runs = {}
    for key, w, rec in (("plugins_1_worker", 1, 0), (f"plugins_{workers}_workers", workers, 0),
                        (f"plugins_all_cores_{allw}_workers", allw, 0), (f"debuggable_{workers}_workers", workers, 1)):
        if key in runs:
            continue
        rate, pods, dt = _timed_oracle(src, n_nodes, w, rec, seconds)
        runs[key] = {"pairs_per_s": rate, "pods": pods, "s": round(dt, 2)}
    head = runs[f"plugins_all_cores_{allw}_workers"]
    return {"value": head["pairs_per_s"], "unit": "pairs/s", "cores": allw, "kind": "port",
            "sample": f"{label}: the first pods of the same queue, each variant run for ~{seconds:.0f} s "
                      f"(oracle = CPU restatement of the upstream plugins, parallelize.Until chunking); "
                      f"value = plugin-only at all cores",
            "variants": runs, "cpu": ci}


def time_queue(s, torch, steps, warmup, dist=None):
    """K timed steps of the whole queue from the same snapshot (reset inside the step),
    bracketed by barrier + synchronize; no kernel sampling inside the timed region."""
    n_pods = s.queue_len

    def step():
        s.reset()
        s.schedule(0, n_pods, wait=False)
        s.wait()

    s.sample_kernel(0)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return max_over_ranks(torch, dist, elapsed)


def max_over_ranks(torch, dist, x):
    """The slowest rank's value (the contract's max-over-ranks timing); the
    tensor lives where the process group's backend reduces (RCCL: the GPU)."""
    if not dist:
        return x
    dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sample_dominant(s, every):
    """One more step, after the timed region, with HIP events on the engine stream
    around every `every`-th launch of the dominant kernel: average duration (ms), samples."""
    s.reset()
    s.sample_kernel(every)
    s.schedule(0, s.queue_len, wait=False)
    s.wait()
    ms, n = s.kernel_time()
    s.sample_kernel(0)
    return ms, n


def dropin_latency(s, doc, n=100):
    """The drop-in path a Go plugin takes per pod, after the
    timed region: ksg_cycle (PreFilter..NormalizeScore on the device, commit=0),
    ksg_cycle_view_acquire (the per-node results the framework's 16 workers then
    index without calls), ksg_reserve on the engine's choice, view release.
    Wall time per call, averaged over n pods (copies of the queue's first pods)."""
    pods = doc["queue"][:n]
    t_cycle = t_view = t_res = 0.0
    done = 0
    for i, p in enumerate(pods):
        p = json.loads(json.dumps(p))
        p["metadata"]["name"] = f"dropin-{i:05d}"
        t0 = time.perf_counter()
        q, r = s.cycle(p, commit=False)
        t1 = time.perf_counter()
        v = s.cycle_view(q)
        t2 = time.perf_counter()
        if r.selected >= 0:
            s.reserve(q, r.selected)
        t3 = time.perf_counter()
        v.release()
        t_cycle += t1 - t0
        t_view += t2 - t1
        t_res += t3 - t2
        done += 1
    k = 1e6 / max(done, 1)
    return {"pods": done, "cycle_us": t_cycle * k, "view_us": t_view * k, "reserve_us": t_res * k,
            "total_us": (t_cycle + t_view + t_res) * k,
            "note": "host wall per drop-in cycle (ksg_cycle commit=0 + ksg_cycle_view + ksg_reserve), after the "
                    "queue's timed steps on the same context"}


# cfg3 / cfg4 (BASELINE.json configs[2], configs[3]) at their full single-GPU size,
# reported beside the cfg2 headline.  Algorithmic bytes: SURVEY.md §8(d), DESIGN.md.
CFG3_PAIR_BYTES = 141      # 120 read + 21 written per (pod, node) pair
# cfg3 runs two kernels over every pair (DESIGN.md "TaintToleration / NodeAffinity"):
CFG3_STATIC_PAIR_BYTES = 64 + 8   # k_static: taint masks 16 + label bitsets 40 + numeric label 8 read, record 8 written
CFG3_WINDOW_PAIR_BYTES = 56 + 8 + 21  # k_window: node row 56 + static record 8 read, filter 1 + 4 raw scores + total written
CFG4_EVAL_NODE_BYTES = 68 + 20  # k_eval: reads node row 56 + zone id 4 + selector-class count 8, writes the
                                # per-pair filter code 4 + the four raw scores 16 (k_final re-reads them)
CFG4_RUN_NODE_BYTES = 68        # SURVEY §8(d) cfg4 per node and pod (row 56, zone id 4, class count 8);
                                # k_chain_run keeps the row and zone id on chip and writes no per-pair outputs


def extra_config(c, torch, steps, warmup, cpu_seconds, cpu_workers, rank=0, world=1, local=0, dist=None, size=None):
    """cfg3 / cfg4 at their BASELINE size, on one GPU or node-sharded over `world`
    ranks (strong scaling); the line on rank 0, else None."""
    from ksg import generator as g
    t0 = time.perf_counter()
    kw = {}
    if size:
        kw = dict(n_nodes=size[0], n_pods=size[1], **({"n_existing": size[2]} if len(size) > 2 else {}))
    blob = g.generate_native(c, **kw)  # native twin of the seeded generator (tests/test_synth.py)
    doc = json.loads(blob)
    gen_s = time.perf_counter() - t0
    from ksg.distributed import sharded_scheduler
    s = sharded_scheduler(doc["profile"], torch, rank, world, local)
    s.load_cluster(blob)
    n_nodes, n_pods = s.n_nodes, s.queue_len  # n_nodes: the whole cluster
    shard = n_nodes // world
    elapsed = time_queue(s, torch, steps, warmup, dist)
    run0 = s.run_counts()
    wr0 = s.window_runs()
    kms, kn = sample_dominant(s, 16)
    run1 = s.run_counts()
    win_persistent = s.batch_path and s.window_runs() > wr0  # one k_window_run launch for the whole queue
    nwin = (n_pods + WINDOW - 1) // WINDOW
    res = s.results()
    per = None
    extra_kernels = None
    if s.batch_path:
        # k_window's own bytes; k_static (the Taint / NodeAffinity records it reads)
        # gets its own line, timed on the same sampled run
        kname = "k_window_run" if win_persistent else "k_window"
        if win_persistent:
            kms /= nwin  # per window inside the persistent launch
        tiles = (shard + TILE - 1) // TILE
        bpl = WINDOW * shard * CFG3_WINDOW_PAIR_BYTES + 2 * tiles * WINDOW * 64 * 8 + 2 * REC_BYTES
        st_ms, st_n, st_pods = s.static_time()
        beside = win_persistent and getattr(s, "static_overlaps", lambda: 0)() > 0
        if st_n:  # (sharded: k_static covers every node of the cluster on every rank)
            sb = st_pods * n_nodes * CFG3_STATIC_PAIR_BYTES
            win_ms_total = kms * nwin
            # beside the loop (KSG_STATIC_OVERLAP): k_static_dec runs on the CUs the
            # persistent launch leaves idle, concurrently: the step is the loop's time
            step_ms = max(st_ms, win_ms_total) if beside else st_ms + win_ms_total
            extra_kernels = {
                "k_static": {"launches": st_n, "total_ms": st_ms, "bytes": sb,
                             "achieved": sb / (st_ms * 1e-3) / 1e9, "frac": sb / (st_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "bytes_per_pair": CFG3_STATIC_PAIR_BYTES,
                             "kernel": "k_static_dec_run" if beside else "k_static_dec",
                             "traffic": pmc_traffic(f"cfg{c}:" + ("k_static_dec_run" if beside else "k_static_dec")),
                             "beside_loop": beside},
                "step": {"note": "both kernels over the whole queue: pairs x (k_static + k_window bytes per pair) / "
                                 "the step's kernel time (k_static + k_window, or the longer of the two when k_static "
                                 "runs beside the persistent loop); the k_window time is its sampled average x windows",
                         "bytes_per_pair": CFG3_STATIC_PAIR_BYTES + CFG3_WINDOW_PAIR_BYTES,
                         "frac": n_pods * (n_nodes * CFG3_STATIC_PAIR_BYTES + shard * CFG3_WINDOW_PAIR_BYTES)
                         / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}}
    elif run1[1] > run0[1]:
        # persistent segments: one k_chain_run launch per segment of pods; the
        # roofline's "launch" is one pod's cycle inside it (launch time / its pods)
        kname = "k_chain_run"
        per = (run1[0] - run0[0]) / (run1[1] - run0[1])
        kms = kms / per
        bpl = shard * CFG4_RUN_NODE_BYTES
    else:  # (sharded: the two-launch chain on the rank's shard, two all-gathers per pod)
        kname = "k_eval"
        bpl = shard * CFG4_EVAL_NODE_BYTES
    achieved = bpl / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    traffic = pmc_traffic(f"cfg{c}:{kname}") if world == 1 else None
    if win_persistent and traffic is not None:
        traffic /= nwin  # (the PMC pass counts the whole-queue launch: per window, like bytes_per_launch)
    if rank != 0:
        del s
        return None
    out = {"metric": "filter+score pod x node pairs/sec", "value": n_nodes * n_pods * steps / elapsed,
           "unit": "pairs/s", "n_gpus": world, "steps": steps, "warmup": warmup, "ms_per_step": elapsed * 1e3 / steps,
           "us_per_pod": elapsed * 1e6 / (steps * n_pods),
           "scheduled_pods_per_s": sum(1 for r in res if r.status == 0) * steps / elapsed,
           "scaling": "strong",
           "config": {"workload": f"cfg{c}", "nodes": n_nodes, "nodes_per_gpu": shard, "existing_pods": len(doc["pods"]),
                      "pods": n_pods, "profile": doc["profile"]["plugins"],
                      "path": "window" if s.batch_path else "table chain",
                      "parallelism": f"node-shard x{world}" if world > 1 else "1 GPU",
                      **({"transport": "rccl"} if world > 1 else {})},
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                        "kernel": kname, "kernel_avg_us": kms * 1e3, "kernel_samples": kn, "bytes_per_launch": bpl,
                        **({"windows_per_launch": nwin, "note": "k_window_run: the whole queue in one persistent "
                            "launch; kernel_avg_us and bytes_per_launch per 32-pod window inside it"} if win_persistent else {}),
                        **({"pods_per_launch": per, "note": "k_chain_run: kernel_avg_us and bytes_per_launch per pod "
                            "cycle inside the persistent launch (launch time / its pods)"} if per else {}),
                        **({"bytes_per_pair": CFG3_WINDOW_PAIR_BYTES, "other_kernels": extra_kernels} if extra_kernels else {})},
           "generate_s": round(gen_s, 1)}
    if c == 4 and world == 1:
        out["dropin"] = dropin_latency(s, doc)
    del s
    if cpu_seconds > 0 and world == 1:
        out["cpu_baseline"] = cpu_baseline(blob, n_nodes, cpu_workers, cpu_seconds, f"cfg{c}")
    return out


def parse_sizes(spec):
    """--extra-sizes "c:nodes:pods[:existing],..." -> {c: (nodes, pods[, existing])}."""
    out = {}
    for part in (x for x in spec.split(",") if x):
        f = [int(v) for v in part.split(":")]
        out[f[0]] = tuple(f[1:])
    return out


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
    """The whole bench line (rank 0; None on the other ranks)."""
    from ksg import generator as g
    from ksg.distributed import sharded_scheduler

    # weak scaling: a cluster of nodes x world nodes, node-sharded (each rank owns
    # `nodes`); every pod is scheduled over the whole cluster (RCCL exchange per batch)
    doc = g.generate(2, n_nodes=a.nodes * world, n_pods=a.pods)
    s = sharded_scheduler(doc["profile"], torch, rank, world, local)
    s.load_cluster(doc)
    n_nodes, n_pods = s.n_nodes, s.queue_len  # n_nodes: whole cluster
    elapsed = time_queue(s, torch, a.steps, a.warmup, dist)
    wr0 = s.window_runs()
    kernel_ms, kcount = sample_dominant(s, 64)
    persistent = s.window_runs() > wr0  # one k_window_run launch for the whole queue
    nwin = (n_pods + WINDOW - 1) // WINDOW
    if persistent:
        kernel_ms /= nwin  # per window inside the persistent launch
    res = s.results()
    dropin = dropin_latency(s, doc) if world == 1 else None
    scheduled = sum(1 for r in res if r.status == 0)
    pairs = float(n_nodes) * n_pods * a.steps  # n_nodes already spans all ranks
    value = pairs / elapsed
    ms_per_step = elapsed * 1e3 / a.steps
    shard = n_nodes // world
    if s.batch_path:
        kname = "k_window_run" if persistent else "k_window"
        bytes_per_launch = window_bytes_per_launch(shard)
    else:
        kname = "k_filter_score"
        bytes_per_launch = shard * algorithmic_bytes_per_node_fit_ba()
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    traffic = pmc_traffic(kname) if world == 1 else None
    if persistent and traffic is not None:
        traffic /= nwin  # (the PMC pass counts the whole-queue launch: per window, like bytes_per_launch)
    del s
    out = None
    if rank == 0:
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
                       "nodes_per_gpu": shard, "nodes_total": n_nodes, "pods": n_pods,
                       "parallelism": f"node-shard x{world} (RCCL all-gather per 32-pod batch)" if world > 1 else "1 GPU",
                       **({"transport": "rccl"} if world > 1 else {})},
            "scheduled_pods_per_s": scheduled * a.steps / elapsed,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": kname, "kernel_avg_us": kernel_ms * 1e3, "kernel_samples": kcount,
                         "bytes_per_launch": bytes_per_launch,
                         **({"note": "k_window_run: the whole queue in one persistent launch; kernel_avg_us and "
                                     "bytes_per_launch per 32-pod window inside it (launch time / windows)",
                             "windows_per_launch": nwin} if persistent else {})},
        }
        if dropin:
            out["dropin"] = dropin
        if a.cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(json.dumps(doc).encode(), n_nodes, a.cpu_workers, a.cpu_seconds, "cfg2")
    # the other BASELINE configs: one GPU, or node-sharded over every rank (each
    # rank runs every leg: the exchanges are collective)
    sizes = parse_sizes(a.extra_sizes)
    for c in (int(x) for x in a.extra.split(",") if x):
        if c == 5:  # what-if steps: 1M nodes x 4,096 pods per step (bench_whatif.py)
            import bench_whatif
            wargs = ["--steps", str(max(a.whatif_steps, 1)), "--warmup", "1",
                     "--cpu-pods", "16" if (a.cpu_baseline and world == 1) else "0", "--cpu-workers", str(a.cpu_workers)]
            if c in sizes:
                wargs += ["--nodes", str(sizes[c][0]), "--step-pods", str(sizes[c][1])]
            r = bench_whatif.run(bench_whatif.parse(wargs), torch, rank, world, local, dist)
            if r is not None and world > 1:
                r["config"]["transport"] = "rccl"
        else:
            r = extra_config(c, torch, a.extra_steps, 1, a.cpu_seconds if (a.cpu_baseline and world == 1) else 0,
                             a.cpu_workers, rank, world, local, dist, sizes.get(c))
        if out is not None:
            out[f"cfg{c}"] = r
    return out


if __name__ == "__main__":
    main()
