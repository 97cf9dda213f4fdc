"""Sequential-queue throughput for the other BASELINE configs (cfg1, cfg3, cfg4):
pairs/s of the scheduling cycle (per-pod kernel chain; Fit/BA-only profiles take
the window path) on one GPU, beside the oracle on a bounded sample.

usage: python tools/bench_config.py CONFIG [--nodes N] [--pods P] [--existing E] [--cpu-pods C]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", type=int)
    ap.add_argument("--nodes", type=int, default=0)
    ap.add_argument("--pods", type=int, default=2000)
    ap.add_argument("--existing", type=int, default=0)
    ap.add_argument("--cpu-pods", type=int, default=100)
    ap.add_argument("--cpu-workers", type=int, default=16)
    a = ap.parse_args()
    import torch  # before libksg.so initialises HIP (ksg_synth_cluster loads it)
    assert torch.cuda.is_available()
    from ksg import Scheduler, generator as g
    kw = {"n_pods": a.pods}
    if a.nodes:
        kw["n_nodes"] = a.nodes
    if a.existing:
        kw["n_existing"] = a.existing
    t0 = time.time()
    if a.config in (2, 3, 4, 5):  # native twin of the generator (tests/test_synth.py)
        blob = g.generate_native(a.config, **kw)
        doc = json.loads(blob)
    else:
        doc = g.generate(a.config, **kw)
        blob = json.dumps(doc).encode()
    print(f"generated in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    s = Scheduler(doc["profile"])
    s.load_cluster(blob)
    n, q = s.n_nodes, s.queue_len
    warm = min(64, q // 4)
    s.schedule(0, warm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.schedule(warm, q - warm)
    dt = time.perf_counter() - t0
    res = s.results()
    # kernel sampling (HIP events on the engine stream) in a second, untimed pass
    s.reset()
    s.sample_kernel(16)
    s.schedule(0, q)
    kms, ks = s.kernel_time()
    s.sample_kernel(0)
    assert [(r.selected, r.status) for r in s.results()] == [(r.selected, r.status) for r in res]
    out = {"config": a.config, "nodes": n, "pods_timed": q - warm, "existing_pods": len(doc["pods"]),
           "profile": doc["profile"]["plugins"], "path": "window" if s.batch_path else "per-pod chain",
           "pairs_per_s": n * (q - warm) / dt, "pods_per_s": (q - warm) / dt, "us_per_pod": dt * 1e6 / (q - warm),
           "scheduled": sum(1 for r in res if r.status == 0), "sampled_kernel_us": kms * 1e3, "samples": ks,
           "run_counts": list(s.run_counts())}  # (persistent-segment pods, segments) over both passes
    if a.cpu_pods:
        from _oracle import Oracle
        o = Oracle(blob)
        o.schedule(n=warm, workers=a.cpu_workers, record=0)
        t0 = time.perf_counter()
        done = o.schedule(n=a.cpu_pods, workers=a.cpu_workers, record=0)
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"pairs_per_s": done * n / cdt, "cores": a.cpu_workers, "kind": "port",
                               "sample": f"pods {warm}..{warm + done} of the same queue, {cdt:.1f} s"}
        out["gpu_over_cpu"] = out["pairs_per_s"] / out["cpu_baseline"]["pairs_per_s"]
        # parity on the CPU sample: same selections
        mism = sum(1 for i in range(warm + done) if (res[i].selected, res[i].feasible, res[i].status) != o.result(i))
        out["parity_mismatches_in_sample"] = mism
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
