"""bench.py's multi-GPU line, on the CPU: two ranks over gloo, the engine stubbed.

The driver's SCALE run launches `bench.py --gpus N` as N processes over RCCL; this
test runs the same `bench.run` at world size 2 with a gloo process group and a
stand-in for the engine context, and checks that every rank runs every leg (the
stand-in's schedule / what-if steps are collectives: a rank that skipped one
would hang the other), that the line carries the sharded cfg3 / cfg4 / cfg5 legs
with their transport and scaling, and that the times are the slowest rank's.
No GPU and no libksg compute call is involved.
"""
import json
import os
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Res:
    def __init__(self, status):
        self.status = status
        self.selected = 0 if status == 0 else -1
        self.feasible = 1
        self.total = 0


class FakeScheduler:
    """Just the calls bench.py / bench_whatif.py make on an engine context."""

    def __init__(self, profile, rank, world, dist):
        self.profile, self.rank, self.world, self.dist = profile, rank, world, dist
        self.n_nodes = 0
        self.queue_len = 0
        self.calls = 0
        self.batch_path = "NodeResourcesFit" in json.dumps(profile) and "PodTopologySpread" not in json.dumps(profile)
        self.L = None

    def load_cluster(self, doc):
        d = json.loads(doc) if isinstance(doc, (bytes, str)) else doc
        self.n_nodes = len(d["nodes"])
        self.queue_len = len(d["queue"])

    def _collective(self):
        # every exchange of a sharded run is collective: a rank that skips a
        # step leaves the other one blocked here
        self.dist.barrier()
        self.calls += 1

    def reset(self):
        pass

    def schedule(self, first=0, count=None, wait=True):
        self._collective()

    def whatif(self, first=0, count=None, wait=True):
        self._collective()

    def wait(self):
        return 0.0

    def sample_kernel(self, every):
        pass

    def kernel_time(self):
        return 0.01 * (1 + self.rank), 4

    def window_runs(self):
        return 0

    def run_counts(self):
        return (0, 0)

    def static_time(self):
        return 0.5, 2, 64

    def whatif_class_chunks(self):
        return 1

    def results(self, first=0, count=None):
        n = self.queue_len - first if count is None else count
        return [_Res(0) for _ in range(n)]


def _fake_ksg(rank, world, dist):
    def doc(c, n_nodes, n_pods, n_existing=0):
        prof = {"plugins": ["NodeResourcesFit", "NodeResourcesBalancedAllocation"] +
                (["PodTopologySpread", "InterPodAffinity"] if c == 4 else []) +
                (["TaintToleration", "NodeAffinity"] if c in (3, 5) else [])}
        return {"profile": prof, "nodes": [{"n": i} for i in range(n_nodes)],
                "pods": [{"p": i} for i in range(n_existing)], "queue": [{"q": i} for i in range(n_pods)]}

    gen = types.ModuleType("ksg.generator")
    gen.generate = lambda c, n_nodes=100, n_pods=100: doc(c, n_nodes, n_pods)
    gen.generate_native = lambda c, n_nodes=100, n_pods=100, n_existing=0, **kw: json.dumps(
        doc(c, n_nodes, n_pods, n_existing), separators=(",", ":")).encode()
    dmod = types.ModuleType("ksg.distributed")
    dmod.sharded_scheduler = lambda profile, torch, r, w, local: FakeScheduler(profile, r, w, dist)
    pkg = types.ModuleType("ksg")
    pkg.generator = gen
    pkg.distributed = dmod
    pkg.__path__ = []
    return {"ksg": pkg, "ksg.generator": gen, "ksg.distributed": dmod}


def _rank_main(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.modules.update(_fake_ksg(rank, world, dist))
    sys.path.insert(0, ROOT)
    import bench
    torch.cuda.synchronize = lambda *a, **k: None  # (no GPU: the stand-in runs nothing)
    sys.argv = ["bench.py", "--gpus", str(world), "--steps", "2", "--warmup", "1", "--nodes", "40", "--pods", "64",
                "--extra-sizes", "3:90:64,4:120:48:200,5:400:32"]
    a = bench.parse()
    out = bench.run(a, torch, rank, world, 0, dist)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(out, f)
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_bench_world2_runs_sharded_legs(tmp_path):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    out_path = str(tmp_path / "line.json")
    mp.spawn(_rank_main, args=(2, port, out_path), nprocs=2, join=True)
    d = json.load(open(out_path))
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["transport"] == "rccl"
    assert d["config"]["nodes_total"] == 80 and d["config"]["nodes_per_gpu"] == 40
    assert "cpu_baseline" not in d and "dropin" not in d
    for c, nodes in ((3, 90), (4, 120), (5, 400)):
        leg = d[f"cfg{c}"]
        assert leg is not None, c
        assert leg["n_gpus"] == 2 and leg["scaling"] == "strong", c
        assert leg["config"]["transport"] == "rccl", c
        assert "cpu_baseline" not in leg, c
    assert d["cfg3"]["config"]["nodes_per_gpu"] == 45 and d["cfg4"]["config"]["nodes_per_gpu"] == 60
    assert d["cfg5"]["config"]["nodes_per_gpu"] == 200
    # value = whole-cluster pairs / the slowest rank's time
    assert d["cfg4"]["value"] == pytest.approx(120 * 48 * 2 / (d["cfg4"]["ms_per_step"] * 2 / 1e3))
