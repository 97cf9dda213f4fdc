"""Probe: the RCCL exchange (ksg_set_exchange mode 1) with 2 ranks sharing one GPU.

The multi-GPU bench uses mode 1 (RCCL all-gather on the engine stream); the
tests use the gloo host callback (mode 2) because they share one GPU.  This
probe tries mode 1 with both ranks on device 0 (torch process group on gloo,
the RCCL unique id broadcast over it) on a small cfg2 and cfg4 cluster and
compares every result with the oracle.  RCCL may refuse two ranks on one
device; the probe then prints the error.

    python tools/rccl_shared_gpu.py
"""
import json
import os
import sys
import time

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator-p9_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def worker(rank, world, port, doc_json, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ksg import Scheduler
    from ksg.distributed import rccl_unique_id_broadcast
    doc = json.loads(doc_json)
    try:
        s = Scheduler(doc["profile"], device=0, shard_rank=rank, shard_count=world)
        s.set_exchange_rccl(rccl_unique_id_broadcast(s.L, rank))
        print(f"rank {rank}: RCCL exchange set", flush=True)
        s.load_cluster(doc)
        t = time.time()
        s.schedule()
        out[rank] = ("ok", [(r.selected, r.feasible, r.status) for r in s.results()], time.time() - t)
    except Exception as e:  # report, do not hang the peer forever
        out[rank] = ("error", repr(e), 0.0)
    print(f"rank {rank}: {out[rank][0]}", flush=True)
    dist.destroy_process_group()


def main():
    import socket
    from _oracle import Oracle
    from ksg import generator as g
    for name, doc in (("cfg2", g.generate(2, n_nodes=600, n_pods=400)),
                      ("cfg4", g.generate(4, n_nodes=300, n_existing=900, n_pods=100, n_zones=6))):
        o = Oracle(doc)
        o.schedule(record=0)
        want = [o.result(q) for q in range(o.n_queue)]
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        with mp.Manager() as m:
            out = m.dict()
            mp.spawn(worker, args=(2, port, json.dumps(doc), out), nprocs=2, join=True)
            for r in range(2):
                st, res, dt = out[r]
                if st != "ok":
                    print(json.dumps({"case": name, "rank": r, "error": res}), flush=True)
                    continue
                bad = sum(1 for q in range(len(want)) if res[q] != want[q])
                print(json.dumps({"case": name, "rank": r, "pods": len(want), "differ": bad, "s": round(dt, 3)}), flush=True)


if __name__ == "__main__":
    main()
