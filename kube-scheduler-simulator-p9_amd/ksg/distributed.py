"""Node-shard exchange plumbing for multi-GPU runs (one process per GPU).

Production: RCCL all-gather inside libksg on the engine stream (mode 1); the
128-byte unique id is created on rank 0 and broadcast with torch.distributed.
Tests: a host callback (mode 2) that all-gathers host buffers over gloo, which
lets several ranks share one GPU.
"""
from __future__ import annotations

import ctypes

EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)


def shard_bounds(n_nodes: int, rank: int, world: int):
    """Nodes [lo, hi) owned by rank (same arithmetic as the C++ encoder)."""
    return n_nodes * rank // world, n_nodes * (rank + 1) // world


def host_allgather(send: bytes, world: int) -> list:
    """All-gather one byte string per rank over the default process group (gloo)."""
    import torch
    import torch.distributed as dist
    t = torch.frombuffer(bytearray(send), dtype=torch.uint8)
    out = [torch.empty(len(send), dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(out, t)
    return [bytes(o.numpy().tobytes()) for o in out]


def make_host_exchange(world: int):
    """ctypes callback for ksg_set_exchange(mode=2). Keep a reference while in use."""
    def cb(user, send, recv, nbytes):
        try:
            parts = host_allgather(ctypes.string_at(send, nbytes), world)
            for r, p in enumerate(parts):
                ctypes.memmove(recv + r * nbytes, p, nbytes)
            return 0
        except Exception:  # never let a Python exception cross the C ABI
            return -1
    return EXCHANGE_FN(cb)


def rccl_unique_id_broadcast(lib, rank: int) -> bytes:
    """Rank 0 creates the RCCL unique id; every rank receives it."""
    import torch.distributed as dist
    obj = [None]
    if rank == 0:
        buf = (ctypes.c_uint8 * 128)()
        rc = lib.ksg_nccl_unique_id(buf)
        if rc != 0:
            raise RuntimeError(f"ksg_nccl_unique_id failed ({rc})")
        obj = [bytes(buf)]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def sharded_scheduler(profile, torch, rank: int, world: int, local: int):
    """An engine context for this rank's node shard (bench.py, bench_whatif.py);
    at world > 1 on torch's current stream with an RCCL exchange (mode 1:
    ncclAllGather on the engine stream, the unique id broadcast from rank 0)."""
    from .engine import Scheduler
    stream = torch.cuda.current_stream().cuda_stream if world > 1 else None
    s = Scheduler(profile, device=local, stream=stream, shard_rank=rank, shard_count=world)
    if world > 1:
        s.set_exchange_rccl(rccl_unique_id_broadcast(s.L, rank))
    return s
