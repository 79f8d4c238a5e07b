"""Multi-process helpers: run `world` ranks over torch.distributed gloo on
127.0.0.1 (spawned processes, so no rank inherits a GPU context)."""
from __future__ import annotations

import multiprocessing as mp
import os
import socket
import traceback

import numpy as np


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def gloo_allreduce(arr: np.ndarray, op: str) -> None:
    """In-place all-reduce of a numpy array over the default gloo group; the
    callback `sqlm_ctx_set_host_comm` drives. uint8 is widened (gloo has no
    uint8 max on every build)."""
    import torch
    import torch.distributed as dist
    rop = dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM
    if arr.dtype == np.uint8:
        t = torch.from_numpy(arr.astype(np.int32))
        dist.all_reduce(t, op=rop)
        arr[:] = t.numpy().astype(np.uint8)
    else:
        t = torch.from_numpy(arr)  # shares memory with arr
        dist.all_reduce(t, op=rop)


def gloo_p2p(arr: np.ndarray, peer: int, op: str) -> None:
    """Point-to-point half of the host transport (sqlm_ctx_set_host_p2p):
    send to / receive from `peer`, or broadcast in place from root `peer`."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(arr.view(np.uint8))  # byte view: every dtype, shares memory with arr
    if op == "send":
        dist.send(t, dst=peer)
    elif op == "recv":
        dist.recv(t, src=peer)
    else:
        dist.broadcast(t, src=peer)


def _entry(fn, rank, world, port, args, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            q.put((rank, fn(rank, world, *args), None))
        finally:
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        q.put((rank, None, traceback.format_exc()))


def run_ranks(fn, world: int, *args, timeout: float = 600.0) -> list:
    """Run fn(rank, world, *args) on `world` spawned ranks; return results by rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out, errs = [None] * world, []
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=timeout)
            if err:
                errs.append(f"rank {rank}:\n{err}")
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    if errs:
        raise RuntimeError("\n".join(errs))
    return out
