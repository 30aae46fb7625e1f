"""Local multi-process launcher (one process per GPU, or per CPU rank with gloo).

Production runs use `python -m torch.distributed.run --nproc-per-node N ...`
(bench.py, the CLI with --launcher torchrun). This helper is for tests and the CLI's
`-D N` convenience path: it starts ranks through a *forkserver* that is created
before this process touches a GPU, so no rank is ever exec'ed from a process that
initialised HIP (and RCCL sees one clean process per device).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import socket
import traceback

_CTX = None


def _ctx():
    global _CTX
    if _CTX is None:
        _CTX = mp.get_context("forkserver")
        _CTX.set_forkserver_preload([])
    return _CTX


def warm_forkserver() -> None:
    """Start the forkserver now (call before any GPU use in this process)."""
    ctx = _ctx()
    p = ctx.Process(target=_noop)
    p.start()
    p.join()


def _noop():
    return None


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, q, env):
    os.environ.update(env)
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank), "LOCAL_WORLD_SIZE": str(world)})
    try:
        q.put((rank, "ok", fn(*args)))
    except BaseException as e:  # report, never hang the parent
        q.put((rank, "err", f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))


def spawn_local(world: int, fn, args=(), timeout: float = 600.0, env: dict | None = None) -> list:
    """Run fn(*args) in `world` ranks; returns the per-rank results (rank order)."""
    ctx = _ctx()
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q, dict(env or {}))) for r in range(world)]
    for p in procs:
        p.start()
    results, errors = {}, []
    try:
        for _ in range(world):
            rank, status, payload = q.get(timeout=timeout)
            if status == "ok":
                results[rank] = payload
            else:
                errors.append(f"rank {rank}: {payload}")
                break
    finally:
        for p in procs:
            p.join(timeout=5 if errors else timeout)
            if p.is_alive():
                p.kill()
                p.join()
    if errors:
        raise RuntimeError("\n".join(errors))
    return [results[r] for r in range(world)]
