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
import sys
import traceback

_CTX = None
_WARM = False


def _ctx():
    global _CTX
    if _CTX is None:
        _CTX = mp.get_context("forkserver")
        _CTX.set_forkserver_preload([])
    return _CTX


def warm_forkserver() -> None:
    """Start the forkserver now (call before any GPU use in this process)."""
    global _WARM
    if _WARM:
        return
    ctx = _ctx()
    p = ctx.Process(target=_noop)
    p.start()
    p.join()
    _WARM = True


def hip_touched() -> bool:
    """True once this process may have initialised HIP: torch's lazy CUDA/HIP init ran, or
    the gfx950 extension was loaded (its engines make HIP calls)."""
    torch = sys.modules.get("torch")
    try:
        if torch is not None and torch.cuda.is_initialized():
            return True
    except Exception:  # pragma: no cover - torch without a cuda module
        pass
    ops = sys.modules.get("dist_gpu_accelerated_tree_search_amd.ops")
    return ops is not None and getattr(ops, "_hip_mod", None) is not None


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
    """Run fn(*args) in `world` ranks; returns the per-rank results (rank order).

    Refuses to start the forkserver from a process that may have initialised HIP: the
    forkserver is a fork+exec, and exec from a GPU-initialised process is forbidden
    (call warm_forkserver() first, as the CLI and the test session do)."""
    if not _WARM and hip_touched():
        raise RuntimeError("spawn_local: the rank forkserver was not started before this process used HIP; "
                           "call parallel.launch.warm_forkserver() before any GPU call")
    warm_forkserver()
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
