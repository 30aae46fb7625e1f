"""Rank entry points (picklable, importable) for launchers, tests and the CLI."""
from __future__ import annotations

from dataclasses import asdict

from ..models.nqueens import QueensModel
from ..models.pfsp import EngineOptions, PfspModel
from .comm import Comm
from .runtime import DistConfig, DistSolver, distributed_solve


def build_model(spec: dict):
    if spec.get("problem", "pfsp") == "pfsp":
        if spec.get("synthetic"):
            j, mm, seed = spec["synthetic"]
            return PfspModel.synthetic(j, mm, seed, lb=spec.get("lb", 1))
        return PfspModel(spec.get("inst", 14), spec.get("lb", 1))
    return QueensModel(spec.get("N", 14), spec.get("G", 1))


def solve_rank(spec: dict) -> dict:
    """Solve spec's problem cooperatively on all ranks of the current process group."""
    backend = spec.get("backend", "gpu")
    if spec.get("heuristic_ub"):  # CLI --heuristic-ub: -u 0 from the host heuristics' incumbent
        import os

        os.environ.setdefault("TTS_DIVE", "32")
    # comm on the GPU (RCCL) unless asked for gloo, e.g. several ranks sharing one GPU
    if backend == "gpu" and "device" in spec and spec.get("comm", "nccl") == "nccl":
        raise ValueError("spec['device'] puts ranks on one GPU: RCCL needs one GPU per rank, use comm='gloo'")
    comm = Comm(use_gpu=(backend == "gpu" and spec.get("comm", "nccl") == "nccl"))
    try:
        model = build_model(spec)
        opts = EngineOptions(**spec.get("engine", {}))
        device = int(spec.get("device", comm.topo.local_rank)) if backend == "gpu" else 0
        if backend == "gpu" and spec.get("pin", False):
            from .topology import pin_to_device

            pin_to_device(device)
        engine = model.make_engine(backend, device, opts)
        cfg = DistConfig(**spec.get("dist", {}))
        if cfg.cpu_workers > 0:  # a CPU worker next to the rank's engine (ref -C 1)
            engine = model.make_hybrid(engine, backend, cfg.cpu_workers, m=cfg.m, cap=4 * cfg.cpu_batch,
                                       batch=cfg.cpu_batch)
        res = None
        window = opts.max_parents if backend == "gpu" else None
        solver = DistSolver(model, engine, comm, cfg, window=window) if spec.get("session") else None
        for _ in range(int(spec.get("repeat", 1))):
            comm.barrier()
            if solver is not None:  # one native call per solve (what bench.py times)
                res = solver.solve(ub=spec.get("ub", 1))
            else:
                res = distributed_solve(model, engine, comm, ub=spec.get("ub", 1), cfg=cfg, window=window)
        out = {"rank": comm.rank, "world": comm.world, "best": res.best, "tree": res.tree, "sol": res.sol,
               "elapsed": res.elapsed, "t_init": res.t_init, "t_search": res.t_search, "extra": res.extra,
               "workers": [asdict(w) for w in res.workers],
               "comm": {"device_transfers": comm.device_transfers, "host_transfers": comm.host_transfers,
                        "bytes_sent": comm.bytes_sent, "bytes_recv": comm.bytes_recv}}
        del engine
        return out
    finally:
        comm.barrier()
        comm.close()


def preflight_rank(spec: dict) -> dict:
    """Point-to-point preflight (Comm.preflight_p2p) on the current process group;
    spec["corrupt_rank"] makes that rank's received data wrong (test of the check)."""
    use_gpu = spec.get("backend", "cpu") == "gpu" and spec.get("comm", "nccl") == "nccl"
    comm = Comm(use_gpu=use_gpu)
    try:
        bad = spec.get("corrupt_rank")
        if bad is not None and comm.rank == int(bad):
            real = comm._p2p

            def corrupt(outgoing, incoming, src, dst, nb):
                real(outgoing, incoming, src, dst, nb)
                dst[0] ^= 1

            comm._p2p = corrupt
        try:
            return {"rank": comm.rank, "ok": True, "info": comm.preflight_p2p(int(spec.get("nbytes", 1 << 16)))}
        except RuntimeError as e:
            return {"rank": comm.rank, "ok": False, "error": str(e)}
    finally:
        comm.barrier()
        comm.close()
