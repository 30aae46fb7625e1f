"""torch.distributed transport for the tree-search runtime (RCCL on MI355X, gloo on CPU).

One process per GPU. The reference moves work between GPUs through host memory
under OpenMP spin locks (ref pfsp_multigpu_cuda.c:343-431) and between nodes with
MPI Allgather/Allgatherv of every donor's nodes (ref pfsp_dist_multigpu_cuda.c:
122-137, 364-469). Here every exchange is a collective or a targeted point-to-point
transfer issued by all ranks in the same order:
  * status round      one all_gather of a small int64 record per rank
                      (pool size, incumbent, idle flag) — replaces the separate
                      Allreduce(best) + Allgather(termination) + Allgather(needs)
  * work transfer     donor -> needy only, straight from the device pool into the
                      peer's pool over xGMI; never an all-gather of everybody's
                      nodes. With GPU engines the transfer is NATIVE: one RCCL
                      communicator of this job (csrc/hip/rccl_transport.hpp, built
                      from a unique id rank 0 broadcasts once) issues ncclGroupStart /
                      ncclSend / ncclRecv / ncclGroupEnd on the engine's transfer
                      stream from inside the native round loop — no Python, no torch
                      tensors per round. Stream-ordered: the copy out of the pool,
                      the send/recv and the copy into the peer's pool are chained
                      with events, without a host wait. (TTS_NATIVE_RCCL=0: the same
                      plan through torch batch_isend_irecv; gloo / CPU engines:
                      host arrays.)
  * final reduction   all_reduce SUM of counters / MIN of the incumbent.
When every rank is on this node (torchrun --nnodes=1) the status records, barriers
and final reductions go through a shared-memory control plane instead
(csrc/core/shm_control.hpp: ~1 us per all-gather instead of a collective plus two
host<->device copies); node payloads still go GPU -> GPU over RCCL/xGMI.
TTS_SHM_CONTROL=0 keeps everything on the process group.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import numpy as np


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


SHM_MAX_VALS = 15  # values per rank in one shared-memory all-gather (ShmControl::kMaxVals)


def shm_control_wanted(topo: "Topology") -> bool:
    """Use the shared-memory control plane when every rank lives on this node
    (TTS_SHM_CONTROL=0 forces the process-group collectives)."""
    if os.environ.get("TTS_SHM_CONTROL", "1") == "0":
        return False
    return topo.world > 1 and topo.local_world == topo.world and os.path.isdir("/dev/shm")


@dataclass
class Topology:
    rank: int
    world: int
    local_rank: int
    local_world: int

    @property
    def node(self) -> int:
        return self.rank // max(1, self.local_world)


class Comm:
    """Process-group wrapper; world == 1 works without any process group."""

    def __init__(self, backend: str | None = None, use_gpu: bool = True, timeout_s: float = 1800.0,
                 device: int | None = None, preflight_raise: bool = True):
        import torch
        import torch.distributed as dist

        self.torch = torch
        self.dist = dist
        self.topo = Topology(rank=_env_int("RANK", 0), world=_env_int("WORLD_SIZE", 1),
                             local_rank=_env_int("LOCAL_RANK", 0),
                             local_world=_env_int("LOCAL_WORLD_SIZE", _env_int("WORLD_SIZE", 1)))
        self.use_gpu = use_gpu
        if use_gpu:
            # device: this rank's GPU (default LOCAL_RANK; tests put several ranks on one)
            dev = self.topo.local_rank if device is None else int(device)
            torch.cuda.set_device(dev)
            self.device = torch.device("cuda", dev)
        else:
            self.device = torch.device("cpu")
        self.backend = backend or ("nccl" if use_gpu else "gloo")
        self._owns_pg = False
        if self.topo.world > 1 and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = dict(backend=self.backend, timeout=datetime.timedelta(seconds=timeout_s))
            if use_gpu and self.backend == "nccl":
                kw["device_id"] = self.device
            dist.init_process_group(**kw)
            self._owns_pg = True
        self._buf = None
        self.bytes_sent = 0
        self.bytes_recv = 0
        self.device_transfers = 0   # transfers through device staging (GPU engines)
        self.host_transfers = 0     # transfers through host arrays (CPU engines)
        self.timeout_s = timeout_s
        self.ctl = None
        self._staging = {}
        if shm_control_wanted(self.topo):
            self.ctl = self._open_shm_control()
        self.preflight = None
        self.p2p_ok = True
        self.rccl = None  # native RCCL transport (GPU ranks over nccl)
        # fault injection (like TTS_FAULT_*): the preflight runs on any backend and the
        # data this rank receives is corrupted
        fault = os.environ.get("TTS_FAULT_P2P_RANK")
        if self.distributed and ((use_gpu and self.backend == "nccl") or fault not in (None, "")):
            try:
                if use_gpu and self.backend == "nccl":
                    self._connect_peers()
                    if os.environ.get("TTS_NATIVE_RCCL", "1") != "0":
                        self.rccl = self._open_rccl()
                if self.rccl is not None:
                    # the native path end to end (what the round loop will use)
                    self.preflight = self.rccl.preflight(
                        4 << 20, corrupt=fault not in (None, "") and int(fault) == self.rank)
                elif fault not in (None, "") and int(fault) == self.rank:
                    real = self._p2p

                    def corrupt(outgoing, incoming, src, dst, nb):
                        real(outgoing, incoming, src, dst, nb)
                        if dst is not None and dst.numel():
                            dst[0] ^= 1

                    self._p2p = corrupt
                    try:
                        self.preflight = self.preflight_p2p()
                    finally:
                        self._p2p = real
                elif os.environ.get("TTS_P2P_PREFLIGHT", "1") != "0" or fault not in (None, ""):
                    self.preflight = self.preflight_p2p()
            except Exception as e:  # noqa: BLE001 - re-raised unless the caller takes it
                if preflight_raise:
                    raise
                # every rank learns that some rank's point-to-point path failed; the caller
                # runs without node transfers (static partition) and reports the failure
                self.preflight = {"ok": False, "error": repr(e)[:300]}
        if self.distributed and not preflight_raise:
            mine = 1 if (self.preflight is None or self.preflight.get("ok")) else 0
            self.p2p_ok = bool(self.allreduce_i64([mine], "min")[0])

    def preflight_p2p(self, nbytes: int = 4 << 20) -> dict:
        """Check the node-transfer path end to end before any solve relies on it.

        Every rank sends a rank-stamped pattern of `nbytes` to every peer and receives
        one from each, through the same grouped isend/irecv (`_p2p`) that
        execute_transfers uses, enqueued on a side stream wrapped as an external stream
        exactly like the engine's transfer stream. Each received buffer is compared
        word for word with the pattern its sender must have written; a mismatch or a
        failed call raises with the peers involved (no silent fallback, no restart).
        Returns {"ok", "peers", "bytes_per_peer", "seconds", "GBps"} (GBps: bytes this
        rank received per second over all its links). With gloo the buffers are host
        tensors (CPU tests drive the same code)."""
        if not self.distributed:
            return {"ok": True, "peers": 0, "bytes_per_peer": 0, "seconds": 0.0, "GBps": 0.0}
        torch = self.torch
        me, n = self.rank, self.world
        peers = [p for p in range(n) if p != me]
        words = max(1, int(nbytes) // 4)
        nccl = self.backend == "nccl"
        dev = self.device if nccl else torch.device("cpu")

        def pattern(src: int, dst: int):
            i = torch.arange(words, dtype=torch.int64, device=dev)
            v = (i * 2654435761 + src * 0x9E3779B1 + dst * 0x85EBCA77 + 12345) & 0x7FFFFFFF
            return v.to(torch.int32)

        ctx = None
        if nccl:
            side = torch.cuda.Stream(device=dev)
            ctx = torch.cuda.ExternalStream(side.cuda_stream, device=dev)
        import contextlib
        import time as _time

        with (torch.cuda.stream(ctx) if ctx is not None else contextlib.nullcontext()):
            src = torch.cat([pattern(me, p) for p in peers]).view(torch.uint8)
            dst = torch.zeros(len(peers) * words, dtype=torch.int32, device=dev).view(torch.uint8)
            plan_out = [(p, words) for p in peers]
            plan_in = [(p, words) for p in peers]
            if nccl:
                ctx.synchronize()
            t0 = _time.perf_counter()
            try:
                self._p2p(plan_out, plan_in, src, dst, 4)
                if nccl:
                    ctx.synchronize()
            except Exception as e:  # noqa: BLE001 - re-raised with context
                raise RuntimeError(f"rank {me}: {self.backend} point-to-point preflight failed "
                                   f"({len(peers)} peers, {words * 4} B each): {e}") from e
            dt = _time.perf_counter() - t0
            got = dst.view(torch.int32).reshape(len(peers), words)
            bad = [p for k, p in enumerate(peers) if not torch.equal(got[k], pattern(p, me))]
        if bad:
            raise RuntimeError(f"rank {me}: {self.backend} point-to-point preflight: data received from "
                               f"rank(s) {bad} does not match what they sent; node transfers over this "
                               "backend would corrupt the pools")
        return {"ok": True, "peers": len(peers), "bytes_per_peer": words * 4, "seconds": dt,
                "GBps": len(peers) * words * 4 / max(dt, 1e-9) / 1e9}

    def _open_rccl(self):
        """This job's native RCCL communicator: rank 0 creates the unique id, one
        broadcast over the process group hands it to every rank, every rank builds
        its communicator (ncclCommInitRank waits for all of them)."""
        from .. import ops

        torch, dist = self.torch, self.dist
        H = ops.hip()
        uid = H.RcclTransport.new_id() if self.rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8, device=self.device)
        dist.broadcast(t, src=0)
        uid = bytes(t.cpu().tolist())
        tr = H.RcclTransport(uid, self.rank, self.world, self.device.index)
        tr.timeout_s = float(self.timeout_s)  # bounded round all-gathers (dead peer -> abort + raise)
        return tr

    def transport(self, engine, node_bytes: int):
        """What the native round loop moves nodes with: the native RCCL transport for a
        GPU engine (no callback into Python), else execute_transfers."""
        if self.rccl is not None and int(getattr(engine, "transfer_stream", 0) or 0):
            return self.rccl
        return lambda plan: self.execute_transfers(plan, engine, node_bytes)

    def round_allgather(self, engine):
        """The round loop's status all-gather when there is no shm board (several nodes,
        TTS_SHM_CONTROL=0): the native RCCL transport for a GPU engine with a transfer
        stream — ncclAllGather on that stream, after the previous round's send / recv, so
        the communicator never has two collectives in flight and no Python runs per
        round — else the process group's all-gather (allgather_i64). Set
        TTS_RCCL_CONTROL=0 for the process-group path."""
        if (self.rccl is not None and int(getattr(engine, "transfer_stream", 0) or 0)
                and os.environ.get("TTS_RCCL_CONTROL", "1") != "0"):
            return self.rccl
        xs = int(getattr(engine, "transfer_stream", 0) or 0)
        if self.rccl is not None and xs:
            # the process group is a second communicator: let the native transport's
            # send / recv of the previous round finish first (NCCL: two communicators in
            # flight on the same GPUs can deadlock)
            stream = self.torch.cuda.ExternalStream(xs, device=self.device)

            def allgather_after_transfers(values):
                stream.synchronize()
                return self.allgather_i64(values)

            return allgather_after_transfers
        return self.allgather_i64

    def _connect_peers(self) -> None:
        """RCCL sets up a point-to-point channel on first use; do it for every pair now
        (one grouped send/recv of one byte per peer), outside any timed region."""
        torch, dist = self.torch, self.dist
        me, n = self.rank, self.world
        send = torch.zeros(n, dtype=torch.uint8, device=self.device)
        recv = torch.empty(n, dtype=torch.uint8, device=self.device)
        ops = []
        for p in range(n):
            if p != me:
                ops.append(dist.P2POp(dist.isend, send[p:p + 1], p))
                ops.append(dist.P2POp(dist.irecv, recv[p:p + 1], p))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        torch.cuda.synchronize(self.device)

    def control_address(self, module) -> int:
        """Address of this rank's shared-memory control plane for the native round loop
        of `module` (the ShmControl object is shared by both native modules, same
        header and layout), or 0 when rounds go through the process group."""
        return int(self.ctl.address) if self.ctl is not None else 0

    def _open_shm_control(self):
        """Shared-memory control plane for a single-node job (csrc/core/shm_control.hpp):
        rank 0 creates a uniquely named segment, the name's nonce travels over the
        process group once, every rank maps it, then the name is unlinked (nothing
        is left in /dev/shm, even if a rank dies later)."""
        from .. import ops

        C = ops.cpu()
        torch = self.torch
        ctl, err = None, None
        nonce = int.from_bytes(os.urandom(6), "little")
        name = f"/tts_ctl_{os.getuid()}_{os.environ.get('MASTER_PORT', '0')}_{nonce:x}"
        if self.rank == 0:
            try:
                ctl = C.ShmControl(name, 0, self.world, True)
            except Exception as e:  # no /dev/shm, quota, ...: fall back to the process group
                err = e
        t = torch.tensor([nonce, int(ctl is not None)], dtype=torch.int64, device=self.device)
        self.dist.broadcast(t, src=0)
        nonce, ok0 = (int(x) for x in t.tolist())
        name = f"/tts_ctl_{os.getuid()}_{os.environ.get('MASTER_PORT', '0')}_{nonce:x}"
        if self.rank != 0 and ok0:
            try:
                ctl = C.ShmControl(name, self.rank, self.world, False)
            except Exception as e:
                err = e
        # every rank must agree on the plane: use it only if all ranks mapped it
        ok = torch.tensor([int(ctl is not None)], dtype=torch.int64, device=self.device)
        self.dist.all_reduce(ok, op=self.dist.ReduceOp.MIN)
        if self.rank == 0 and ctl is not None:
            ctl.unlink()
        if int(ok.item()) == 0:
            if err is not None:
                print(f"[tts] rank {self.rank}: shared-memory control plane unavailable ({err}); "
                      "using the process group", flush=True)
            return None
        return ctl

    def _pg_barrier(self) -> None:
        if self.use_gpu and self.backend == "nccl":
            self.dist.barrier(device_ids=[self.device.index])
        else:
            self.dist.barrier()

    # ---- basic properties ----
    @property
    def rank(self) -> int:
        return self.topo.rank

    @property
    def world(self) -> int:
        return self.topo.world

    @property
    def distributed(self) -> bool:
        return self.topo.world > 1

    def sync_device(self) -> None:
        if self.use_gpu:
            self.torch.cuda.synchronize(self.device)

    def barrier(self) -> None:
        if self.distributed:
            if self.ctl is not None:
                self.ctl.barrier(self.timeout_s)
            else:
                self._pg_barrier()
        self.sync_device()

    def close(self) -> None:
        self.ctl = None
        self.rccl = None
        if self._owns_pg and self.dist.is_initialized():
            self.dist.destroy_process_group()
            self._owns_pg = False

    # ---- collectives on small int64 records ----
    def allgather_i64(self, values) -> np.ndarray:
        vals = np.asarray(values, dtype=np.int64).reshape(-1)
        if not self.distributed:
            return vals.reshape(1, -1)
        if self.ctl is not None and vals.size <= SHM_MAX_VALS:
            return self.ctl.allgather(vals, self.timeout_s)
        t = self.torch.as_tensor(vals, dtype=self.torch.int64).to(self.device)
        out = self.torch.empty(self.world * vals.size, dtype=self.torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(out, t)
        return out.cpu().numpy().reshape(self.world, vals.size)

    def allreduce_i64(self, values, op: str = "sum") -> np.ndarray:
        vals = np.asarray(values, dtype=np.int64).reshape(-1)
        if not self.distributed:
            return vals
        if self.ctl is not None and vals.size <= SHM_MAX_VALS:
            g = self.ctl.allgather(vals, self.timeout_s)
            return {"sum": g.sum(axis=0), "min": g.min(axis=0), "max": g.max(axis=0)}[op].astype(np.int64)
        t = self.torch.as_tensor(vals, dtype=self.torch.int64).to(self.device)
        rop = {"sum": self.dist.ReduceOp.SUM, "min": self.dist.ReduceOp.MIN, "max": self.dist.ReduceOp.MAX}[op]
        self.dist.all_reduce(t, op=rop)
        return t.cpu().numpy()

    def allgather_f64(self, values) -> np.ndarray:
        vals = np.asarray(values, dtype=np.float64).reshape(-1)
        if not self.distributed:
            return vals.reshape(1, -1)
        if self.ctl is not None and vals.size <= SHM_MAX_VALS:
            return self.ctl.allgather(vals.view(np.int64), self.timeout_s).view(np.float64)
        t = self.torch.as_tensor(vals, dtype=self.torch.float64).to(self.device)
        out = self.torch.empty(self.world * vals.size, dtype=self.torch.float64, device=self.device)
        self.dist.all_gather_into_tensor(out, t)
        return out.cpu().numpy().reshape(self.world, vals.size)

    # ---- node transfers ----
    def _stage(self, device, nbytes: int, slot: str):
        key = (str(device), slot)
        buf = self._staging.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = self.torch.empty(max(nbytes, 1 << 20), dtype=self.torch.uint8, device=device)
            self._staging[key] = buf
        return buf

    def execute_transfers(self, plan, engine, node_bytes: int) -> tuple[int, int]:
        """Run the planned (donor, receiver, count) transfers. Every rank calls this
        with the same plan. Returns (nodes_sent, nodes_received) for this rank.

        GPU engine + RCCL: pool -> device staging -> send/recv over xGMI -> peer
        staging -> peer pool, every step enqueued on the engine's streams and
        ordered by events (engine_api.hpp): no host wait, no device-wide sync.
        GPU engine + gloo (ranks sharing a GPU in tests): the same device staging,
        with a host hop around the gloo send/recv.
        CPU engine: host arrays (engine.pop / engine.push)."""
        me = self.rank
        outgoing = [(r, k) for (d, r, k) in plan if d == me and k > 0]
        incoming = [(d, k) for (d, r, k) in plan if r == me and k > 0]
        if not outgoing and not incoming:
            return 0, 0
        if self.rccl is not None and int(getattr(engine, "transfer_stream", 0) or 0):
            sent, got = self.rccl.execute([tuple(t) for t in plan], engine)
            self.device_transfers += 1
            self.bytes_sent += sent * node_bytes
            self.bytes_recv += got * node_bytes
            return sent, got
        total_out = sum(k for _, k in outgoing)
        total_in = sum(k for _, k in incoming)
        torch, dist = self.torch, self.dist
        xs = int(getattr(engine, "transfer_stream", 0) or 0)
        if xs:
            self.device_transfers += 1
            dev = torch.device("cuda", engine.device)
            stream = torch.cuda.ExternalStream(xs, device=dev)
            nccl = self.backend == "nccl"
            with torch.cuda.stream(stream):
                src = dst = None
                if outgoing:
                    src = self._stage(dev, total_out * node_bytes, "out")
                    got = engine.export_to(src.data_ptr(), total_out)
                    if got != total_out:
                        raise RuntimeError(f"rank {me}: planned to send {total_out} nodes, pool gave {got}")
                    if not nccl:  # host hop (on the transfer stream, after the export copy)
                        src = src[:total_out * node_bytes].cpu()
                if incoming:
                    dst = self._stage(dev, total_in * node_bytes, "in")
                    if not nccl:
                        dst_dev, dst = dst, torch.empty(total_in * node_bytes, dtype=torch.uint8)
                self._p2p(outgoing, incoming, src, dst, node_bytes)
                if incoming:
                    if not nccl:
                        dst_dev[:total_in * node_bytes].copy_(dst, non_blocking=False)
                        dst = dst_dev
                    engine.import_from(dst.data_ptr(), total_in)
        else:
            self.host_transfers += 1
            src = None
            if outgoing:
                host = engine.pop(total_out)
                if len(host) != total_out:
                    raise RuntimeError(f"rank {me}: planned to send {total_out} nodes, pool gave {len(host)}")
                src = torch.from_numpy(np.ascontiguousarray(host).reshape(-1))
            dst = torch.empty(total_in * node_bytes, dtype=torch.uint8) if incoming else None
            self._p2p(outgoing, incoming, src, dst, node_bytes)
            if incoming:
                engine.push(dst.numpy().reshape(total_in, node_bytes))
        self.bytes_sent += total_out * node_bytes
        self.bytes_recv += total_in * node_bytes
        return total_out, total_in

    def _p2p(self, outgoing, incoming, src, dst, node_bytes: int) -> None:
        """Grouped isend/irecv; with RCCL, wait() only orders the current (transfer)
        stream after the communication — the host does not block."""
        dist = self.dist
        ops = []
        off = 0
        for r, k in outgoing:
            ops.append(dist.P2POp(dist.isend, src[off * node_bytes:(off + k) * node_bytes], r))
            off += k
        off = 0
        for d, k in incoming:
            ops.append(dist.P2POp(dist.irecv, dst[off * node_bytes:(off + k) * node_bytes], d))
            off += k
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def plan_sharing(sizes, m: int, cap: int, node_of=None, intra: bool = True, inter: bool = True,
                 donor_min: int | None = None):
    """Deterministic steal-half matching computed identically on every rank
    (Python reference of the native plan_transfers in csrc/core/dist_rounds.hpp,
    which the runtime uses; tests check that the two agree).

    needy  = ranks whose pool holds fewer than m nodes (ref popBackBulk threshold),
    donors = ranks with at least donor_min (default 2m) nodes (ref `size >= 2*m`).
    Each needy rank is served by the donor with the most nodes left, which hands
    over half of what it has (capped at `cap`, ref 5*M). intra/inter restrict pairs
    to the same node (-w) or to different nodes (-L)."""
    sizes = [int(s) for s in sizes]
    n = len(sizes)
    node_of = node_of or (lambda r: 0)
    left = list(sizes)
    needy = [r for r in range(n) if sizes[r] < m]
    needy_set = set(needy)
    plan = []
    dmin = 2 * m if donor_min is None else donor_min
    for r in needy:
        cands = [d for d in range(n) if left[d] >= dmin and d not in needy_set and
                 ((intra and node_of(d) == node_of(r)) or (inter and node_of(d) != node_of(r)))]
        if not cands:
            continue
        d = max(cands, key=lambda x: (left[x], -x))
        k = min(left[d] // 2, cap)
        if k <= 0:
            continue
        left[d] -= k
        left[r] += k
        plan.append((d, r, k))
    return plan
