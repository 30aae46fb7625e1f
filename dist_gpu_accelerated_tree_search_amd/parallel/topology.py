"""GPU <-> host topology for rank placement.

Parity: ref common/get_numa_affinity.py writes an affinity.txt from lscpu and
rocm-smi output that nothing reads. Here a rank pins itself to the CPUs of its
GPU's NUMA node (PCI bus id from HIP -> /sys/bus/pci/devices/<id>/numa_node ->
/sys/devices/system/node/node<N>/cpulist), which keeps the host thread that
drives the device, its pinned staging buffers and the RCCL proxy threads local.
"""
from __future__ import annotations

import os

from .. import ops


def device_cpus(device: int) -> list[int]:
    """NUMA-local CPUs of `device` ([] when unknown, e.g. no sysfs entry)."""
    try:
        return list(ops.hip().device_cpus(int(device)))
    except Exception:  # noqa: BLE001 - topology is advisory
        return []


def pin_to_device(device: int) -> list[int]:
    """Restrict this process to the NUMA-local CPUs of `device` that it may already
    use. Returns the new CPU set ([] = left unchanged)."""
    cpus = set(device_cpus(device))
    try:
        allowed = os.sched_getaffinity(0)
    except AttributeError:
        return []
    mine = sorted(cpus & allowed)
    if not mine:
        return []
    os.sched_setaffinity(0, mine)
    return mine


def describe(n_devices: int | None = None) -> list[dict]:
    """One record per visible GPU: bus id, NUMA-local CPUs (for logs and tools)."""
    H = ops.hip()
    n = H.device_count() if n_devices is None else n_devices
    return [{"device": d, "pci_bus_id": H.device_pci_bus_id(d), "cpus": list(H.device_cpus(d))} for d in range(n)]


if __name__ == "__main__":
    import json

    import torch  # noqa: F401  (one HIP runtime)

    for rec in describe():
        print(json.dumps(rec))
