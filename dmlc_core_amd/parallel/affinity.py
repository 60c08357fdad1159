"""Bind a rank's host threads to the NUMA node of its MI355X.

On a two-socket MI355X node each GPU hangs off one socket's PCIe root
complex.  The ingestion path DMAs text straight out of the page cache
(mmap + hipHostRegister, ``src/gpu/zero_copy_source.h``), so the pages a GPU
reads should live in DRAM on *its* socket: otherwise every byte crosses the
inter-socket link, and with 8 GPUs x 55 GB/s of H2D that link, not PCIe,
becomes the bound.  Linux places page-cache and anonymous pages on the node
of the CPU that first touches them, so binding each rank (and every thread it
spawns afterwards: reader pools, generator threads) to its GPU's node before
it generates or reads data is enough -- no libnuma needed.

The reference has no GPU and no affinity logic; its launcher only forwards
``OMP_NUM_THREADS`` / ``KMP_AFFINITY`` (`tracker/dmlc_tracker/ssh.py:23-35`).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional


def _parse_cpulist(text: str) -> List[int]:
    cpus: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            cpus.extend(range(int(lo), int(hi) + 1))
        else:
            cpus.append(int(part))
    return cpus


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def gpu_pci_address(device: int) -> Optional[str]:
    """``dddd:bb:dd.0`` of HIP device `device`, from torch's device properties."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device)
    except Exception:  # noqa: BLE001 - no GPU / no torch
        return None
    bus = getattr(p, "pci_bus_id", None)
    dev = getattr(p, "pci_device_id", None)
    dom = getattr(p, "pci_domain_id", 0) or 0
    if bus is None or dev is None:
        return None
    return f"{int(dom):04x}:{int(bus):02x}:{int(dev):02x}.0"


def numa_node_of_pci(addr: str, sysfs: str = "/sys") -> int:
    """NUMA node of a PCI function (-1 if unknown / single-node system)."""
    v = _read(os.path.join(sysfs, "bus/pci/devices", addr, "numa_node"))
    try:
        return int(v) if v is not None else -1
    except ValueError:
        return -1


def node_cpus(node: int, sysfs: str = "/sys") -> List[int]:
    v = _read(os.path.join(sysfs, "devices/system/node", f"node{node}", "cpulist"))
    return _parse_cpulist(v) if v else []


def bind_to_gpu(device: int, sysfs: str = "/sys") -> Dict[str, object]:
    """Restrict this process to the CPUs of `device`'s NUMA node.

    Only CPUs already allowed (cgroup cpuset / parent affinity) are kept; if
    the intersection is empty or the node is unknown nothing changes.
    Returns a small report for logs / benchmark JSON.  ``DMLC_NUMA_BIND=0``
    disables it.
    """
    info: Dict[str, object] = {"device": device, "pci": None, "numa_node": -1, "bound_cpus": 0}
    if os.environ.get("DMLC_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return info
    addr = gpu_pci_address(device)
    info["pci"] = addr
    if addr is None:
        return info
    node = numa_node_of_pci(addr, sysfs)
    info["numa_node"] = node
    if node < 0:
        return info
    allowed = os.sched_getaffinity(0)
    cpus = sorted(set(node_cpus(node, sysfs)) & allowed)
    if not cpus:
        return info
    os.sched_setaffinity(0, cpus)
    info["bound_cpus"] = len(cpus)
    return info
