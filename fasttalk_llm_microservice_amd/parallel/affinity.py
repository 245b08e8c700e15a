"""CPU affinity of a rank: every thread of the process (and of its helper processes,
such as the bench's WebSocket load generator) on the cores of its GPU's NUMA node.

On a two-socket 8 x MI355X node the step-building host path (scheduler, pinned
staging copies, hipGraph launches, the asyncio WebSocket writer) is latency-critical
(README "Service event loop"); left floating, its threads migrate across sockets and
every pinned-buffer copy and graph launch pays the remote-memory path.  vLLM's
equivalent placement is one worker process per GPU (``--tensor-parallel-size``,
``/root/reference/docker-compose.vllm.yml:42``); here the mask is applied INSIDE the
process (never a launcher re-exec: a process that has touched the GPU must not exec).

The GPU's PCI address comes from the device properties (``pci_domain_id`` /
``pci_bus_id`` / ``pci_device_id``), the cores from sysfs
(``/sys/bus/pci/devices/<addr>/local_cpulist``, else its ``numa_node``'s
``cpulist``), intersected with the cores this process may use (cgroup cpuset /
taskset), so a container's CPU share is respected.  ``FT_NUMA_PIN=0`` turns it off.
"""
from __future__ import annotations

import logging
import os
from typing import Iterable, List, Optional, Set

log = logging.getLogger(__name__)


def parse_cpulist(text: str) -> Set[int]:
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11} (sysfs cpulist format)."""
    cpus: Set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            cpus.update(range(int(lo), int(hi) + 1))
        else:
            cpus.add(int(part))
    return cpus


def pci_address(domain: int, bus: int, device: int, function: int = 0) -> str:
    return f"{domain:04x}:{bus:02x}:{device:02x}.{function:x}"


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def device_cpus(pci_addr: str, sysfs: str = "/sys") -> Optional[Set[int]]:
    """Cores local to the PCI device (its NUMA node), or None when sysfs does not say."""
    dev = os.path.join(sysfs, "bus", "pci", "devices", pci_addr.lower())
    lst = _read(os.path.join(dev, "local_cpulist"))
    if lst:
        cpus = parse_cpulist(lst)
        if cpus:
            return cpus
    node = _read(os.path.join(dev, "numa_node"))
    if node is None or not node.lstrip("-").isdigit() or int(node) < 0:
        return None
    lst = _read(os.path.join(sysfs, "devices", "system", "node", f"node{int(node)}", "cpulist"))
    return parse_cpulist(lst) if lst else None


def numa_node(pci_addr: str, sysfs: str = "/sys") -> Optional[int]:
    node = _read(os.path.join(sysfs, "bus", "pci", "devices", pci_addr.lower(), "numa_node"))
    return int(node) if node is not None and node.lstrip("-").isdigit() else None


def affinity_mask(pci_addr: str, allowed: Iterable[int], sysfs: str = "/sys") -> Optional[Set[int]]:
    """The device-local cores this process may use; None (leave the mask alone) when
    sysfs has no locality for the device or none of its cores are allowed."""
    local = device_cpus(pci_addr, sysfs)
    if not local:
        return None
    mask = local & set(allowed)
    return mask or None


def _threads(pid: int) -> List[int]:
    try:
        return [int(t) for t in os.listdir(f"/proc/{pid}/task")]
    except OSError:
        return [pid]


def apply_mask(mask: Set[int], pids: Iterable[int] = ()) -> int:
    """Every thread of this process and of ``pids`` onto ``mask``; returns threads set."""
    n = 0
    for pid in [os.getpid(), *pids]:
        for tid in _threads(pid):
            try:
                os.sched_setaffinity(tid, mask)
                n += 1
            except OSError:
                pass
    return n


def device_pci_address(device_index: int) -> Optional[str]:
    import torch

    p = torch.cuda.get_device_properties(device_index)
    try:
        return pci_address(int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
    except AttributeError:
        return None


def pin_to_device(device_index: int, pids: Iterable[int] = (), sysfs: str = "/sys") -> dict:
    """Pin this process (every thread) and ``pids`` to the cores local to GPU
    ``device_index``.  Returns a description for logs / the bench JSON."""
    info = {"device": device_index, "pci": None, "numa_node": None, "cpus": None, "pinned": False}
    if os.environ.get("FT_NUMA_PIN", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return info
    addr = device_pci_address(device_index)
    info["pci"] = addr
    if addr is None:
        return info
    info["numa_node"] = numa_node(addr, sysfs)
    mask = affinity_mask(addr, os.sched_getaffinity(0), sysfs)
    if mask is None:
        return info
    apply_mask(mask, pids)
    info["cpus"] = len(mask)
    info["pinned"] = True
    log.info("GPU %d (%s, NUMA node %s): %d threads pinned to %d local cores", device_index, addr,
             info["numa_node"], len(_threads(os.getpid())), len(mask))
    return info
