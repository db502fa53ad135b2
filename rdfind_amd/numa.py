"""Host placement next to the GPU (the `numactl --cpunodebind` a deployment would use, done in-process).

The hand-over copies the result into page-locked host memory, and the synthetic / parsed inputs are uploaded from
host memory.  On the two-socket GPU hosts, a process may run on the socket that is not the GPU's, and its pinned
buffers then land on the remote NUMA node (first touch), so every copy crosses the inter-socket link.  Some c2 bench
processes on one box spent ~1 ms per step on the hand-over where others spent ~0.15 ms (profiles/r06_numa_ab.log).
Binding the process to the CPUs of the GPU's node before any host buffer is allocated keeps them local; it is what a
deployment does with `numactl --cpunodebind`.
"""
import glob
import os


def _parse_cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def device_numa_node(device=0):
    """NUMA node of GPU `device` (sysfs of its PCI function), or None when unknown."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device)
        pattern = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.*/numa_node"
    except Exception:
        return None
    for f in sorted(glob.glob(pattern)):
        try:
            node = int(open(f).read())
        except (OSError, ValueError):
            continue
        if node >= 0:
            return node
    return None


def bind_to_device_node(device=0):
    """Restrict this process's CPUs to the GPU's NUMA node (within its current affinity).  Returns the node, or
    None when the topology is unknown or binding would leave no CPU (then nothing changes)."""
    node = device_numa_node(device)
    if node is None:
        return None
    try:
        cpus = _parse_cpulist(open(f"/sys/devices/system/node/node{node}/cpulist").read())
        allowed = cpus & os.sched_getaffinity(0)
        if not allowed:
            return None
        os.sched_setaffinity(0, allowed)
    except OSError:
        return None
    return node
