"""NUMA-local copies of an input dataset held in tmpfs.

tmpfs pages live on the NUMA node of the CPU that wrote them. On a two-socket 8-GPU node a
single shared copy of the benchmark cohort makes the ranks whose GPUs hang off the other socket
read every input byte across the socket interconnect — with weak scaling that is half the ranks,
each reading the whole cohort every step. `ensure_node_replicas` writes one copy per NUMA node
(the generating thread pinned to that node's CPUs, so first touch places the pages there) and
`localize_items` points a rank's work list at the copy on its GPU's node. On single-node hosts
(or with NM03_NUMA=0) everything degenerates to the one shared copy.

The reference has no such concern (one laptop, one process: `main_parallel.cpp:389-411`); this is
part of the per-GPU host placement that `src/runtime/numa.cpp` does for threads and pinned buffers.
"""
import os

NODE_DIR = "/sys/devices/system/node"


def numa_nodes(node_cpus):
    """NUMA nodes that have CPUs this process may run on (`node_cpus(k)` → list of CPUs)."""
    if os.environ.get("NM03_NUMA", "1") == "0" or not os.path.isdir(NODE_DIR):
        return []
    nodes = sorted(int(e[4:]) for e in os.listdir(NODE_DIR) if e.startswith("node") and e[4:].isdigit())
    nodes = [k for k in nodes if node_cpus(k)]
    return nodes if len(nodes) > 1 else []


def replica_root(data_root, node):
    return data_root.rstrip("/") + f"-node{node}"


def ensure_node_replicas(data_root, nodes, generate, node_cpus):
    """Write the dataset once per node in `nodes` (or once at `data_root` when `nodes` is empty).
    `generate(root)` writes one copy; a `.complete` marker makes this idempotent. Returns the roots."""
    roots = [replica_root(data_root, k) for k in nodes] or [data_root]
    saved = os.sched_getaffinity(0) if nodes else None
    # CPU lists first: node_cpus() filters by the current affinity, which the loop narrows.
    cpus = {k: list(node_cpus(k)) for k in nodes}
    try:
        for k, root in zip(nodes or [None], roots):
            marker = os.path.join(root, ".complete")
            if os.path.exists(marker):
                continue
            if k is not None:
                try:  # inherited by the generator's worker threads
                    os.sched_setaffinity(0, cpus[k] or saved)
                except OSError:  # cpuset narrower than the affinity mask: place what we can
                    os.sched_setaffinity(0, saved)
            generate(root)
            open(marker, "w").close()
    finally:
        if saved is not None:
            os.sched_setaffinity(0, saved)
    return roots


def localize_items(items, plan_root, local_root):
    """Rewrite the input paths of (path, out_dir) items from `plan_root` to `local_root`."""
    if plan_root == local_root:
        return list(items)
    a = plan_root.rstrip("/") + "/"
    b = local_root.rstrip("/") + "/"
    return [(b + p[len(a):] if p.startswith(a) else p, od) for p, od in items]
