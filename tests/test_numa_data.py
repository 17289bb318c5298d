"""NUMA-local input copies for the benchmark (parallel/numa_data.py): replica generation is
idempotent, pins the generator to the node's CPUs and restores the affinity; work-list paths are
re-rooted onto the rank's local copy."""
import os

from nm03_capstone_project_amd.parallel.numa_data import (ensure_node_replicas, localize_items, numa_nodes,
                                                          replica_root)


def test_replicas_and_localize(tmp_path, monkeypatch):
    cpus = sorted(os.sched_getaffinity(0))
    seen = []

    def generate(root):
        os.makedirs(root, exist_ok=True)
        seen.append((root, sorted(os.sched_getaffinity(0))))
        open(os.path.join(root, "1-1.dcm"), "w").close()

    def node_cpus(k):  # like numa_node_cpus: the node's CPUs within the CURRENT affinity
        aff = os.sched_getaffinity(0)
        return [c for c in {0: cpus[:1], 1: cpus[-1:]}[k] if c in aff]

    base = str(tmp_path / "data")
    roots = ensure_node_replicas(base, [0, 1], generate, node_cpus)
    assert roots == [replica_root(base, 0), replica_root(base, 1)] == [base + "-node0", base + "-node1"]
    assert seen == [(roots[0], cpus[:1]), (roots[1], cpus[-1:])]
    assert sorted(os.sched_getaffinity(0)) == cpus
    assert ensure_node_replicas(base, [0, 1], generate, node_cpus) == roots and len(seen) == 2  # idempotent
    # single-node host: one shared copy at the base path
    assert ensure_node_replicas(base, [], generate, node_cpus) == [base] and seen[-1] == (base, cpus)

    items = [(roots[0] + "/PGBM-001/s/1-1.dcm", "/out/a"), ("/elsewhere/x.dcm", "/out/b")]
    loc = localize_items(items, roots[0], roots[1])
    assert loc == [(roots[1] + "/PGBM-001/s/1-1.dcm", "/out/a"), ("/elsewhere/x.dcm", "/out/b")]
    assert localize_items(items, roots[0], roots[0]) == items

    monkeypatch.setenv("NM03_NUMA", "0")
    assert numa_nodes(node_cpus) == []
