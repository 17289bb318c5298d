"""Per-rank CPU partitions (include/nm03/numa.h rank_partition) on fake sysfs topologies: the ranks
of one node never share CPUs, SMT siblings stay together, pools are sized to the partition and to
the rank's share of the CPU budget (the reference's one machine-wide thread budget,
main_parallel.cpp:401)."""
import pytest


def _fake_host(root, sockets=2, cores=64, smt=2):
    """An EPYC-like host: socket s owns cores s*cores..; CPU c and c + sockets*cores are siblings."""
    ncpu = sockets * cores * smt
    for s in range(sockets):
        lists = []
        for t in range(smt):
            a = t * sockets * cores + s * cores
            lists.append(f"{a}-{a + cores - 1}")
        d = root / "devices/system/node" / f"node{s}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(",".join(lists) + "\n")
    for c in range(ncpu):
        d = root / "devices/system/cpu" / f"cpu{c}" / "topology"
        d.mkdir(parents=True)
        core = c % (sockets * cores)
        (d / "core_id").write_text(f"{core % cores}\n")
        (d / "physical_package_id").write_text(f"{core // cores}\n")
    return list(range(ncpu))


def _parts(native, root, allowed, nodes, budget, cap=16):
    return [native.rank_partition(nodes, r, budget, cap, str(root), allowed) for r in range(len(nodes))]


def test_eight_ranks_two_sockets_disjoint(native, tmp_path):
    allowed = _fake_host(tmp_path)
    parts = _parts(native, tmp_path, allowed, [0, 0, 0, 0, 1, 1, 1, 1], budget=256)
    seen = set()
    for r, p in enumerate(parts):
        cpus = set(p["cpus"])
        assert cpus and not (cpus & seen), (r, p)
        seen |= cpus
        assert p["node"] == (0 if r < 4 else 1) and p["count"] == 4 and p["index"] == r % 4
        assert len(cpus) == 32 and p["threads"] == 16
        # whole cores: every CPU's SMT sibling is in the same partition
        assert all(((c + 128) % 256) in cpus for c in cpus)
        # on the rank's own socket
        sock = {c % 128 // 64 for c in cpus}
        assert sock == {p["node"]}
    assert len(seen) == 256


def test_budget_caps_threads(native, tmp_path):
    """A 16-CPU cgroup quota shared by 8 ranks: 2 pool threads each, CPU sets still disjoint."""
    allowed = _fake_host(tmp_path)
    parts = _parts(native, tmp_path, allowed, [0, 0, 0, 0, 1, 1, 1, 1], budget=16)
    assert [p["threads"] for p in parts] == [2] * 8
    assert sum(len(p["cpus"]) for p in parts) == len(set().union(*(p["cpus"] for p in parts)))


def test_ranks_sharing_one_gpu_split_its_node(native, tmp_path):
    """NM03_DEVICE_OVERRIDE rehearsal: 8 ranks on GPU 0 split socket 0 (8 cores each)."""
    allowed = _fake_host(tmp_path)
    parts = _parts(native, tmp_path, allowed, [0] * 8, budget=256)
    union = set()
    for p in parts:
        assert len(p["cpus"]) == 16 and not (set(p["cpus"]) & union)
        union |= set(p["cpus"])
    assert union == set(range(0, 64)) | set(range(128, 192))


def test_single_rank_gets_its_node(native, tmp_path):
    """The 1-GPU box: a 16-CPU quota keeps 2 CPUs for the slot and runtime threads (14 pool threads);
    a 32-CPU share is capped at 16."""
    allowed = _fake_host(tmp_path)
    (p,) = _parts(native, tmp_path, allowed, [1], budget=16)
    assert p["node"] == 1 and p["cpus"] == list(range(64, 128)) + list(range(192, 256)) and p["threads"] == 14
    (p,) = _parts(native, tmp_path, allowed, [1], budget=32)
    assert p["threads"] == 16


def test_unknown_nodes_and_affinity_mask(native, tmp_path):
    """Ranks whose GPU node is unknown split the allowed CPUs; the affinity mask is respected."""
    _fake_host(tmp_path, sockets=1, cores=8, smt=2)
    allowed = [0, 1, 2, 3, 8, 9, 10, 11]  # 4 cores with their siblings
    parts = _parts(native, tmp_path, allowed, [-1, -1], budget=8)
    assert [sorted(p["cpus"]) for p in parts] == [[0, 1, 8, 9], [2, 3, 10, 11]]
    assert [p["threads"] for p in parts] == [3, 3]  # share 4, one CPU kept for the other threads


@pytest.mark.parametrize("ranks", [3, 5])
def test_more_ranks_than_cores_never_empty(native, tmp_path, ranks):
    _fake_host(tmp_path, sockets=1, cores=1, smt=2)  # 1 core, 2 CPUs
    parts = _parts(native, tmp_path, [0, 1], [0] * ranks, budget=2)
    assert all(p["cpus"] and p["threads"] == 1 for p in parts)


def test_no_numa_tree(native, tmp_path):
    """No sysfs NUMA information: one pseudo node with every allowed CPU."""
    parts = _parts(native, tmp_path, [0, 1, 2, 3], [0, 0], budget=4)
    assert [p["cpus"] for p in parts] == [[0, 1], [2, 3]] and [p["threads"] for p in parts] == [2, 2]


def test_cpulist_format(native):
    assert native.format_cpulist([5, 0, 1, 2, 7, 8, 64]) == "0-2,5,7-8,64"
    assert native.numa_parse_cpulist(native.format_cpulist([3, 4, 9])) == [3, 4, 9]
