"""NUMA binding of a rank to its GPU's socket, against a fake sysfs tree."""
import os

from dmlc_core_amd.parallel import affinity


def _fake_sysfs(root, addr, node, cpulist):
    d = root / "bus/pci/devices" / addr
    d.mkdir(parents=True)
    (d / "numa_node").write_text(f"{node}\n")
    n = root / "devices/system/node" / f"node{node}"
    n.mkdir(parents=True)
    (n / "cpulist").write_text(cpulist + "\n")


def test_parse_cpulist():
    assert affinity._parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert affinity._parse_cpulist("") == []


def test_numa_lookup(tmp_path):
    _fake_sysfs(tmp_path, "0000:05:00.0", 1, "4-7")
    assert affinity.numa_node_of_pci("0000:05:00.0", str(tmp_path)) == 1
    assert affinity.numa_node_of_pci("0000:06:00.0", str(tmp_path)) == -1
    assert affinity.node_cpus(1, str(tmp_path)) == [4, 5, 6, 7]


def test_bind_intersects_allowed_cpus(tmp_path, monkeypatch):
    allowed = sorted(os.sched_getaffinity(0))
    keep = allowed[: max(1, len(allowed) // 2)]
    _fake_sysfs(tmp_path, "0000:05:00.0", 0, ",".join(map(str, keep + [100000])))
    monkeypatch.setattr(affinity, "gpu_pci_address", lambda d: "0000:05:00.0")
    before = os.sched_getaffinity(0)
    try:
        info = affinity.bind_to_gpu(0, str(tmp_path))
        assert info["numa_node"] == 0 and info["bound_cpus"] == len(keep)
        assert sorted(os.sched_getaffinity(0)) == keep
    finally:
        os.sched_setaffinity(0, before)


def test_bind_disabled_or_unknown(tmp_path, monkeypatch):
    monkeypatch.setattr(affinity, "gpu_pci_address", lambda d: "0000:09:00.0")
    before = os.sched_getaffinity(0)
    assert affinity.bind_to_gpu(0, str(tmp_path))["bound_cpus"] == 0  # no sysfs entry
    monkeypatch.setenv("DMLC_NUMA_BIND", "0")
    assert affinity.bind_to_gpu(0, str(tmp_path))["pci"] is None
    assert os.sched_getaffinity(0) == before
