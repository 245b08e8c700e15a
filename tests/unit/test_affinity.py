"""NUMA placement of a rank (parallel/affinity.py): the GPU's
local cores from sysfs, intersected with the cores the process may use, checked
against a fake sysfs tree."""
import os

from fasttalk_llm_microservice_amd.parallel import affinity as A


def _sysfs(tmp_path, devs, nodes):
    for addr, (numa, local) in devs.items():
        d = tmp_path / "bus" / "pci" / "devices" / addr
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{numa}\n")
        if local is not None:
            (d / "local_cpulist").write_text(local + "\n")
    for n, lst in nodes.items():
        d = tmp_path / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(lst + "\n")
    return str(tmp_path)


def test_parse_cpulist():
    assert A.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert A.parse_cpulist("") == set()
    assert A.pci_address(0, 0x75, 0) == "0000:75:00.0"


def test_mask_from_local_cpulist_and_numa_fallback(tmp_path):
    root = _sysfs(tmp_path, {"0000:05:00.0": (0, "0-47,96-143"), "0000:85:00.0": (1, None),
                             "0000:f5:00.0": (-1, None)},
                  {0: "0-47,96-143", 1: "48-95,144-191"})
    allowed = set(range(192))
    assert A.affinity_mask("0000:05:00.0", allowed, root) == set(range(48)) | set(range(96, 144))
    # no local_cpulist: the device's NUMA node's cpulist
    assert A.affinity_mask("0000:85:00.0", allowed, root) == set(range(48, 96)) | set(range(144, 192))
    assert A.numa_node("0000:85:00.0", root) == 1
    # numa_node -1 (no locality) or an unknown device: leave the mask alone
    assert A.affinity_mask("0000:f5:00.0", allowed, root) is None
    assert A.affinity_mask("0000:99:00.0", allowed, root) is None


def test_mask_respects_the_allowed_cores(tmp_path):
    root = _sysfs(tmp_path, {"0000:05:00.0": (0, "0-47")}, {0: "0-47"})
    # a container's cpuset: only cores 40..63 usable -> the local ones among them
    assert A.affinity_mask("0000:05:00.0", range(40, 64), root) == set(range(40, 48))
    # none of the local cores allowed: do not pin (a foreign node is better than nothing)
    assert A.affinity_mask("0000:05:00.0", range(100, 110), root) is None


def test_apply_mask_sets_every_thread():
    import threading

    before = os.sched_getaffinity(0)
    ev = threading.Event()
    t = threading.Thread(target=ev.wait, daemon=True)
    t.start()
    try:
        mask = {min(before)}
        n = A.apply_mask(mask)
        assert n >= 2   # this thread and the waiting one
        assert os.sched_getaffinity(0) == mask
        assert os.sched_getaffinity(t.native_id) == mask
    finally:
        A.apply_mask(before)
        ev.set()


def test_pin_disabled_by_env(monkeypatch):
    monkeypatch.setenv("FT_NUMA_PIN", "0")
    info = A.pin_to_device(0)
    assert info["pinned"] is False and info["pci"] is None
