"""CPU: the multi-GPU tests (tests/test_gpu_multi.py) are collected and NOT
skipped when the box shows several devices.

The device count is mocked with NKV_TEST_DEVICE_COUNT, which
tests/test_gpu_multi.visible_devices() reads before torch's count.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _collect(count):
    env = dict(os.environ, NKV_TEST_DEVICE_COUNT=str(count))
    out = subprocess.run([sys.executable, "-m", "pytest", "--collect-only", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                          "tests/test_gpu_multi.py"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    return [x for x in out.stdout.splitlines() if "::" in x]


def test_collected_over_eight_devices():
    ids = _collect(8)
    assert "tests/test_gpu_multi.py::test_group_rccl_distinct_devices[devs01234567]" in ids
    assert "tests/test_gpu_multi.py::test_group_rccl_distinct_devices[devs01]" in ids
    assert "tests/test_gpu_multi.py::test_group_split_distinct_devices[65537-devs01234567]" in ids
    assert "tests/test_gpu_multi.py::test_group_split_fuzz_distinct_devices[0-devs01234567]" in ids
    assert "tests/test_gpu_multi.py::test_group_refuses_pointers_on_another_device[devs01234567]" in ids
    assert "tests/test_gpu_multi.py::test_group_mixed_copy_transport[devs001]" in ids
    assert "tests/test_gpu_multi.py::test_group_peer_access[devs01234567]" in ids
    assert "tests/test_gpu_multi.py::test_group_peer_access[devs01]" in ids
    assert "tests/test_gpu_multi.py::test_bench_nccl_world_n[world8]" in ids


def test_no_skip_marks_with_several_devices(monkeypatch):
    monkeypatch.setenv("NKV_TEST_DEVICE_COUNT", "8")
    sys.path.insert(0, ROOT)
    from tests import test_gpu_multi as m
    for params in (m.device_sets(8), m.mixed_sets(8), m.world_sizes(8), m.device_sets(2), m.world_sizes(2)):
        assert params and all(not p.marks for p in params)
    assert [p.values[0] for p in m.device_sets(8)] == [list(range(8)), [0, 1]]
    assert [p.values[0] for p in m.world_sizes(8)] == [8]
    # one device: g = 1 runs (RCCL over one device), the rest is skipped
    assert [p.values[0] for p in m.device_sets(1)] == [[0]] and not m.device_sets(1)[0].marks
    assert all(p.marks for p in m.mixed_sets(1) + m.world_sizes(1))
