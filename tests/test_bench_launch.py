"""CPU: bench.py's --gpus handling (one process per GPU, the driver's contract).

`python bench.py --gpus N` without a launcher must start N ranks through
torch.distributed.run (a child process, before any GPU call) instead of
silently measuring one GPU; under a launcher WORLD_SIZE must equal N.
"""
import os
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _args(gpus):
    return types.SimpleNamespace(gpus=gpus)


def test_single_gpu_runs_in_process(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.ensure_ranks(_args(1), [], run=lambda cmd: pytest.fail("must not spawn")) is None


def test_multi_gpu_spawns_launcher(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = []
    rc = bench.ensure_ranks(_args(8), ["--gpus", "8", "--steps", "5"], run=lambda cmd: seen.append(cmd) or 7)
    assert rc == 7  # the launcher's exit code is the bench's
    (cmd,) = seen
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert any(a.startswith("--master-port=") for a in cmd)
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5"]


def test_launcher_world_must_match(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.ensure_ranks(_args(4), [], run=lambda cmd: pytest.fail("must not spawn")) is None
    assert bench.ensure_ranks(_args(8), [], run=lambda cmd: pytest.fail("must not spawn")) == 2


def test_spawned_ranks_see_their_rank(tmp_path):
    """The real launcher on CPU: two ranks start and each sees WORLD_SIZE=2 and its
    own LOCAL_RANK (a stand-in script, so no GPU is needed)."""
    import subprocess
    script = tmp_path / "probe.py"
    out = tmp_path / "out"
    out.mkdir()
    script.write_text("import os\nopen(os.path.join(%r, os.environ['LOCAL_RANK']), 'w').write("
                      "os.environ['WORLD_SIZE'])\n" % str(out))
    cmd = bench.launcher_cmd([], 2, 29731)
    cmd[cmd.index(os.path.abspath(bench.__file__))] = str(script)
    assert subprocess.call(cmd, timeout=120) == 0
    assert sorted(os.listdir(out)) == ["0", "1"]
    assert all((out / r).read_text() == "2" for r in ("0", "1"))
