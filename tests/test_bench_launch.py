"""CPU: bench.py's --gpus handling (one process per GPU, the driver's contract).

`python bench.py --gpus N` without a launcher must start N ranks through
torch.distributed.run (a child process, before any GPU call) instead of
silently measuring one GPU; under a launcher WORLD_SIZE must equal N.  The
per-step root all-gather (RootGather) is pipelined over two tree buffers.
"""
import json
import os
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _args(gpus):
    return types.SimpleNamespace(gpus=gpus)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


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
    cmd = bench.launcher_cmd([], 2, _free_port())
    cmd[cmd.index(os.path.abspath(bench.__file__))] = str(script)
    assert subprocess.call(cmd, timeout=120) == 0
    assert sorted(os.listdir(out)) == ["0", "1"]
    assert all((out / r).read_text() == "2" for r in ("0", "1"))


def _gather_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rg = bench.RootGather(torch.zeros(100, dtype=torch.uint8), torch.zeros(world * 20, dtype=torch.uint8), dist)
    seen = []
    for i in range(7):
        buf = rg.begin()
        if i >= 2:  # begin() waited for gather i - 2: its output is final until end()
            seen.append(rg.outs[i % 2].tolist())
        buf[-20:] = (rank * 16 + i) % 256  # this step's "root"
        rg.end(buf)
    rg.drain()
    seen += [rg.outs[5 % 2].tolist(), rg.last_roots().tolist()]
    q.put((rank, seen))
    dist.destroy_process_group()


def test_root_gather_pipeline_world2():
    """RootGather over gloo, world size 2: every step's gathered roots are every
    rank's root of that step, though step i + 1 runs while gather i is in flight."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    # step i's gathered roots: rank 0's i, then rank 1's 16 + i
    want = [[i] * 20 + [16 + i] * 20 for i in range(7)]
    assert res[0] == want and res[1] == want


@pytest.mark.gpu
def test_rccl_root_gather_on_gpu():
    """The N > 1 code path on hardware, at world size 1 (the GPU box has one
    device): torch.distributed.run starts the rank, which joins the nccl (RCCL)
    group bound to its LOCAL_RANK device and all-gathers every step's root; the
    gathered slot must hold the rank's own root and the root must match the oracle."""
    import json
    import subprocess
    cmd = bench.launcher_cmd(["--gpus", "1", "--dist", "--leaves", "65536", "--steps", "4", "--warmup", "1",
                              "--preroll-s", "0", "--no-cpu-baseline", "--verify"], 1, _free_port())
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["steps"] == 4
    assert line["root_gather_ok"] is True
    assert line["verified_vs_oracle"] is True


def _batched_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nodes = torch.zeros(100, dtype=torch.uint8)
    rg = bench.BatchedRootGather(nodes, world, dist, cap=3)
    seen = []
    for i in range(7):  # cap 3: drains itself before the 4th and 7th slot
        buf = rg.begin()
        buf[-20:] = (rank * 16 + i) % 256
        rg.end(buf)
        if i in (2, 5):
            seen.append(None if rg.last is None else rg.last_roots().tolist())
    rg.drain()
    seen.append(rg.last_roots().tolist())
    q.put((rank, seen, rg.k))
    dist.destroy_process_group()


def test_batched_root_gather_world2():
    """BatchedRootGather over gloo, world size 2: the roots of every step are
    kept and gathered in one call (or one per cap slots); last_roots() is every
    rank's root of the last step gathered."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batched_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (seen, k) for r, seen, k in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        seen, k = res[r]
        assert k == 0
        # after step 2 nothing was gathered yet; step 5's check sees the drain
        # before slot 4 (steps 0-2); the final drain has step 6
        assert seen[0] is None
        assert seen[1] == [2] * 20 + [18] * 20
        assert seen[2] == [6] * 20 + [22] * 20


def _preroll_worker(rank, world, port, q):
    import time as _t
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    count = [0]

    def step():  # rank 1 steps three times slower
        _t.sleep(0.002 * (1 + 2 * rank))
        count[0] += 1

    t0 = _t.perf_counter()
    n = bench.preroll(step, lambda: None, lambda: None, 0.1, dist, lambda v: torch.tensor([v], dtype=torch.int32))
    q.put((rank, n, count[0], _t.perf_counter() - t0))
    dist.destroy_process_group()


def test_preroll_same_step_count_on_every_rank():
    """The time-based pre-roll must run the same number of steps on every rank
    (collectives inside a step are matched by order): gloo world 2, one rank
    three times slower; both stop together, after each ran >= 0.1 s."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_preroll_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (n, c, dt) for r, n, c, dt in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    assert res[0][0] == res[1][0] == res[0][1] == res[1][1]
    assert res[0][0] % 8 == 0 and min(res[0][2], res[1][2]) >= 0.1


def test_every_option_flag_reaches_the_context(monkeypatch):
    """bench.set_options maps each override flag to its NKV_OPT_* key (no GPU:
    a recording stand-in for the context)."""
    from nakevaleng_amd import _lib
    monkeypatch.setattr(sys, "argv", ["bench.py", "--leaf-load", "11", "--queue-split", "8", "--queue-waves", "2",
                                      "--records-fused", "0", "--bucket", "1", "--table-lanes", "3"])
    args = bench.parse()

    class Rec:
        def __init__(self):
            self.opts = {}

        def set_option(self, k, v):
            self.opts[k] = v
    r = Rec()
    bench.set_options(args, _lib, r)
    assert r.opts == {_lib.NKV_OPT_LEAF_LOAD: 11, _lib.NKV_OPT_QUEUE_SPLIT: 8, _lib.NKV_OPT_QUEUE_WAVES: 2,
                      _lib.NKV_OPT_RECORDS_FUSED: 0, _lib.NKV_OPT_BUCKET: 1, _lib.NKV_OPT_TABLE_LANES: 3}
    for cfg in ("sstable4k", "mixed", "records", "records_verify", "one_tree", "runs4", "api_flush"):
        monkeypatch.setattr(sys, "argv", ["bench.py", "--config", cfg])
        assert bench.parse().config == cfg


def test_valu_ceiling_prices_each_kernel_at_its_own_count():
    """records / records_verify are priced at their kernels' PMC counts
    (profiles/r03_records_pmc.json), every other config at the leaf kernel's."""
    assert bench.valu_kind("records_verify") == "verify"
    assert bench.valu_kind("records") == "records"
    for c in ("cfg2", "mixed", "runs4", "one_tree"):
        assert bench.valu_kind(c) == "leaf"
    assert bench.valu_ceiling(None, "leaf") is None
    # 1024 SIMDs at 2.2 GHz, one VALU per 4 cycles, 620.1 per 4 KiB wave-block
    assert abs(bench.valu_ceiling(2200.0, "leaf") - 1024 * 2.2e9 / (620.1 * 4) * 4096 / 1e9) < 1e-6
    assert bench.valu_ceiling(2200.0, "verify") < bench.valu_ceiling(2200.0, "records") < bench.valu_ceiling(2200.0, "leaf")


# ---------------------------------------------------------------------------
# round 4: the line verifies every rank against committed
# roots, carries the CPU baseline at every N, and merges the one-process C-ABI
# group runs (fresh child processes) as sub-records.

def test_merged_line_shape(monkeypatch, capsys):
    """main() on rank 0: the ranks' line + capi_group + capi_one_tree + the CPU
    baseline, one JSON line (stand-ins for the GPU run and the children)."""
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "1", "--steps", "3", "--warmup", "1"])
    base = {"metric": "m", "value": 1.0, "n_gpus": 1, "verified_vs_oracle": True,
            "verified_ranks": [True], "cpu_baseline": None}
    monkeypatch.setattr(bench, "run_ranks", lambda args, T: dict(base))
    calls = []

    def fake_child(args, world, extra, timeout, run=None):
        calls.append((world, tuple(extra)))
        return {"value": 2.0, "verified_vs_oracle": True, "n_gpus": world}
    monkeypatch.setattr(bench, "capi_child", fake_child)
    subs = []

    def fake_sub(args, config, timeout, run=None):
        subs.append(config)
        return {"value": 3.0 if config == "mixed" else 4.0, "verified_vs_oracle": True,
                "roofline": {"frac": 0.4}, "cpu_baseline": {"value": 20.0, "best": "all_cores_openssl"}}
    monkeypatch.setattr(bench, "sub_child", fake_sub)
    monkeypatch.setattr(bench, "cpu_baseline", lambda a: {"value": 1.25, "unit": "GiB/s", "cores": 1,
                                                           "kind": "port", "port_1core": {"value": 0.5},
                                                           "sample": f"{a.leaves} x {a.value_bytes}"})
    bench.main()
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["verified_vs_oracle"] is True and line["verified_ranks"] == [True]
    assert line["capi_group"]["value"] == 2.0 and line["capi_one_tree"]["verified_vs_oracle"] is True
    assert line["cpu_baseline"]["cores"] == 1 and line["cpu_baseline"]["sample"] == f"{1 << 20} x 4096"
    assert line["vs_cpu_best"] == 0.8 and line["vs_cpu_port_1core"] == 2.0
    assert calls == [(1, ()), (1, ("--config", "one_tree", "--tables", "1")),
                     (1, ("--leaves", str(8 << 20), "--tables", "1"))]
    assert line["capi_config4"]["n_gpus"] == 1
    # configs[2] and the records form of configs[1] as
    # fresh-child sub-records, each with its own roofline and CPU baseline;
    # the compaction read (every Crc checked) and
    # the host-inclusive flush as well
    assert subs == ["mixed", "records", "records_verify", "api_flush"]
    assert line["config2_mixed"]["value"] == 3.0 and line["config1_records"]["value"] == 4.0
    for k in ("config2_mixed", "config1_records", "config1_records_verify", "api_flush"):
        assert line[k]["verified_vs_oracle"] is True and "roofline" in line[k] and "cpu_baseline" in line[k]


def test_merged_line_at_n_gpus_keeps_cpu_baseline(monkeypatch, capsys):
    """Under the launcher (N = 8, rank 0) the CPU baseline is still measured,
    and runs4 gets the group sub-record but no one-tree run."""
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--config", "runs4", "--no-capi"])
    monkeypatch.setattr(bench, "run_ranks", lambda args, T: {"n_gpus": 8, "value": 8.0})
    monkeypatch.setattr(bench, "capi_child", lambda *a, **k: pytest.fail("--no-capi"))
    monkeypatch.setattr(bench, "cpu_baseline", lambda a: {"value": 1.0, "cores": 1, "port_1core": {"value": 1.0}})
    monkeypatch.setattr(bench, "sub_child", lambda *a, **k: pytest.fail("sub-configs are N = 1 only"))
    bench.main()
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["cpu_baseline"]["value"] == 1.0 and "capi_group" not in line
    assert "config2_mixed" not in line and line["vs_cpu_best"] == 8.0


def test_other_ranks_print_nothing(monkeypatch, capsys):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.setattr(bench, "run_ranks", lambda args, T: None)
    monkeypatch.setattr(bench, "capi_child", lambda *a, **k: pytest.fail("only rank 0"))
    bench.main()
    assert capsys.readouterr().out == ""


def test_capi_child_command_env_and_errors(monkeypatch):
    """The group child: this run's flags + --backend capi --gpus N, outside the
    launcher's process group (no WORLD_SIZE / RANK / MASTER_*), its line's keys
    kept; a failing or hung child gives {"error": ...}, never an exception."""
    import subprocess
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "7"])
    for k, v in (("WORLD_SIZE", "4"), ("RANK", "0"), ("LOCAL_RANK", "0"), ("MASTER_PORT", "1234")):
        monkeypatch.setenv(k, v)
    args = bench.parse(["--gpus", "4", "--steps", "7"])
    seen = {}

    class P:
        returncode = 0
        stdout = "noise\n" + json.dumps({"value": 9.5, "n_gpus": 4, "root_gather_ok": True,
                                         "verified_vs_oracle": True, "verified_members": [True] * 4,
                                         "config": {"parallelism": "4 tables"}, "roofline": {"frac": 0.44}}) + "\n"

    def run(cmd, **kw):
        seen["cmd"], seen["env"] = cmd, kw["env"]
        return P()
    sub = bench.capi_child(args, 4, ["--config", "one_tree", "--tables", "1"], 60, run=run)
    cmd = seen["cmd"]
    assert cmd[1] == os.path.abspath(bench.__file__)
    assert cmd[cmd.index("--backend") + 1] == "capi"
    assert cmd[len(cmd) - 1 - cmd[::-1].index("--gpus") + 1] == "4"  # the last --gpus wins
    assert cmd[len(cmd) - 1 - cmd[::-1].index("--config") + 1] == "one_tree"
    assert not any(k in seen["env"] for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"))
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert sub["value"] == 9.5 and sub["verified_members"] == [True] * 4 and sub["roofline_frac"] == 0.44
    assert sub["parallelism"] == "4 tables"
    # the child's command line parses to the group backend over 4 GPUs
    child = bench.parse(cmd[2:])
    assert child.backend == "capi" and child.gpus == 4 and child.config == "one_tree" and child.steps == 7

    class Bad:
        returncode = 1
        stdout = ""
    assert "error" in bench.capi_child(args, 4, [], 60, run=lambda cmd, **kw: Bad())

    def hang(cmd, **kw):
        raise subprocess.TimeoutExpired(cmd, 60)
    assert "timed out" in bench.capi_child(args, 4, [], 60, run=hang)["error"]


def test_verdict_codes():
    assert bench.verdict([1, 1, 1]) is True
    assert bench.verdict([1, 0, 1]) is False
    assert bench.verdict([1, -1]) is None
    assert bench.verdict([0, -1]) is False
    assert bench.verdict([]) is None


def test_expected_roots_cover_the_driver_shapes():
    """The committed roots cover configs[1] on ranks 0-7 (tables 0-3) and the
    one tree over 1-8 ranks; other shapes fall back to --verify."""
    for r in range(8):
        assert len(bench.expected_roots("sstable4k", 1 << 20, 4096, r, 1)) == 1
        assert len(bench.expected_roots("runs4", 1 << 20, 4096, r, 4)) == 4
    for N in range(1, 9):
        assert len(bench.expected_one_tree(1 << 20, 4096, N)) == 40
    assert bench.expected_roots("sstable4k", 1 << 20, 4096, 8, 1) is None
    # the records and mixed configs (rank r's table, one per step)
    assert len(bench.expected_roots("records_verify", 1 << 20, 4096, 3, 1, key_bytes=16)) == 1
    assert bench.expected_roots("records", 1 << 20, 4096, 3, 1, key_bytes=20) is None
    assert len(bench.expected_roots("mixed", None, None, 5, 1, mixed_bytes=4 << 30)) == 1
    assert bench.expected_roots("mixed", None, None, 5, 1, mixed_bytes=1 << 30) is None
    assert bench.expected_roots("mixed", None, None, 5, 2) is None
    assert bench.expected_roots("sstable4k", 65536, 4096, 0, 1) is None
    assert bench.expected_one_tree(65536, 4096, 2) is None


def _verify_worker(rank, world, port, bad_rank, q):
    import torch.distributed as dist
    from oracle import oracle_c as oc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # this rank's table at configs[0]'s size, built by the oracle standing in
    # for the device, seeded as bench.build_tables seeds rank r's table
    data = oc.splitmix64_bytes(1024 * 1024, bench.SEED + rank)
    root = oc.tree_from_digests(oc.leaf_hashes_strided(data, 1024, 1024, 1024))[-1].tobytes().hex()
    if rank == bad_rank:
        root = ("0" if root[0] != "0" else "1") + root[1:]
    want = bench.expected_roots("sstable4k", 1024, 1024, rank, 1)
    code = -1 if want is None else int([root] == want)
    codes = bench.rank_codes(dist, world, rank, code, "cpu")
    q.put((rank, codes, bench.verdict(codes)))
    dist.destroy_process_group()


@pytest.mark.parametrize("bad_rank", [-1, 1])
def test_rank_verification_world2(oracle, bad_rank):
    """gloo world 2: each rank checks its own root against the committed roots
    and every rank learns every rank's result; one wrong rank fails the line."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_verify_worker, args=(r, 2, port, bad_rank, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (codes, v) for r, codes, v in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    want_codes = [1, 1] if bad_rank < 0 else [1, 0]
    assert res[0] == res[1] == (want_codes, bad_rank < 0)


def test_sub_child_command_env_and_errors(monkeypatch):
    """The sub-config child: this run's flags + --config C --gpus 1 --no-capi
    --no-subconfigs (no recursion), outside any launcher; its line's keys kept;
    a failing or hung child gives {"error": ...}."""
    import subprocess
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "7", "--warmup", "2"])
    monkeypatch.setenv("WORLD_SIZE", "1")
    args = bench.parse(["--steps", "7", "--warmup", "2"])
    seen = {}

    class P:
        returncode = 0
        stdout = json.dumps({"value": 2700.0, "n_gpus": 1, "roofline": {"frac": 0.37, "chain_frac": 0.9},
                             "verified_vs_oracle": True, "cpu_baseline": {"value": 25.0},
                             "vs_cpu_best": 108.0, "config": {"workload": "mixed"}, "other": 1}) + "\n"

    def run(cmd, **kw):
        seen["cmd"], seen["env"] = cmd, kw["env"]
        return P()
    sub = bench.sub_child(args, "mixed", 100, run=run)
    cmd = seen["cmd"]
    child = bench.parse(cmd[2:])
    assert child.config == "mixed" and child.gpus == 1 and child.no_capi and child.no_subconfigs
    assert child.steps == 7 and child.warmup == 2 and child.tables == 1
    assert "WORLD_SIZE" not in seen["env"] and seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert sub["value"] == 2700.0 and sub["roofline"]["chain_frac"] == 0.9 and sub["cpu_baseline"]["value"] == 25.0
    assert sub["workload"] == "mixed" and "other" not in sub

    class Bad:
        returncode = 1
        stdout = ""
    assert "error" in bench.sub_child(args, "records", 100, run=lambda cmd, **kw: Bad())

    def hang(cmd, **kw):
        raise subprocess.TimeoutExpired(cmd, 100)
    assert "timed out" in bench.sub_child(args, "records", 100, run=hang)["error"]


def test_cpu_baseline_variants_small(oracle, monkeypatch):
    """cpu_baseline times the four SURVEY 8(d) variants on the same sample (the
    portable port and OpenSSL, one core and every core), they agree on the root,
    and `value` is the strongest; for every config kind."""
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    for argv, n in ((["--leaves", "64", "--value-bytes", "4096", "--cpu-sample-leaves", "64"], 64),
                    (["--config", "records", "--leaves", "48", "--cpu-sample-leaves", "48"], 48),
                    (["--config", "mixed", "--mixed-bytes", str(1 << 20)], None)):
        a = bench.parse(argv)
        cb = bench.cpu_baseline(a)
        vals = {k: cb[k]["value"] for k, _, _ in bench.CPU_VARIANTS}
        assert cb["value"] == max(vals.values()) and cb["best"] in vals
        assert cb["port_1core"]["cores"] == 1 and cb["all_cores_openssl"]["cores"] == 2
        assert cb["cpu_model"] and cb["host_threads"] == 2
        s = bench.cpu_sample(a)
        if n:
            assert s["n"] == n
        want = (oracle.tree_from_digests(oracle.leaf_hashes_strided(s["data"], s["stride"], s["L"], s["n"]))
                if "stride" in s else oracle.tree_from_digests(oracle.leaf_hashes(s["data"], s["off"], s["lens"])))
        assert cb["root"] == want[-1].tobytes().hex()


def test_records_cpu_sample_layout():
    """The records CPU sample hashes each record's Value where the GPU line's
    table has it: record r at r x record size, its Value at +30 + KeySize
    (record.go:191-199), ValueSize = record size - 30 - KeySize."""
    a = bench.parse(["--config", "records", "--leaves", "1024", "--cpu-sample-leaves", "1024",
                     "--value-bytes", "1024"])
    s = bench.cpu_sample(a)
    assert s["n"] == 1024 and int(s["lens"][0]) == 1024 - 30 - 16 and int(s["off"][1]) == 1024 + 46
