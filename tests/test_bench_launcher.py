"""bench.py's N-rank launcher (``python bench.py --gpus N`` without torchrun):
one child per GPU with the torchrun rank environment, worst exit code
returned, stuck peers of a failed rank terminated.  The worker is a stub
script, so no GPU is touched (CPU test)."""
import json
import os
import sys
import textwrap
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def _stub(tmp_path, body):
    p = tmp_path / "stub.py"
    p.write_text(textwrap.dedent(body))
    return [sys.executable, str(p)]


@pytest.mark.parametrize("n", [2, 4, 8])
def test_spawn_sets_rank_environment(tmp_path, n):
    cmd = _stub(tmp_path, f"""
        import json, os
        keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                "FMIDX_BENCH_LAUNCHER", "HSA_ENABLE_IPC_MODE_LEGACY"]
        with open(os.path.join({str(tmp_path)!r}, "rank%s.json" % os.environ["RANK"]), "w") as f:
            json.dump({{k: os.environ.get(k) for k in keys}}, f)
    """)
    assert bench.spawn_ranks(n, cmd) == 0
    envs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(n)]
    assert [int(e["RANK"]) for e in envs] == list(range(n))
    assert [int(e["LOCAL_RANK"]) for e in envs] == list(range(n))
    assert {e["WORLD_SIZE"] for e in envs} == {str(n)}
    assert {e["LOCAL_WORLD_SIZE"] for e in envs} == {str(n)}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1 and int(envs[0]["MASTER_PORT"]) > 0
    assert {e["FMIDX_BENCH_LAUNCHER"] for e in envs} == {"spawn"}
    assert {e["HSA_ENABLE_IPC_MODE_LEGACY"] for e in envs} == {"0"}


def test_spawn_children_rendezvous_over_gloo(tmp_path):
    """The environment is enough for init_process_group's env:// rendezvous:
    two children form a world of 2 and all-reduce (gloo, CPU)."""
    cmd = _stub(tmp_path, f"""
        import os, torch, torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.tensor([int(os.environ["RANK"]) + 1])
        dist.all_reduce(t)
        assert dist.get_world_size() == 2 and int(t) == 3, (dist.get_world_size(), int(t))
        open(os.path.join({str(tmp_path)!r}, "ok%d" % dist.get_rank()), "w").close()
        dist.destroy_process_group()
    """)
    assert bench.spawn_ranks(2, cmd) == 0
    assert (tmp_path / "ok0").exists() and (tmp_path / "ok1").exists()


def test_spawn_failure_terminates_stuck_peers(tmp_path):
    """Rank 1 fails; rank 0 (stuck, as in a collective with a dead peer) is
    terminated after the grace period and the failure code is returned."""
    cmd = _stub(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(600)
    """)
    t0 = time.time()
    rc = bench.spawn_ranks(2, cmd, grace_s=1.0)
    assert rc == 3
    assert time.time() - t0 < 60


def test_bench_refuses_more_gpus_than_visible(tmp_path):
    """`bench.py --gpus N` on a machine with fewer GPUs exits 2 before any
    rank starts (this container has none)."""
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300,
                       env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert r.returncode == 2, r.stderr[-2000:]
    assert "GPU(s) visible" in r.stderr


def test_visible_gpus_from_topology(tmp_path):
    """The launcher's GPU count reads the KFD topology (CPU nodes have gpu_id 0)
    and honours the visibility lists -- no HIP runtime involved."""
    for i, gid in enumerate([0, 1234, 0, 5678, 91011]):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "gpu_id").write_text(f"{gid}\n")
    topo = str(tmp_path)
    assert bench.visible_gpus({}, topo) == 3
    assert bench.visible_gpus({"HIP_VISIBLE_DEVICES": "0,1"}, topo) == 2
    assert bench.visible_gpus({"ROCR_VISIBLE_DEVICES": ""}, topo) == 0
    assert bench.visible_gpus({"CUDA_VISIBLE_DEVICES": "0,1,2,3,4,5"}, topo) == 3
    assert bench.visible_gpus({}, str(tmp_path / "missing")) == 0


def test_launcher_parent_never_calls_torch_cuda(monkeypatch):
    """`bench.py --gpus N` without WORLD_SIZE: the parent counts GPUs and
    spawns the ranks without a single torch.cuda call (any of them could
    initialise HIP in the parent, whose children are then new programs)."""
    import torch

    calls = []

    def boom(name):
        def f(*a, **k):
            calls.append(name)
            raise AssertionError(f"the launcher parent called torch.cuda.{name}")
        return f

    for name in ("device_count", "is_available", "init", "set_device", "current_device", "synchronize",
                 "get_device_properties", "mem_get_info", "_lazy_init"):
        monkeypatch.setattr(torch.cuda, name, boom(name))
    spawned = []
    monkeypatch.setattr(bench, "visible_gpus", lambda *a, **k: 8)
    monkeypatch.setattr(bench, "spawn_ranks", lambda n, cmd, **k: spawned.append((n, cmd)) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 0
    assert not calls
    assert spawned and spawned[0][0] == 4 and spawned[0][1][-4:] == ["--gpus", "4", "--steps", "3"]


def _run_stub(tmp_path, body, timeout=60):
    import subprocess

    head = textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {REPO!r})
        from bench import LegWatchdog
    """)
    cmd = _stub(tmp_path, head + textwrap.dedent(body))
    t0 = time.time()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    return p, time.time() - t0


def test_leg_watchdog_prints_and_fails_when_the_leg_hangs(tmp_path):
    """The N > 1 sharded leg's watchdog (bench.LegWatchdog): a leg that never returns
    (a thread stuck in a collective) ends the process with status 3 (WATCHDOG_EXIT: a
    hang fails the run) right after the expiry callback printed the line."""
    p, dt = _run_stub(tmp_path, """
        def expire():
            print('{"value": 1, "sharded": {"error": "watchdog"}}', flush=True)
        dog = LegWatchdog(0.5, expire)
        time.sleep(30)          # the stuck leg
        print("not reached")
    """)
    assert p.returncode == 3, p.stderr
    assert '"watchdog"' in p.stdout and "not reached" not in p.stdout
    assert dt < 20


def test_leg_watchdog_finish_cancels(tmp_path):
    """A leg that returns in time: finish() cancels the timer, the process goes on and
    the expiry callback never runs."""
    p, _ = _run_stub(tmp_path, """
        def expire():
            print("expired", flush=True)
        dog = LegWatchdog(1.0, expire)
        time.sleep(0.1)
        dog.finish()
        time.sleep(1.5)         # past the timer's deadline
        print("line", flush=True)
    """)
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["line"]


def test_peer_preflight_outcomes(tmp_path, monkeypatch):
    """bench.peer_preflight (the N > 1 sharded leg's cross-device check, run in a child so a GPU
    fault ends only the child): an exact child, a failing child, a crashed child and a hung
    child (killed at the limit) give (True, ...), (False, "exit status 1"), (False, "killed by
    signal ..."), (False, "timed out ..."); the child's rendezvous port is MASTER_PORT + 101 and
    its stdout never reaches the parent's stdout (the JSON line's channel)."""
    import subprocess

    monkeypatch.setenv("MASTER_PORT", "29611")
    ok = _stub(tmp_path, f"""
        import os, sys
        print("chatter on stdout")
        open(os.path.join({str(tmp_path)!r}, "port"), "w").write(os.environ["FMIDX_PREFLIGHT_PORT"])
    """)
    p = subprocess.run([sys.executable, "-c", textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {REPO!r})
        import bench
        print(repr(bench.peer_preflight(cmd={ok!r})))
    """)], capture_output=True, text=True, timeout=120, env=dict(os.environ))
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip().startswith("(True, 'exact"), p.stdout
    assert "chatter on stdout" in p.stderr and "chatter" not in p.stdout
    assert (tmp_path / "port").read_text() == str(29611 + bench.PREFLIGHT_PORT_OFFSET)
    fail = _stub(tmp_path, "import sys; sys.exit(1)")
    assert bench.peer_preflight(cmd=fail)[0] is False
    assert bench.peer_preflight(cmd=fail)[1].startswith("exit status 1")
    crash = _stub(tmp_path, "import os, signal; os.kill(os.getpid(), signal.SIGABRT)")
    r = bench.peer_preflight(cmd=crash)
    assert r[0] is False and r[1].startswith("killed by signal 6"), r
    hang = _stub(tmp_path, "import time; time.sleep(60)")
    t0 = time.time()
    r = bench.peer_preflight(timeout_s=1.0, cmd=hang)
    assert r == (False, "timed out after 1 s") and time.time() - t0 < 20
