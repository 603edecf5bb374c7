"""`bench.py --gpus N` runs N ranks by itself, on the CPU: the launch decision
(argument -> world and per-rank environment; a launcher's WORLD_SIZE that disagrees with --gpus ->
non-zero exit before any GPU call) and the parent's relay of its ranks' output and exit codes."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def bench(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    sys.path.insert(0, ROOT)
    import bench as b
    return b


def test_one_gpu_runs_in_process(bench):
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == ("run", 1)


def test_n_gpus_without_launcher_spawns_n_ranks(bench):
    kind, envs = bench.launch_plan(4, {"PATH": "/usr/bin"}, device_count=8)
    assert kind == "spawn" and len(envs) == 4
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1 and int(envs[0]["MASTER_PORT"]) > 0
    assert {e["HSA_ENABLE_IPC_MODE_LEGACY"] for e in envs} == {"0"}
    assert all(e["PATH"] == "/usr/bin" for e in envs)


def test_launcher_world_size_must_match(bench):
    assert bench.launch_plan(8, {"WORLD_SIZE": "8", "RANK": "3"}) == ("run", 8)
    kind, msg = bench.launch_plan(2, {"WORLD_SIZE": "4"})
    assert kind == "error" and "WORLD_SIZE=4" in msg
    assert bench.launch_plan(0, {})[0] == "error"


def test_rccl_ranks_need_devices_gloo_rehearses(bench):
    assert bench.launch_plan(2, {}, device_count=1)[0] == "error"
    kind, envs = bench.launch_plan(2, {"BENCH_DIST_BACKEND": "gloo"}, device_count=1)
    assert kind == "spawn" and len(envs) == 2


def test_mismatch_exits_nonzero_before_gpu():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 2, out.stderr[-500:]
    assert "must agree" in out.stderr
    assert out.stdout.strip() == ""


def test_spawn_relays_rank0_line_and_worst_exit_code(bench, tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(
        "import json, os, sys\n"
        "r = int(os.environ['RANK'])\n"
        "if r == 0: print(json.dumps({'n_gpus': int(os.environ['WORLD_SIZE']), 'argv': sys.argv[1:]}))\n"
        "sys.exit(int(os.environ.get('FAIL_RANK', '-1')) == r and 3 or 0)\n")
    kind, envs = bench.launch_plan(3, {"BENCH_DIST_BACKEND": "gloo", "PATH": os.environ.get("PATH", "")},
                                   device_count=0)
    assert kind == "spawn"
    child = (f"import sys; sys.path.insert(0, {ROOT!r}); sys.argv = ['bench.py']; import bench, json; "
             f"envs = json.loads(sys.stdin.read()); "
             f"sys.exit(bench.spawn_ranks(envs, ['--gpus', '3'], grace_s=5, script={str(script)!r}))")
    import json
    ok = subprocess.run([sys.executable, "-c", child], input=json.dumps(envs), capture_output=True, text=True,
                        timeout=300)
    assert ok.returncode == 0, ok.stderr[-500:]
    assert json.loads(ok.stdout.strip().splitlines()[-1]) == {"n_gpus": 3, "argv": ["--gpus", "3"]}
    bad_envs = [dict(e, FAIL_RANK="2") for e in envs]
    bad = subprocess.run([sys.executable, "-c", child], input=json.dumps(bad_envs), capture_output=True, text=True,
                         timeout=300)
    assert bad.returncode == 3, bad.stderr[-500:]


def test_watchdog_returns_the_leg_or_prints_and_exits(tmp_path):
    """bench.run_with_watchdog (the N > 1 update leg): a leg that finishes returns its value; one that
    hangs past the timeout runs on_timeout (rank 0's line) and ends the process with code 0."""
    code = (f"import sys, time, json; sys.path.insert(0, {ROOT!r}); sys.argv = ['bench.py']; import bench\n"
            "print(json.dumps({'fast': bench.run_with_watchdog(lambda: 7, 5.0, lambda: print('no'))}), flush=True)\n"
            "bench.run_with_watchdog(lambda: time.sleep(60), 0.5, lambda: print(json.dumps({'timed_out': True})))\n"
            "print('unreachable')\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-500:]
    lines = out.stdout.strip().splitlines()
    assert lines == ['{"fast": 7}', '{"timed_out": true}'], lines
