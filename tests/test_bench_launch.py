"""bench.py --gpus N without an external launcher: the parent starts N ranks
itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1, child
processes, no exec), they rendezvous (gloo here: the launcher self-test stub
runs no GPU work) and rank 0 alone prints the JSON line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, tmp):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                           "--launcher-selftest", str(tmp)], env=env, capture_output=True,
                          text=True, timeout=180)


def test_self_launch_two_ranks(tmp_path):
    r = _run(2, tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]   # (gloo logs to stdout)
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rccl_world"] == 2 and out["sum_ranks"] == 3.0
    # the per-rank diagnostics bench.py writes at world > 1, gathered over gloo
    rk = out["ranks"]
    assert rk["world"] == 2 and rk["pace_rank"] == 1
    assert rk["fir"] == {"min": 1.0, "max": 2.0, "max_rank": 1}
    assert rk["right_halo_wait"]["max"] == 0.1 and rk["left_halo_wait"]["max"] == 0.0
    assert rk["ms_per_step"]["max"] == 11.0
    assert [r["ms_per_step"] for r in rk["per_rank"]] == [10.0, 11.0]
    for k in ("fir", "psd", "xcorr", "refine", "left_halo_wait", "right_halo_wait", "gather_wait"):
        assert set(rk[k]) == {"min", "max", "max_rank"}
    envs = [json.load(open(tmp_path / f"rank{k}.json")) for k in range(2)]
    assert [e["RANK"] for e in envs] == ["0", "1"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1"]
    assert {e["WORLD_SIZE"] for e in envs} == {"2"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_self_launch_failure_propagates(tmp_path):
    """A rank that fails (here: an unwritable report dir) makes the parent exit
    non-zero instead of hanging on the collective."""
    r = _run(2, tmp_path / "missing" / "dir")
    assert r.returncode != 0


def test_launcher_stops_children_on_sigterm(tmp_path):
    """SIGTERM to the launcher stops its rank processes too (nothing that may
    hold a GPU outlives it)."""
    import signal
    import time
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env["VSIG_SELFTEST_HANG"] = "1"
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--launcher-selftest", str(tmp_path)], env=env,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        deadline = time.time() + 120
        while time.time() < deadline and not all((tmp_path / f"rank{k}.json").exists()
                                                  for k in range(2)):
            time.sleep(0.2)
        time.sleep(0.5)
        pids = [json.load(open(tmp_path / f"rank{k}.json"))["pid"] for k in range(2)]
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) != 0
        for pid in pids:
            for _ in range(100):
                try:
                    os.kill(pid, 0)
                except ProcessLookupError:
                    break
                time.sleep(0.1)
            else:
                raise AssertionError(f"rank process {pid} still alive")
    finally:
        if p.poll() is None:
            p.kill()
