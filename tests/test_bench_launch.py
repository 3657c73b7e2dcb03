"""bench.py --gpus N without torchrun (bench.self_launch): N rank processes with RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1, rank 0's JSON line
carries n_gpus == N and every rank's topology (gloo on the CPU here; the GPU form with
two self-launched ranks on one card is tests/test_gpu_bench_rehearsal.py). A launcher
whose WORLD_SIZE disagrees with --gpus is an error, raised before any GPU call."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_gathers_every_rank(capfd, n):
    import bench
    rc = bench.self_launch(n, ["--gpus", str(n)], script=os.path.join(ROOT, "tests", "helpers", "launch_probe.py"),
                           timeout=120)
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    lines = [json.loads(v) for v in out if v.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == n and line["world"]["size"] == n and line["world"]["backend"] == "gloo"
    assert [r["rank"] for r in line["world"]["ranks"]] == list(range(n))
    assert [r["local_rank"] for r in line["world"]["ranks"]] == list(range(n))
    assert line["max_over_ranks"] == float(n)
    assert line["argv"] == ["--gpus", str(n)]


def test_self_launch_failing_rank_fails_the_job():
    import bench
    rc = bench.self_launch(2, [], script=os.path.join(ROOT, "tests", "helpers", "no_such_script.py"), timeout=60)
    assert rc != 0


def test_world_size_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr
