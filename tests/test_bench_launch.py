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


def test_scaling_anchor_names_rank0_workload_at_8(capfd):
    """The N = 1 line's scaling_anchor (bench.scaling_anchor) fits config 4's shard of rank 0 at
    N = 8: eight gloo ranks launched like `bench.py --gpus 8`, rank 0's workload string equals
    the anchor's, and it is the 10M-segment record's 1/8."""
    import bench
    rc = bench.self_launch(8, ["--gpus", "8"], script=os.path.join(ROOT, "tests", "helpers", "launch_probe.py"),
                           timeout=180)
    assert rc == 0
    lines = [json.loads(v) for v in capfd.readouterr().out.strip().splitlines() if v.startswith("{")]
    assert len(lines) == 1 and lines[0]["n_gpus"] == 8
    anchor = bench.plan_workload(bench.ANCHOR_WORLD)
    assert lines[0]["config"]["workload"] == anchor["workload"]
    assert anchor["nseg"] * 8 == lines[0]["config"]["record_segments"] == bench.CONFIG4_SEGMENTS
    assert bench.plan_workload(1)["workload"].startswith("config2: 100000 segments/GPU")


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


def test_rank_late_for_rendezvous_fails_fast_and_is_named(capfd):
    """A rank that never reaches the rendezvous in time (rank 1 sleeps 60 s before joining,
    the rendezvous timeout is 5 s): rank 0's init_process_group raises, the launcher takes
    the job down, exits non-zero well inside the sleep and names rank 1 on stderr."""
    import time

    import bench
    t0 = time.monotonic()
    rc = bench.self_launch(2, [], script=os.path.join(ROOT, "tests", "helpers", "launch_probe.py"), timeout=120,
                           env_extra={"DFMI_RDZV_DELAY": "1:60", "PROBE_RDZV_TIMEOUT": "5"})
    dt = time.monotonic() - t0
    err = capfd.readouterr().err
    assert rc != 0 and dt < 45, (rc, dt)
    assert "never reached the rendezvous: [1]" in err, err[-2000:]


def test_launch_timeout_kills_and_names_the_ranks(capfd):
    """The launcher's own bound: rank 0 stuck before the rendezvous, rank 1 waiting in it
    (rendezvous timeout 120 s), both past the launch timeout of 8 s: killed, exit 124, rank 0
    named as never arriving, both as not having joined."""
    import time

    import bench
    t0 = time.monotonic()
    rc = bench.self_launch(2, [], script=os.path.join(ROOT, "tests", "helpers", "launch_probe.py"), timeout=8,
                           env_extra={"DFMI_RDZV_DELAY": "0:60", "PROBE_RDZV_TIMEOUT": "120"})
    dt = time.monotonic() - t0
    err = capfd.readouterr().err
    assert rc == 124 and dt < 40, (rc, dt)
    assert "launch timeout" in err and "never reached the rendezvous: [0];" in err, err[-2000:]
    assert "did not complete it: [0, 1]" in err, err[-2000:]


def test_launch_timeout_scales_with_the_work():
    import argparse

    import bench
    a = argparse.Namespace(segments=None, steps=100, warmup=10, rdzv_timeout=120.0, no_extra=False)
    t8 = bench.launch_timeout(a, 8)
    a.steps = 1000
    assert bench.launch_timeout(a, 8) > t8 > 600
