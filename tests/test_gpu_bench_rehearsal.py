"""bench.py's N > 1 line in its current form (the driver's multi-GPU scaling run):
two ranks sharing the one GPU of the test box, over gloo (RCCL refuses two ranks on
one device), weak scaling with --segments 20000 per rank. Checks the JSON rank 0
prints: n_gpus, scaling, the all-reduced timings (MAX over ranks), the roofline's
min-over-ranks fraction, and that every segment of the batch fitted with status 0.
(Static shard, no data-path collective: DESIGN.md §6; fitters.py:403-423.)"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_weak_scaling_line(tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2",
               DFMI_DIST_BACKEND="gloo", LOCAL_RANK="0")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "1",
           "--segments", "20000", "--no-cpu-baseline"]
    procs = []
    for rank in (1, 0):
        out = open(tmp_path / f"r{rank}.out", "w")
        err = open(tmp_path / f"r{rank}.err", "w")
        procs.append((rank, subprocess.Popen(cmd, env=dict(env, RANK=str(rank)), stdout=out, stderr=err, cwd=ROOT),
                      out, err))
    rcs = {}
    for rank, p, out, err in procs:
        try:
            rcs[rank] = p.wait(timeout=240)
        finally:
            if p.poll() is None:
                p.kill()
            out.close()
            err.close()
    assert rcs == {0: 0, 1: 0}, (rcs, (tmp_path / "r0.err").read_text()[-2000:], (tmp_path / "r1.err").read_text()[-2000:])
    assert "{" not in (tmp_path / "r1.out").read_text()  # only rank 0 prints the JSON line
    line = json.loads((tmp_path / "r0.out").read_text().strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["steps"] == 5
    assert line["config"]["segments_per_gpu"] == 20000 and line["config"]["parallelism"] == "shard2"
    roof = line["roofline"]
    assert "frac_min_over_ranks" in roof and "avg_launch_ms_max_over_ranks" in roof
    assert 0 < roof["frac_min_over_ranks"] <= roof["frac"] + 1e-12
    assert line["batch_status0_frac"] == 1.0
    assert abs(line["batch_m_mean"] - 6.0) < 1e-3
    assert line["value"] > 0 and "cpu_baseline" not in line and "extra_configs" not in line


def test_bench_self_launch_two_ranks(tmp_path):
    """`python bench.py --gpus 2` with no torchrun: bench.self_launch starts the two rank
    processes itself (gloo, both on this box's one card); rank 0's line says n_gpus 2 and
    lists both ranks' devices."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["DFMI_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "1",
           "--segments", "20000", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [v for v in p.stdout.strip().splitlines() if v.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["world"]["size"] == 2 and line["world"]["backend"] == "gloo"
    assert line["world"]["launcher"] == "bench.py self-launch"
    ranks = line["world"]["ranks"]
    assert [r["rank"] for r in ranks] == [0, 1] and all(r["device"].startswith("cuda:") for r in ranks)
    assert line["batch_status0_frac"] == 1.0 and line["value"] > 0
