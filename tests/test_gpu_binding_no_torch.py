"""The C-ABI boundary as the reference's own process would use it:
each case runs in a FRESH child interpreter (subprocess.run([sys.executable, ...]); never a
re-exec of this process) — tests/helpers/boundary_child.py:

  - INTEGRATION.md §B (numpy + ctypes) with torch never imported: the library runs under the
    HIP runtime it links (/opt/rocm/lib/libamdhip64.so.7, checked in /proc/self/maps) and fits
    every golden record in seq / c1 / par4 modes to the reference's outputs;
  - the reference's fork-based callers (fitters.py:421-423, experiments.py:381-384): the
    library loaded without a GPU call, then a 'fork' Pool(2) whose workers each fit a golden
    record with dff.fit(label, n=20, parallel=False) — both with the package's default
    runtime choice and with the system runtime (DFMI_HIP_RUNTIME=system);
  - torch imported AFTER the library initialised the GPU: torch still sees and uses the GPU
    and one HIP runtime is mapped (deepfmkit_amd._lib._bind_runtime)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tests", "helpers", "boundary_child.py")


def _run(what, **env):
    e = dict(os.environ)
    e.update(env)
    p = subprocess.run([sys.executable, CHILD, what], capture_output=True, text=True, timeout=300, env=e, cwd=ROOT)
    assert p.returncode == 0, (p.returncode, p.stdout[-3000:], p.stderr[-5000:])
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)[what]
    print(what, env, json.dumps(res)[:2000])
    return res


def test_integration_binding_without_torch():
    res = _run("binding", DFMI_HIP_RUNTIME="system")
    assert res["torch_imported"] is False
    assert res["hip_runtimes"][0].startswith("/opt/rocm")
    assert res["fits"] >= 15


@pytest.mark.parametrize("runtime", ["default", "system"])
def test_fork_pool_after_load(runtime):
    env = {"DFMI_HIP_RUNTIME": "system"} if runtime == "system" else {"DFMI_HIP_RUNTIME": ""}
    res = _run("fork", **env)
    assert res["torch_imported"] is False
    assert res["parent_before_fork"]["kfd_open"] is False  # no HIP initialisation before the fork
    assert len(res["workers"]) == 4 and all(w["rows"] > 0 for w in res["workers"])


def test_torch_imported_after_library_init():
    res = _run("torch_after", DFMI_HIP_RUNTIME="")
    assert res["torch_cuda_available"] and res["torch_sum"] == 45.0
    assert len(res["hip_runtimes"]) == 1
