"""One HIP runtime per process (deepfmkit_amd._lib._bind_runtime), checked on the
CPU in fresh child interpreters (no GPU call is made: only which runtime files get mapped).

- default: the library binds to PyTorch's runtime file WITHOUT importing torch, and a later
  `import torch` maps no second libamdhip64 / libhsa-runtime64;
- DFMI_HIP_RUNTIME=system: the library binds to /opt/rocm's runtime and torch is not touched;
- torch imported first: the library binds to the runtime torch already mapped.
(Loaded first without this, the process mapped both runtimes: the round-4 symptom.)"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
sys.path.insert(0, {root!r})
def maps(p):
    with open('/proc/self/maps') as f:
        return sorted({{l.split()[-1] for l in f if p in l and '/' in l}})
if {torch_first}:
    import torch
from deepfmkit_amd import _lib
_lib.load()
out = {{'torch_imported_by_load': 'torch' in sys.modules and not {torch_first}, 'runtime': _lib.RUNTIME,
       'hip_after_load': maps('libamdhip64')}}
if {import_after}:
    import torch
out['hip_final'] = maps('libamdhip64')
out['hsa_final'] = maps('libhsa-runtime64')
print(json.dumps(out))
"""


def _child(torch_first=False, import_after=True, **env):
    e = dict(os.environ)
    e.update(env)
    src = CHILD.format(root=ROOT, torch_first=torch_first, import_after=import_after)
    p = subprocess.run([sys.executable, "-c", src], capture_output=True, text=True, timeout=300, env=e)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def torch_hip():
    from deepfmkit_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libdfmi.so not built")
    p = _lib._torch_hip_runtime()
    if p is None:
        pytest.skip("no ROCm PyTorch")
    return p


def test_default_binds_torch_runtime_without_importing_torch(torch_hip):
    r = _child(DFMI_HIP_RUNTIME="")
    assert r["torch_imported_by_load"] is False
    assert r["runtime"] == torch_hip
    assert r["hip_after_load"] == [os.path.realpath(torch_hip)] or r["hip_after_load"] == [torch_hip]
    assert len(r["hip_final"]) == 1 and len(r["hsa_final"]) == 1, r


def test_system_runtime_when_asked(torch_hip):
    r = _child(import_after=False, DFMI_HIP_RUNTIME="system")
    assert r["runtime"] is None
    assert len(r["hip_final"]) == 1 and r["hip_final"][0].startswith("/opt/rocm"), r


def test_torch_first_shares_its_runtime(torch_hip):
    r = _child(torch_first=True, import_after=False, DFMI_HIP_RUNTIME="")
    assert r["runtime"] == torch_hip
    assert len(r["hip_final"]) == 1 and len(r["hsa_final"]) == 1, r


def test_soname_check_reads_the_elf_dynamic_section(torch_hip):
    """The preload happens only when torch's runtime carries the soname libdfmi.so needs
    (_lib._elf_dynamic_strings: DT_SONAME / DT_NEEDED from the section headers)."""
    from deepfmkit_amd import _lib
    need = [n for n in _lib._elf_dynamic_strings(_lib.LIB_PATH, 1) if n.startswith("libamdhip64")]
    assert need == ["libamdhip64.so.7"]
    assert _lib._elf_dynamic_strings(torch_hip, 14) == need
    assert _lib._elf_dynamic_strings(__file__, 14) == []  # not an ELF file


def test_mismatched_torch_runtime_is_not_preloaded(torch_hip, tmp_path, monkeypatch):
    """A torch whose runtime has another soname (e.g. a ROCm 6 build): no preload, a warning,
    the system runtime."""
    import warnings
    from deepfmkit_amd import _lib
    fake = tmp_path / "libamdhip64.so"
    fake.write_bytes(b"not an ELF")
    monkeypatch.setattr(_lib, "_torch_hip_runtime", lambda: str(fake))
    monkeypatch.setitem(os.environ, "DFMI_HIP_RUNTIME", "")
    monkeypatch.delitem(sys.modules, "torch", raising=False)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert _lib._bind_runtime() is None
    assert any("not the one libdfmi.so needs" in str(x.message) for x in w)
