"""the reference-side ctypes binding a DeepFMKit maintainer would
add (fitters_hip.py next to fitters.py, one more fitter_map entry, core.py:452-459) is
executed as written, so the documented boundary cannot drift from include/dfmi.h.

The code blocks are extracted from INTEGRATION.md and imported as the module
`<shim>.fitters_hip` of a stand-in package whose `fit` and `fitters` modules are
deepfmkit_amd's (the reference never travels to the GPU box); only the library path
placeholder is substituted.
- CPU: the binding's ctypes structures have the C layouts (field offsets of
  deepfmkit_amd._lib's mirrors of dfmi_lm_config / dfmi_wdfmi_config) and the
  argtypes cover every C parameter of dfmi_nls_record / dfmi_wdfmi_fit.
- GPU: HipNLSFitter on every golden record in seq / c1 / par4 modes against the
  reference's own outputs (tests/golden/records.npz), at the parity tolerances."""
import os
import re
import sys
import types

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = "dfmk_binding_shim"


def _python_blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec_b = text[text.index("## B."):text.index("## C.")]
    sec_c = text[text.index("## C."):]
    grab = lambda s: re.findall(r"```python\n(.*?)```", s, flags=re.S)  # noqa: E731
    return grab(sec_b), grab(sec_c)


def _binding_module():
    """Import the documented fitters_hip.py (§B block 1 + §C block 1) into a stand-in
    package; returns the module."""
    if f"{SHIM}.fitters_hip" in sys.modules:
        return sys.modules[f"{SHIM}.fitters_hip"]
    import deepfmkit_amd.fit as dfit
    import deepfmkit_amd.fitters as dfitters
    from deepfmkit_amd import _lib
    b, c = _python_blocks()
    src = b[0] + "\n" + c[0]
    assert '"/path/to/deepfmkit_amd/libdfmi.so"' in src
    src = src.replace('"/path/to/deepfmkit_amd/libdfmi.so"', repr(_lib.LIB_PATH))
    pkg = types.ModuleType(SHIM)
    pkg.__path__ = []
    pkg.fit, pkg.fitters = dfit, dfitters
    sys.modules[SHIM] = pkg
    sys.modules[f"{SHIM}.fit"] = dfit
    sys.modules[f"{SHIM}.fitters"] = dfitters
    mod = types.ModuleType(f"{SHIM}.fitters_hip")
    mod.__package__ = SHIM
    sys.modules[mod.__name__] = mod
    exec(compile(src, "INTEGRATION.md:fitters_hip.py", "exec"), mod.__dict__)
    return mod


def _offsets(st):
    return [(name, getattr(st, name).offset, getattr(st, name).size) for name, _ in st._fields_]


def test_binding_structs_match_the_c_layouts():
    from deepfmkit_amd import _lib
    m = _binding_module()
    assert _offsets(m._Cfg) == _offsets(_lib.LMConfig)
    import ctypes
    assert ctypes.sizeof(m._Cfg) == ctypes.sizeof(_lib.LMConfig)
    assert _offsets(m._WCfg) == _offsets(_lib.WdfmiConfig)
    assert ctypes.sizeof(m._WCfg) == ctypes.sizeof(_lib.WdfmiConfig)
    # one argtype per C parameter (include/dfmi.h)
    assert len(m._lib.dfmi_nls_record.argtypes) == 16
    assert len(m._lib.dfmi_wdfmi_fit.argtypes) == 12


def test_fitter_map_entry_names_the_binding():
    b, _ = _python_blocks()
    assert "from .fitters_hip import HipNLSFitter" in b[1]
    assert "'nls_hip': HipNLSFitter" in b[1]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["seq", "c1", "par4"])
def test_binding_fits_golden_records(manifest, records_npz, mode):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from conftest import compare_fit, make_record, record_tol
    m = _binding_module()
    n_done = 0
    for e in manifest["records"]:
        if e["name"] == "ragged_tail":
            continue
        key = f"{e['name']}_{mode}_amp"
        if key not in records_npz.files:
            continue
        raw = make_record(e).raws[e["name"]]
        kw = dict(ndata=e["ndata"], init_m=e["init_m"])
        fitter = m.HipNLSFitter({"n": e["n"]})
        if mode == "seq":
            df = fitter.fit(raw, parallel=False, **kw)
        elif mode == "c1":
            df = fitter.fit(raw, parallel=True, **kw)
        else:
            df = fitter.fit(raw, parallel=True, n_cores=4, **kw)
        assert list(df.columns) == ["amp", "m", "phi", "psi", "dc", "ssq", "fitok"]
        ref = {k: records_npz[f"{e['name']}_{mode}_{k}"] for k in ("amp", "m", "phi", "psi", "dc", "ssq", "fitok")}
        ours = {k: df[k].to_numpy() for k in ref}
        compare_fit(ours, ref, tol=record_tol(e["ndata"], records_npz[f"{e['name']}_qi"], ref))
        n_done += 1
    assert n_done >= 5
