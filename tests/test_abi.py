"""The C-ABI library loads and exports every symbol include/dfmi.h declares
(no compute calls: this runs on the CPU-only container)."""
import ctypes
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "dfmi.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dfmi_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("dfmi_demod", "dfmi_lm", "dfmi_nls_record", "dfmi_ekf", "dfmi_last_error", "dfmi_device_count",
              "dfmi_wdfmi_fit"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from deepfmkit_amd import _lib
    lib = _lib.load()
    nm = ctypes.CDLL(_lib.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(nm, s), s
    assert set(declared_symbols()) == set(_lib.SYMBOLS)
    assert lib.dfmi_version().decode().startswith("dfmi")


def test_library_is_gfx950_code_object():
    from deepfmkit_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_default_config_matches_fit_constants():
    """dfmi_lm_config_default == the reference constants fit.py:5-16, 222, 230."""
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    lib = _lib.load()
    c = _lib.LMConfig()
    lib.dfmi_lm_config_default(ctypes.byref(c))
    p = F.lm_config()
    for name, _ in _lib.LMConfig._fields_:
        a, b = getattr(c, name), getattr(p, name)
        if name == "lambdas":
            assert list(a) == list(b)
        else:
            assert a == b, name
    assert c.n_lambda == 8 and list(c.lambdas)[:8] == [0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0]


def test_lm_config_reads_live_module_globals():
    """Overwriting deepfmkit_amd.fit constants (as notebooks/0.0_benchmark cell 1 does
    for the reference) changes what the next engine call receives."""
    from deepfmkit_amd import fit as F
    old = F.MAX_LMA_STEPS
    try:
        F.MAX_LMA_STEPS = 7
        assert F.lm_config().max_lma_steps == 7
    finally:
        F.MAX_LMA_STEPS = old


def test_period_detection_host_function():
    """dfmi_detect_period is pure host code (no GPU): L = f_samp/f_mod when integral."""
    from deepfmkit_amd import _lib
    from deepfmkit_amd.fitters import w0_of
    lib = _lib.load()
    assert lib.dfmi_detect_period(w0_of(1000.0, 200000.0), 4000, 10) == 200
    assert lib.dfmi_detect_period(w0_of(400.0, 30000.0), 1500, 10) == 75
    assert lib.dfmi_detect_period(w0_of(1500.0, 200000.0), 2666, 10) == 400
    assert lib.dfmi_detect_period(w0_of(1000.0, 199999.7), 4000, 10) == 0


def test_no_gpu_here_is_a_loud_error():
    """Without a GPU the engine must fail loudly (no silent CPU fallback)."""
    import pytest
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from deepfmkit_amd import fit as F
    from deepfmkit_amd._lib import DFMIError
    with pytest.raises(DFMIError):
        F.demodulate(np.zeros((2, 400)), 10, w0=2 * np.pi / 200)


def test_wdfmi_argument_errors_before_any_device_work():
    """dfmi_wdfmi_fit validates its arguments on the host (no GPU needed) and, with
    valid arguments but no GPU, fails loudly rather than computing on the CPU."""
    from deepfmkit_amd import _lib
    lib = _lib.load()
    x = np.zeros(8000)
    w = np.zeros(4000)
    out = np.zeros((7, 2))
    ok = np.zeros(2, dtype=np.int32)

    def call(method=1, R=4000, ndata=10, ndata_psi=40, f_samp=200000.0):
        cfg = _lib.WdfmiConfig(method, ndata, ndata_psi, 0, f_samp, 1000.0, 1e9, 0.0, 6e-10, 1.6, 0.0, 0.0)
        return lib.dfmi_wdfmi_fit(_lib.ptr(x), 1, 8000, 2, R, _lib.ptr(w), 0, cfg, _lib.ptr(out), _lib.ptr(ok),
                                  _lib.DFMI_MEM_HOST, None)

    assert call(method=7) == -1
    assert call(R=2) == -1
    assert call(R=20000) == -4
    assert call(method=0, ndata=40) == -4
    assert call(method=2, ndata_psi=80) == -4
    assert call(f_samp=0.0) == -1
    import pytest
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        assert call() == -3  # DFMI_ERR_NODEV


def test_moments_and_ekf_fit_argument_errors():
    """dfmi_record_moments / dfmi_ekf_fit check their arguments on the host; with valid
    arguments and no GPU they fail loudly (no host-side numpy fallback)."""
    from deepfmkit_amd import _lib
    lib = _lib.load()
    x = np.zeros(100)
    m, v = np.zeros(2), np.zeros(2)
    H = _lib.DFMI_MEM_HOST
    assert lib.dfmi_record_moments(_lib.ptr(x), 2, 50, 0, _lib.ptr(m), _lib.ptr(v), H, None) == -1
    assert lib.dfmi_record_moments(_lib.ptr(x), 2, 40, 50, _lib.ptr(m), _lib.ptr(v), H, None) == -1
    assert lib.dfmi_record_moments(_lib.ptr(x), 2, 50, 50, None, _lib.ptr(v), H, None) == -1
    st = np.zeros((1, 5))
    p0, qd = np.ones(5), np.ones(5)
    assert lib.dfmi_ekf_fit(_lib.ptr(x), 1, 100, 100, None, _lib.ptr(p0), _lib.ptr(qd), None, 1.0, 1.0, 100, 1,
                            _lib.ptr(st), H, None) == -1
    import pytest
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        assert lib.dfmi_record_moments(_lib.ptr(x), 2, 50, 50, _lib.ptr(m), _lib.ptr(v), H, None) == -3
