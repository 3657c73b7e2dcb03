"""raw_data / fit_data text formats (core.py:129-174, 259-332; data.py:178-208)
through libdfmi's host parser/writer, against the calls the reference makes:
pandas.read_csv(sep=' ', skiprows=13, usecols=[c]) for raw files,
numpy.genfromtxt(skip_header=13, invalid_raise=False) for fit files, str(float)
for the writer. Host code only: runs without a GPU."""
import os
import struct
import warnings

import numpy as np
import pandas as pd
import pytest

from deepfmkit_amd import _lib, textio

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def ref_parse_header(path, kind):
    """core.py:129-174 restated: lines 2..10, characters of '1234567890.' only."""
    with open(path) as f:
        lines = [f.readline() for _ in range(11)]
    v = ["".join(c for c in lines[i] if c in "1234567890.") for i in range(2, 11)]
    out = {"channr": int(v[0]), "t0": int(v[1]), "f_samp": float(v[2]), "f_mod": float(v[3])}
    if kind == textio.FIT:
        out.update(n=int(v[4]), R=int(v[5]), fs=float(v[6]))
    return out


def ref_to_txt(fit, path):
    """data.py:178-208 restated."""
    lines = ["% fit_data", "% Message goes here", "% Number of channels: {}".format(1),
             "% Start time: {}".format(fit.t0), "% Sampling frequency: {}".format(fit.f_samp),
             "% Modulation frequency: {}".format(fit.f_mod), "% n: {}".format(int(fit.n)),
             "% Downsampling factor: {}".format(int(fit.R)), "% Fit data rate: {}".format(fit.fs),
             "% Initial amplitude: {}".format(fit.init_a), "% Initial modulation depth: {}".format(fit.init_m),
             "%", "ssq0 amp0 m0 phi0 psi0 dc0 "]
    with open(path, "w") as f:
        for line in lines:
            f.write(line + "\n")
        for i in range(len(fit.ssq)):
            f.write(" ".join(str(getattr(fit, k)[i]) for k in ("ssq", "amp", "m", "phi", "psi", "dc")) + " \n")


def test_reference_fit_file_reads_like_genfromtxt():
    """The reference's own fixture test/fit_data.txt (203 rows, 30 kHz / 400 Hz)."""
    path = os.path.join(GOLD, "fit_data_ref.txt")
    hdr = textio.parse_header(path, textio.FIT)
    assert hdr == ref_parse_header(path, textio.FIT)
    assert (hdr["channr"], hdr["n"], hdr["R"], hdr["fs"]) == (1, 20, 1500, 20.0)
    _, data = textio.read_fit(path)
    ref = np.genfromtxt(path, dtype="double", skip_header=13, invalid_raise=False)
    assert data.shape == (1, 6, 203)
    np.testing.assert_array_equal(data[0], ref.T)


def test_facade_load_fit_and_to_txt_roundtrip(tmp_path):
    import deepfmkit_amd as dfm
    dff = dfm.DeepFitFramework()
    dff.raw_file = "rec"
    dff.load_fit(os.path.join(GOLD, "fit_data_ref.txt"))
    fit = dff.fits["rec_ch0"]
    assert fit.nbuf == 203 and fit.R == 1500 and fit.fs == 20.0
    np.testing.assert_array_equal(fit.time, np.arange(0, 203 / 20.0, 1 / 20.0))
    ours, theirs = tmp_path / "ours.txt", tmp_path / "ref.txt"
    fit.to_txt(str(ours))
    ref_to_txt(fit, str(theirs))
    assert ours.read_bytes() == theirs.read_bytes()
    with pytest.raises(TypeError):  # core.py:301: None + '_ch0', as the reference
        dfm.DeepFitFramework().load_fit(os.path.join(GOLD, "fit_data_ref.txt"))


def _random_doubles(n, seed):
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 2**63 - 1, size=n, dtype=np.int64) * rng.choice([1, -1], size=n)
    vals = bits.view(np.float64)
    vals = vals[np.isfinite(vals)]
    extra = [0.0, -0.0, 1.0, 1e16, 1e15, 9999999999999998.0, 1e-4, 1e-5, 0.0001234, 123456789012.0, 5e-324,
             1.7976931348623157e308, 2.5, 100.0, 1.5e300, -3.25e-7]
    return np.concatenate([vals, rng.normal(size=n), rng.normal(size=n) * 1e-6, np.round(rng.normal(size=n) * 1e6),
                           np.array(extra)])


def test_py_repr_matches_cpython():
    lib = _lib.load()
    import ctypes
    buf = ctypes.create_string_buffer(40)
    for v in _random_doubles(20000, 1).tolist():
        k = lib.dfmi_py_repr(v, buf, 40)
        assert k > 0 and buf.value.decode() == repr(v), (v, buf.value, repr(v))


def test_fit_writer_bytes_and_bit_exact_readback(tmp_path):
    from deepfmkit_amd.data import DeepFitObject
    vals = _random_doubles(3000, 2)
    n = len(vals) // 6
    fit = DeepFitObject()
    fit.t0, fit.f_samp, fit.f_mod, fit.n, fit.R, fit.fs = 0, 200000.0, 1000, 20, 4000, 50.0
    for i, k in enumerate(("ssq", "amp", "m", "phi", "psi", "dc")):
        setattr(fit, k, vals[i * n:(i + 1) * n])
    ours, theirs = tmp_path / "ours.txt", tmp_path / "ref.txt"
    fit.to_txt(str(ours))
    ref_to_txt(fit, str(theirs))
    assert ours.read_bytes() == theirs.read_bytes()
    _, data = textio.read_fit(str(ours))
    for i, k in enumerate(("ssq", "amp", "m", "phi", "psi", "dc")):
        assert data[0, i].tobytes() == getattr(fit, k).tobytes(), k


def test_raw_reader_matches_pandas(tmp_path):
    rng = np.random.default_rng(5)
    chans = [1.0 + np.cos(rng.normal(size=5000)), rng.normal(size=5000) * 1e-3, _random_doubles(1300, 3)[:5000]]
    path = tmp_path / "raw_data.txt"
    textio.write_raw(str(path), chans, t0=20210818171519, f_samp=200000.0, f_mod=1000.0)
    hdr, got = textio.read_raw(str(path))
    assert hdr == ref_parse_header(str(path), textio.RAW)
    for c in range(3):
        ref = pd.read_csv(str(path), sep=" ", skiprows=13, usecols=[c], names=["ch" + str(c)])["ch" + str(c)]
        # bit for bit what load_raw's pandas gets — which is often not the written
        # number: pandas' converter keeps 17 digits counting leading zeros and
        # rounds twice (csrc/textio.cpp pandas_xstrtod)
        assert got[c].tobytes() == ref.to_numpy().tobytes()


def test_pandas_converter_fuzz(tmp_path):
    """The raw reader's float converter against pandas itself on many spellings."""
    rng = np.random.default_rng(11)
    v = _random_doubles(4000, 9)
    v = v[np.abs(v) < 1e300]
    fmts = [repr, lambda x: "%.17g" % x, lambda x: "%.6f" % x, lambda x: "%.12e" % x, lambda x: "%.3E" % x,
            lambda x: ("+" if x >= 0 else "") + repr(x), lambda x: "%d" % int(x) if abs(x) < 1e18 else repr(x),
            lambda x: "%.25f" % x if abs(x) < 1e3 else repr(x), lambda x: "%.1e" % (x * 1e-300)]
    lines = []
    for i, x in enumerate(v.tolist()):
        lines.append(fmts[i % len(fmts)](x))
    path = tmp_path / "fuzz.txt"
    head = ["% raw_data", "% m", "% Number of channels: 1", "% Start time: 0", "% Sampling frequency: 1.0",
            "% Modulation frequency: 1.0"] + ["%"] * 6 + ["ch0"]
    path.write_text("\n".join(head + lines) + "\n")
    _, got = textio.read_raw(str(path))
    ref = pd.read_csv(str(path), sep=" ", skiprows=13, usecols=[0], names=["ch0"])["ch0"].to_numpy()
    bad = np.nonzero(got[0].view(np.int64) != ref.view(np.int64))[0]
    assert len(bad) == 0, [(lines[i], got[0][i], ref[i]) for i in bad[:5]]


def test_raw_reader_ragged_rows_like_pandas(tmp_path):
    """Missing fields (short rows, doubled spaces) read as NaN like pandas sep=' '."""
    path = tmp_path / "ragged.txt"
    head = ["% raw_data", "% m", "% Number of channels: 2", "% Start time: 7", "% Sampling frequency: 1000.0",
            "% Modulation frequency: 10.0"] + ["%"] * 6 + ["ch0 ch1"]
    body = ["1.5 2.5", "3.25", "4.0  5.0", "-1e-300 +7", "8.5 9.5 "]
    path.write_text("\n".join(head + body) + "\n")
    _, got = textio.read_raw(str(path))
    for c in range(2):
        ref = pd.read_csv(str(path), sep=" ", skiprows=13, usecols=[c], names=["ch" + str(c)])["ch" + str(c)]
        np.testing.assert_array_equal(got[c], ref.to_numpy().astype(np.float64))


def test_fit_reader_skips_invalid_rows_like_genfromtxt(tmp_path):
    path = tmp_path / "fit.txt"
    src = open(os.path.join(GOLD, "fit_data_ref.txt")).read().splitlines()
    src.insert(20, "1.0 2.0 3.0")        # wrong field count: dropped with a warning by genfromtxt
    src.insert(30, "# a comment line")   # comments='#'
    path.write_text("\n".join(src) + "\n")
    _, data = textio.read_fit(str(path))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ref = np.genfromtxt(str(path), dtype="double", skip_header=13, invalid_raise=False)
    np.testing.assert_array_equal(data[0], ref.T)


def test_missing_file_raises():
    with pytest.raises(FileNotFoundError):
        textio.read_fit("/nonexistent/fit_data.txt")
