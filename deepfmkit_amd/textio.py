"""The reference's raw_data / fit_data text formats through libdfmi's host parser.

Reference (file:line in /root/reference):
  DeepFitFramework.parse_header  core.py:129-174
  DeepFitFramework.load_raw      core.py:259-286  (pandas.read_csv(sep=' ', skiprows=13, usecols=[c]))
  DeepFitFramework.load_fit      core.py:288-332  (numpy.genfromtxt(skip_header=13, invalid_raise=False))
  DeepFitObject.to_txt           data.py:178-208

The numbers are parsed by csrc/textio.cpp (std::from_chars, correctly rounded,
multi-threaded over line ranges) and written in CPython repr() digits, so files
are byte-identical to the reference's writer and read back bit-exact. No GPU is
involved; `read_raw(..., device=...)` hands the columns to the GPU from pinned
host memory.

The reference has no raw_data writer; `write_raw` lays a file out the way
`parse_header` / `load_raw` read it (13 header lines, one space-separated
column per channel).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib

HEADER_LINES = 13
RAW, FIT = 0, 1
SINGLE_SPACE, WHITESPACE = 0, 1


class TxtHeader(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("channels", ctypes.c_int32), ("t0", ctypes.c_int64),
                ("f_samp", ctypes.c_double), ("f_mod", ctypes.c_double), ("n", ctypes.c_int32),
                ("R", ctypes.c_int32), ("fs", ctypes.c_double)]


def _check(lib, rc, what):
    if rc < 0:
        raise ValueError(f"{what}: {lib.dfmi_txt_last_error().decode()}")


def _threads():
    return max(1, min(16, os.cpu_count() or 1))


def parse_header(path, kind):
    """core.py:129-174: the numbers of header lines 3..11 (index 2..10), each line
    reduced to its characters in '1234567890.'. Returns a dict with the keys the
    reference sets (channr, t0, f_samp, f_mod; + n, R, fs for fit files)."""
    lib = _lib.load()
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    h = TxtHeader()
    _check(lib, lib.dfmi_txt_parse_header(os.fsencode(path), kind, ctypes.byref(h)), "parse_header")
    out = {"channr": int(h.channels), "t0": int(h.t0), "f_samp": float(h.f_samp), "f_mod": float(h.f_mod)}
    if kind == FIT:
        out.update(n=int(h.n), R=int(h.R), fs=float(h.fs))
    return out


def read_columns(path, cols, mode, skip=HEADER_LINES):
    """Numeric columns `cols` of the data rows after `skip` lines: (len(cols), rows)
    float64, NaN where a row lacks the field."""
    lib = _lib.load()
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    rows, ncols = ctypes.c_int64(), ctypes.c_int32()
    _check(lib, lib.dfmi_txt_shape(os.fsencode(path), skip, mode, ctypes.byref(rows), ctypes.byref(ncols)), "shape")
    cols = np.ascontiguousarray(cols, dtype=np.int32)
    out = np.empty((len(cols), rows.value), dtype=np.float64)
    _check(lib, lib.dfmi_txt_read(os.fsencode(path), skip, mode, len(cols), _lib.ptr(cols), _lib.ptr(out),
                                  rows.value, _threads()), "read")
    return out, int(ncols.value)


def read_raw(path, device=None):
    """load_raw's data (core.py:279-280): channel c = column c of every row after the
    13 header lines, pandas sep=' ' semantics. Returns (header dict, list of channel
    arrays); with `device` ("cuda:0", ...) the channels are torch tensors there."""
    hdr = parse_header(path, RAW)
    data, _ = read_columns(path, list(range(hdr["channr"])), SINGLE_SPACE)
    if device is None:
        return hdr, [data[c] for c in range(hdr["channr"])]
    import torch
    host = torch.from_numpy(data).pin_memory()
    dev = host.to(device, non_blocking=True)
    torch.cuda.current_stream(dev.device).synchronize()
    return hdr, [dev[c] for c in range(hdr["channr"])]


def read_fit(path):
    """load_fit's data (core.py:306-330): 6 columns per channel, genfromtxt semantics.
    Returns (header dict, (channels, 6, rows) array: ssq, amp, m, phi, psi, dc)."""
    hdr = parse_header(path, FIT)
    nch = hdr["channr"]
    data, _ = read_columns(path, list(range(6 * nch)), WHITESPACE)
    return hdr, data.reshape(nch, 6, -1)


def fit_header_text(fit):
    """The 13 header lines of data.py:180-192, formatted from the DeepFitObject's
    own (Python-typed) fields exactly as the reference does."""
    lines = ["% fit_data", "% Message goes here", "% Number of channels: {}".format(1),
             "% Start time: {}".format(fit.t0), "% Sampling frequency: {}".format(fit.f_samp),
             "% Modulation frequency: {}".format(fit.f_mod), "% n: {}".format(int(fit.n)),
             "% Downsampling factor: {}".format(int(fit.R)), "% Fit data rate: {}".format(fit.fs),
             "% Initial amplitude: {}".format(fit.init_a), "% Initial modulation depth: {}".format(fit.init_m),
             "%", "ssq0 amp0 m0 phi0 psi0 dc0 "]
    return "".join(line + "\n" for line in lines)


def write_fit(fit, path):
    """data.py:178-208: header + one row per buffer, str(float) values each followed by
    a space."""
    lib = _lib.load()
    cols = [np.ascontiguousarray(np.asarray(getattr(fit, k), dtype=np.float64))
            for k in ("ssq", "amp", "m", "phi", "psi", "dc")]
    n = len(cols[0])
    if any(len(c) != n for c in cols):
        raise ValueError("fit columns differ in length")
    _check(lib, lib.dfmi_fit_txt_write(os.fsencode(path), fit_header_text(fit).encode(),
                                       *[_lib.ptr(c) for c in cols], n), "write_fit")


def write_raw(path, channels, t0, f_samp, f_mod, message="Message goes here"):
    """A raw_data file as parse_header/load_raw read it: line 3 channels, 4 start
    time, 5 sampling frequency, 6 modulation frequency, filler up to 13 header
    lines, then one row per sample with the channels separated by single spaces
    (values in repr() digits, so they read back bit-exact)."""
    chans = [np.asarray(c, dtype=np.float64).reshape(-1) for c in channels]
    n = len(chans[0])
    if any(len(c) != n for c in chans):
        raise ValueError("channels differ in length")
    head = ["% raw_data", f"% {message}", f"% Number of channels: {len(chans)}", f"% Start time: {t0}",
            f"% Sampling frequency: {f_samp}", f"% Modulation frequency: {f_mod}", "%", "%", "%", "%", "%", "%",
            " ".join(f"ch{c}" for c in range(len(chans)))]
    stack = np.stack(chans, axis=1).tolist()
    with open(path, "w") as f:
        f.write("".join(h + "\n" for h in head))
        f.writelines(" ".join(map(repr, row)) + "\n" for row in stack)
