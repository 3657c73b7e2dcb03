"""Fitter strategies — the reference's plugin boundary (fitters.py:164-447).

`DeepFitFramework.fit` (core.py) picks a class from a method map and calls
`FitterClass({'n': n}).fit(main_raw, **kwargs) -> DataFrame` with the columns
amp, m, phi, psi, dc, ssq, fitok — exactly the reference's contract
(fitters.py:186-208). Here the NLS and EKF strategies run on the GPU through
libdfmi.so; there is no CPU fallback.

Reference map:
  _calculate_fit_params ......... fitters.py:62-86
  BaseFitter .................... fitters.py:164-208
  EKFFitter.fit ................. fitters.py:214-320
  StandardNLSFitter.fit ......... fitters.py:330-368
    _fit_sequential ............. fitters.py:370-393  (parallel=False)
    _fit_parallel ............... fitters.py:395-428  (parallel=True)
  WDFMI_NLSFitter.fit ........... fitters.py:481-570  (EXPERIMENTAL in the reference)
  WDFMI_OrthogonalFitter.fit .... fitters.py:572-648
  WDFMI_SequentialFitter.fit .... fitters.py:650-776
  HWDFMI_Fitter.fit ............. fitters.py:778-891
"""
from __future__ import annotations

import logging
import time
import weakref
from abc import ABC, abstractmethod

import numpy as np
import pandas as pd
import scipy.constants as sc

from . import _lib
from . import fit as _fit

log = logging.getLogger(__name__)

COLUMNS = ["amp", "m", "phi", "psi", "dc", "ssq", "fitok"]

# Facade timing marks (scripts/profile_facade.py sets a list here): (label, perf_counter())
# appended at each stage of DeepFitFramework.fit's NLS path; None = off (one test per mark).
MARKS = None


def mark(label):
    if MARKS is not None:
        MARKS.append((label, time.perf_counter()))


def _calculate_fit_params(raw_obj, n):
    """fitters.py:62-86: R = int(f_samp/f_mod*n), fs = f_samp/R, nbuf = int(N/R)."""
    R = int(raw_obj.f_samp / raw_obj.f_mod * n)
    fs = raw_obj.f_samp / R
    nbuf = int(raw_obj.n_samples() / R)
    if nbuf == 0:
        logging.error("Check buffer size! nbuf is zero.")
    return R, fs, nbuf


def _is_device_tensor(x):
    return hasattr(x, "data_ptr") and getattr(x, "is_cuda", False)


def _torch_stream(device=None):
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def _on_device(x):
    """Context that makes x's GPU the current HIP device for the library call: the C ABI
    launches on hipGetDevice(), so a tensor on cuda:1 must be fitted with cuda:1 current."""
    import torch
    return torch.cuda.device(x.device)


def w0_of(f_mod, f_samp):
    """fitters.py:39 / 376 / 434: w0 = 2*pi*f_mod/f_samp (same operation order)."""
    return 2.0 * np.pi * f_mod / f_samp


def nls_records(records, f_samp, f_mod, R, nbuf, ndata=10, init_guess=(1.6, 6.0, 0.0, 0.0), parallel=True,
                n_cores=None):
    """Run the StandardNLSFitter pipeline on one or more equal-length records in ONE
    GPU call (config 3: several channels as one batch).

    records: list of 1-D float64 arrays (host) or CUDA tensors, or a 2-D array/tensor
    (nrec, >= nbuf*R). init_guess: (4,) shared or (nrec, 4). Returns (cols (6, nrec*nbuf)
    in the order amp, m, phi, psi, dc, ssq; fitok (nrec*nbuf,)), as numpy arrays for host
    input and as CUDA tensors for device input."""
    lib = _lib.load()
    w0 = w0_of(f_mod, f_samp)
    if isinstance(records, (list, tuple)):
        if _is_device_tensor(records[0]):
            import torch
            x = torch.stack([r[: nbuf * R] for r in records]).contiguous()
        else:
            x = np.ascontiguousarray(np.stack([np.asarray(r, np.float64)[: nbuf * R] for r in records]))
    else:
        x = records
    nrec = int(x.shape[0])
    rec_stride = int(x.stride(0)) if _is_device_tensor(x) else int(x.strides[0] // 8)
    g = np.asarray(init_guess, dtype=np.float64)
    g = np.ascontiguousarray(np.broadcast_to(g, (nrec, 4)) if g.ndim == 1 else g)
    nchunk = (nbuf - 1) if n_cores is None else max(1, min(int(n_cores), nbuf))
    cfg = _fit.lm_config()
    nseg = nrec * nbuf
    if _is_device_tensor(x):
        import torch
        if x.dtype != torch.float64 or x.stride(-1) != 1:
            raise ValueError("device records must be contiguous float64 rows")
        # rows 0..5 of one (7, nseg) block: the six result columns; row 6 receives fitok as
        # int64 (frame_from), so the whole result leaves the device in one copy
        out = torch.empty((7, nseg), dtype=torch.float64, device=x.device)[:6]
        out._dfmi_block = True  # frame_from may use row 6 (this function's own allocation)
        ok = torch.empty(nseg, dtype=torch.int32, device=x.device)
        mark("alloc")
        with _on_device(x):
            rc = lib.dfmi_nls_record(x.data_ptr(), nrec, rec_stride, nbuf, R, ndata, w0, 0, _lib.ptr(g),
                                     1 if parallel else 0, max(nchunk, 1), cfg, out.data_ptr(), ok.data_ptr(),
                                     _lib.DFMI_MEM_DEVICE, _torch_stream(x.device))
        _lib.check(rc, "dfmi_nls_record")
        mark("enqueue")
        return out, ok
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty((6, nseg))
    ok = np.empty(nseg, dtype=np.int32)
    rc = lib.dfmi_nls_record(_lib.ptr(x), nrec, rec_stride, nbuf, R, ndata, w0, 0, _lib.ptr(g),
                             1 if parallel else 0, max(nchunk, 1), cfg, _lib.ptr(out), _lib.ptr(ok),
                             _lib.DFMI_MEM_HOST, None)
    _lib.check(rc, "dfmi_nls_record")
    return out, ok


def nls_record_devices(x, f_samp, f_mod, R, nbuf, devices, ndata=10, init_guess=(1.6, 6.0, 0.0, 0.0)):
    """One record's _fit_parallel with chunk size 1 (fitters.py:395-428: buffer 0 fitted from
    init_guess, every other buffer seeded with its result) spread over several GPUs of this
    process: buffers 1..nbuf-1 are cut into len(devices) contiguous shards (np.array_split),
    shard s is fitted on devices[s] as its own record with buffer 0 prepended — every device
    fits the seed buffer itself, as every reference Pool chunk receives it (no exchange) —
    and the rows come back in record order. All devices' work is enqueued before any result
    is read, so the GPUs run concurrently; each shard's samples go host -> device (or
    device -> device) once. x: 1-D float64 numpy array or CUDA tensor (>= nbuf*R samples).
    Returns (cols (6, nbuf) numpy in the order amp, m, phi, psi, dc, ssq; fitok (nbuf,)),
    bit-identical to one nls_records call (segments are independent once the seed is known).
    Same-device entries are allowed (shards then run one after another on that GPU)."""
    import torch
    devs = [torch.device("cuda", int(d)) if not isinstance(d, torch.device) else d for d in devices]
    if not devs:
        raise ValueError("devices: at least one GPU")
    if nbuf < 1:
        raise ValueError("nbuf must be >= 1")
    parts = [c for c in np.array_split(np.arange(1, nbuf), len(devs)) if c.size] if nbuf > 1 else []
    if not parts:
        parts = [np.arange(1, 1)]
    host = not _is_device_tensor(x)
    if host:
        x = np.asarray(x, dtype=np.float64)
    pending = []
    for dev, idx in zip(devs, parts):
        b0, b1 = (int(idx[0]), int(idx[-1]) + 1) if idx.size else (1, 1)
        n_s = 1 + (b1 - b0)
        with torch.cuda.device(dev):
            xs = torch.empty(n_s * R, dtype=torch.float64, device=dev)
            if host:
                xs[:R].copy_(torch.from_numpy(x[:R]))
                if b1 > b0:
                    xs[R:].copy_(torch.from_numpy(x[b0 * R:b1 * R]))
            else:
                xs[:R].copy_(x[:R])
                if b1 > b0:
                    xs[R:].copy_(x[b0 * R:b1 * R])
            cols, ok = nls_records(xs.view(1, -1), f_samp, f_mod, R, n_s, ndata, init_guess, parallel=True)
        pending.append((cols, ok, b1 > b0))
    out_cols, out_ok = [], []
    for k, (cols, ok, has_rows) in enumerate(pending):
        c = cols.cpu().numpy()
        o = ok.cpu().numpy()
        if k == 0:
            out_cols.append(c)
            out_ok.append(o)
        elif has_rows:
            out_cols.append(c[:, 1:])
            out_ok.append(o[1:])
    return np.concatenate(out_cols, axis=1), np.concatenate(out_ok)


# The 1-D column arrays a frame_from frame was built over, by id(frame) while the frame lives
# (and, for the facade, the frame with core.py:506-509's tau column already appended): core's
# _finish takes them from here for the package's own NLS fitter (a pandas column access costs
# ~10 us each, a frame construction ~40 us) after checking the entry belongs to that frame.
_FRAME_ARRAYS = {}
NO_TAU = object()


def _remember(df, arrays, with_tau=None):
    key = id(df)
    _FRAME_ARRAYS[key] = (weakref.ref(df), arrays, with_tau)
    weakref.finalize(df, _FRAME_ARRAYS.pop, key, None)
    return df


def frame_arrays(df):
    """The column arrays of a frame built by frame_from (dict name -> array) and, when frame_from
    formed it, (the frame with tau appended, the tau array) (else None); None for other frames."""
    e = _FRAME_ARRAYS.get(id(df))
    if e is None or e[0]() is not df or list(df.columns) != list(e[1]):
        return None
    return e[1], e[2]


def tau_divisor(raw):
    """core.py:506-509: tau = m / (2 pi df), or 0.0 without a simulation object (None here)."""
    return 2 * np.pi * raw.sim.laser.df if raw.sim else None


def frame_from(cols, fitok, tau_div=NO_TAU):
    """DataFrame with the reference's column set and dtypes (fitters.py:55-58, 428): float64
    amp, m, phi, psi, dc, ssq and int64 fitok, one 1-D array per column (a dict frame built
    with copy=False wraps them as they are: no consolidation copy).

    Device results (nls_records' (6, n) rows of a (7, n) block and the int32 status): the status
    is widened to int64 into the block's spare row on the device, the whole block goes to
    pinned host memory in ONE asynchronous copy, and the frame is built over that memory while
    the kernels and the copy run; one stream synchronisation, then the frame is returned. The
    pinned block belongs to this frame's arrays (torch's caching host allocator reuses it once
    they are gone). With tau_div (tau_divisor(raw), the facade's NLS path) the frame core's
    _finish stores — the same columns plus tau = m / tau_div, numpy's division — is prebuilt
    too, tau filled after the synchronisation."""
    if hasattr(cols, "cpu"):
        import torch
        n = cols.shape[1]
        if getattr(cols, "_dfmi_block", False):  # nls_records' (7, n) block: row 6 is ours
            base = torch.as_strided(cols, (7, n), (n, 1))
        else:  # a caller's own (6, n) tensors: same copy through a fresh block
            base = torch.empty((7, n), dtype=torch.float64, device=cols.device)
            base[:6].copy_(cols)
        stream = torch.cuda.current_stream(cols.device)
        base[6].view(torch.int64).copy_(fitok)
        host = torch.empty((7, n), dtype=torch.float64, pin_memory=True)
        host.copy_(base, non_blocking=True)
        done = torch.cuda.Event()
        done.record(stream)
        h = host.numpy()
        arrays = dict(zip(COLUMNS, [h[0], h[1], h[2], h[3], h[4], h[5], h[6].view(np.int64)]))
        with_tau = tau = None
        if tau_div is not NO_TAU:
            tau = np.empty(n) if tau_div is not None else np.zeros(n)
            with_tau = pd.DataFrame({**arrays, "tau": tau}, copy=False)
        df = _remember(pd.DataFrame(arrays, copy=False), arrays, None if with_tau is None else (with_tau, tau))
        mark("frame_prebuilt")
        if MARKS is not None:  # profiling: the wait for the kernels apart from the copy
            stream.synchronize()
            mark("gpu_done")
        done.synchronize()
        mark("d2h")
        if tau is not None and tau_div is not None:
            np.divide(h[1], tau_div, out=tau)
        return df
    cols = np.ascontiguousarray(cols, dtype=np.float64)
    arrays = dict(zip(COLUMNS, [cols[0], cols[1], cols[2], cols[3], cols[4], cols[5],
                                np.asarray(fitok).astype(np.int64)]))
    df = _remember(pd.DataFrame(arrays, copy=False), arrays)
    mark("frame")
    return df


class BaseFitter(ABC):
    """fitters.py:164-208."""

    def __init__(self, fit_config: dict):
        self.config = fit_config
        if "n" not in self.config:
            raise ValueError("Fit configuration must include 'n'.")

    @abstractmethod
    def fit(self, main_raw, **kwargs) -> pd.DataFrame:
        ...


class StandardNLSFitter(BaseFitter):
    """Frequency-domain NLS, one GPU call per record (fitters.py:322-447).

    kwargs: ndata (10), parallel (True), init_a (1.6), init_m (6.0), init_psi (0.0),
    n_cores (None), devices (None: the current GPU; a list of GPU indices spreads a
    parallel=True, n_cores=None fit over those GPUs, nls_record_devices).  parallel=True follows _fit_parallel: buffer 0 is fitted from
    the default seed and seeds the rest; with n_cores=None every remaining buffer
    is its own chunk (the GPU-natural split; the reference's own chunk choice
    changes results by <= 2.5e-10), with n_cores=k the buffers are
    split into k warm-start chains exactly as np.array_split does.
    parallel=False follows _fit_sequential (one warm-start chain)."""

    def fit(self, main_raw, **kwargs) -> pd.DataFrame:
        n = self.config["n"]
        ndata = int(kwargs.pop("ndata", self.config.get("ndata", 10)))
        parallel = kwargs.get("parallel", True)
        init_a = kwargs.get("init_a", 1.6)
        init_m = kwargs.get("init_m", 6.0)
        init_psi = kwargs.get("init_psi", 0.0)
        R, _, nbuf = _calculate_fit_params(main_raw, n)
        if nbuf == 0:
            return pd.DataFrame()
        x = main_raw.samples()
        N = int(x.shape[0])
        if N % R != 0:
            # the reference reshapes the whole column with reshape(-1, R) (fitters.py:375, 412)
            raise ValueError(f"cannot reshape array of size {N} into shape ({R})")
        if not _is_device_tensor(x):
            x = np.asarray(x, dtype=np.float64)
        devices = kwargs.get("devices")
        if devices is not None and (not parallel or kwargs.get("n_cores") is not None):
            # a device list spreads the chunk-size-1 parallel fit only; a warm-start chain
            # (parallel=False, or the n_cores array_split chains) runs on the current GPU
            raise ValueError("devices= applies to parallel=True without n_cores (chunk size 1); "
                             f"got parallel={parallel}, n_cores={kwargs.get('n_cores')}")
        mark("fitter_args")
        if devices is not None:
            cols, ok = nls_record_devices(x, main_raw.f_samp, main_raw.f_mod, R, nbuf, devices, ndata,
                                          (init_a, init_m, 0.0, init_psi))
            return frame_from(cols, ok)
        cols, ok = nls_records(x.reshape(1, N), main_raw.f_samp, main_raw.f_mod, R, nbuf, ndata,
                               (init_a, init_m, 0.0, init_psi), parallel=parallel,
                               n_cores=kwargs.get("n_cores") if parallel else None)
        return frame_from(cols, ok, tau_divisor(main_raw))


class EKFFitter(BaseFitter):
    """Per-sample EKF on the GPU (fitters.py:210-320)."""

    def fit(self, main_raw, **kwargs) -> pd.DataFrame:
        kw = {k: v for k, v in kwargs.items() if k != "n"}
        res = ekf_records([main_raw], self.config["n"], **kw)[0]
        nbuf = res.shape[0]
        return pd.DataFrame({"amp": res[:, 0], "m": res[:, 1], "phi": res[:, 2], "psi": res[:, 3], "dc": res[:, 4],
                             "ssq": np.zeros(nbuf), "fitok": np.ones(nbuf, dtype=int)}, columns=COLUMNS)


def ekf_records(raws, n, **kwargs):
    """EKF over several channels of equal length in one launch (lane = channel)."""
    lib = _lib.load()
    xs = [np.asarray(r.samples(), dtype=np.float64) for r in raws]
    n_samp = xs[0].size
    if any(x.size != n_samp for x in xs):
        raise ValueError("EKF batch needs channels of equal length")
    f_samp, f_mod = raws[0].f_samp, raws[0].f_mod
    R, _, nbuf = _calculate_fit_params(raws[0], n)
    init = [kwargs.get("init_a", 1.6), kwargs.get("init_m", 6.0), kwargs.get("init_phi", 0.0),
            kwargs.get("init_psi", 0.0)]
    p0 = np.ascontiguousarray(kwargs.get("P0_diag", [1.0] * 5), dtype=np.float64)
    qd = np.ascontiguousarray(kwargs.get("Q_diag", [1e-8, 1e-8, 1e-6, 1e-6, 1e-8]), dtype=np.float64)
    r_val = kwargs.get("R_val", None)
    x = np.ascontiguousarray(np.stack(xs))
    init4 = np.ascontiguousarray(init, dtype=np.float64)
    # x0[4] = np.mean(data) (fitters.py:253) and, without R_val, np.var(data) (:256):
    # formed on the device by dfmi_ekf_fit, in numpy's summation order
    rv = None if r_val is None else np.ascontiguousarray([r_val], dtype=np.float64)
    states = np.zeros((len(xs), max(nbuf, 0), 5))
    w_m = 2 * np.pi * f_mod
    rc = lib.dfmi_ekf_fit(_lib.ptr(x), len(xs), n_samp, n_samp, _lib.ptr(init4), _lib.ptr(p0), _lib.ptr(qd),
                          None if rv is None else _lib.ptr(rv), w_m, float(f_samp), R, max(nbuf, 0), _lib.ptr(states),
                          _lib.DFMI_MEM_HOST, None)
    _lib.check(rc, "dfmi_ekf_fit")
    return states


WDFMI_COLUMNS = ["amp", "m", "phi", "psi", "tau", "dc", "ssq", "fitok"]


def wdfmi_records(method, mains, witnesses, f_samp, f_mod, R, nbuf, df=0.0, f_ref=0.0, tau_init=0.0, ndata=10,
                  ndata_psi=40, init_a=1.6, init_phi=0.0, init_psi=0.0, period=0):
    """Run one witness-based fitter over one or more records in ONE GPU call.

    mains: (nrec, >= nbuf*R) array / CUDA tensor or a list of 1-D records; witnesses:
    the same for the witness channels (only the first R samples are used), or one
    1-D witness shared by every record. Returns (cols (7, nrec*nbuf) in the order
    amp, m, phi, psi, tau, dc, ssq; fitok (nrec*nbuf,)), numpy for host input and CUDA
    tensors for device input."""
    lib = _lib.load()
    dev = _is_device_tensor(mains if not isinstance(mains, (list, tuple)) else mains[0])
    if dev:
        import torch
        x = torch.stack([r[: nbuf * R] for r in mains]) if isinstance(mains, (list, tuple)) else mains
        x = x.contiguous()
        w = torch.stack([r[:R] for r in witnesses]) if isinstance(witnesses, (list, tuple)) else witnesses
        w = w.contiguous()
        if x.dtype != torch.float64 or w.dtype != torch.float64:
            raise ValueError("device records must be float64")
    else:
        if isinstance(mains, (list, tuple)):
            x = np.ascontiguousarray(np.stack([np.asarray(r, np.float64)[: nbuf * R] for r in mains]))
        else:
            x = np.ascontiguousarray(np.asarray(mains, np.float64))
        if isinstance(witnesses, (list, tuple)):
            w = np.ascontiguousarray(np.stack([np.asarray(r, np.float64)[:R] for r in witnesses]))
        else:
            w = np.ascontiguousarray(np.asarray(witnesses, np.float64))
    if x.ndim == 1:
        x = x.reshape(1, -1)
    nrec = int(x.shape[0])
    if w.ndim == 1:
        wit_stride = 0
    else:
        wit_stride = int(w.stride(0)) if dev else int(w.strides[0] // 8)
        if int(w.shape[0]) != nrec:
            raise ValueError("one witness per record (or a single shared one) is required")
    if int(w.shape[-1]) < R:
        raise ValueError(f"witness needs at least R={R} samples")
    rec_stride = int(x.stride(0)) if dev else int(x.strides[0] // 8)
    if int(x.shape[1]) < nbuf * R:
        raise ValueError("records shorter than nbuf*R")
    cfg = _lib.WdfmiConfig(_lib.WDFMI_METHODS[method], int(ndata), int(ndata_psi), int(period), float(f_samp),
                           float(f_mod), float(df), float(f_ref), float(tau_init), float(init_a), float(init_phi),
                           float(init_psi))
    nseg = nrec * nbuf
    if dev:
        import torch
        out = torch.empty((7, nseg), dtype=torch.float64, device=x.device)
        ok = torch.empty(nseg, dtype=torch.int32, device=x.device)
        if w.device != x.device:
            raise ValueError("main and witness records must be on the same device")
        with _on_device(x):
            rc = lib.dfmi_wdfmi_fit(x.data_ptr(), nrec, rec_stride, nbuf, R, w.data_ptr(), wit_stride, cfg,
                                    out.data_ptr(), ok.data_ptr(), _lib.DFMI_MEM_DEVICE, _torch_stream(x.device))
    else:
        out = np.empty((7, nseg))
        ok = np.empty(nseg, dtype=np.int32)
        rc = lib.dfmi_wdfmi_fit(_lib.ptr(x), nrec, rec_stride, nbuf, R, _lib.ptr(w), wit_stride, cfg, _lib.ptr(out),
                                _lib.ptr(ok), _lib.DFMI_MEM_HOST, None)
    _lib.check(rc, "dfmi_wdfmi_fit")
    return out, ok


def wdfmi_frame(cols, fitok):
    """DataFrame with the witness fitters' columns (fitters.py:563-567, 640-645, 768-773, 883-888)."""
    if hasattr(cols, "cpu"):
        cols = cols.cpu().numpy()
        fitok = fitok.cpu().numpy()
    d = {k: np.asarray(cols[i]) for i, k in enumerate(WDFMI_COLUMNS[:7])}
    d["fitok"] = np.asarray(fitok).astype(np.int64)
    return pd.DataFrame(d, columns=WDFMI_COLUMNS)


class _WitnessFitter(BaseFitter):
    """Shared plumbing of the witness-based fitters: geometry, config, one GPU call."""

    METHOD = None

    def _run(self, main_raw, witness_raw, tau_init, **kw):
        R, _, nbuf = _calculate_fit_params(main_raw, self.config["n"])
        if nbuf == 0:
            return pd.DataFrame()
        laser = main_raw.sim.laser
        x = main_raw.samples()
        wv = witness_raw.samples()
        if not _is_device_tensor(x):
            x = np.asarray(x, dtype=np.float64)
            wv = np.asarray(wv, dtype=np.float64)
        cols, ok = wdfmi_records(self.METHOD, x[: nbuf * R].reshape(1, nbuf * R), wv[:R], main_raw.f_samp,
                                 laser.f_mod, R, nbuf, df=laser.df, tau_init=tau_init, **kw)
        return wdfmi_frame(cols, ok)


class WDFMI_NLSFitter(_WitnessFitter):
    """fitters.py:481-570: direct 4-parameter NLS (C, tau, phi, psi) on the harmonic
    residuals, MINPACK lmdif as least_squares(method='lm') runs it, warm-started
    buffer to buffer. ndata comes from the fit config (default 10), as in the reference."""

    METHOD = "wdfmi_nls"

    def fit(self, main_raw, witness_raw, **kwargs) -> pd.DataFrame:
        ifo = main_raw.sim.ifo
        tau_init = (ifo.meas_arml - ifo.ref_arml) / sc.c
        return self._run(main_raw, witness_raw, tau_init, ndata=self.config.get("ndata", 10),
                         init_a=kwargs.get("init_a", 1.6), init_phi=kwargs.get("init_phi", 0.0),
                         init_psi=kwargs.get("init_psi", 0.0))


class WDFMI_OrthogonalFitter(_WitnessFitter):
    """fitters.py:572-648: Nelder-Mead over (tau, psi) of the VarPro residual."""

    METHOD = "wdfmi_ortho"

    def fit(self, main_raw, witness_raw, **kwargs) -> pd.DataFrame:
        laser, ifo = main_raw.sim.laser, main_raw.sim.ifo
        tau_init = (ifo.meas_arml - ifo.ref_arml) / sc.c if laser.df > 0 else 0.0
        return self._run(main_raw, witness_raw, tau_init, init_psi=kwargs.get("init_psi", 0.0))


class WDFMI_SequentialFitter(_WitnessFitter):
    """fitters.py:650-776: tau by Brent (VarPro), psi by bounded Brent on the harmonic
    phase error (40 harmonics), then the linear fit; buffers are independent."""

    METHOD = "wdfmi_seq"

    def fit(self, main_raw, witness_raw, **kwargs) -> pd.DataFrame:
        laser, ifo = main_raw.sim.laser, main_raw.sim.ifo
        tau_init = (ifo.meas_arml - ifo.ref_arml) / sc.c if laser.df > 0 else 0.0
        return self._run(main_raw, witness_raw, tau_init, init_psi=kwargs.get("init_psi", 0.0))


class HWDFMI_Fitter(_WitnessFitter):
    """fitters.py:778-891: 1-D VarPro search for tau against the heterodyne witness's
    integrated laser phase; f_ref from the witness ifo's arml_mod_f (fitters.py:827-831)."""

    METHOD = "hwdfmi"

    def fit(self, main_raw, witness_raw, **kwargs) -> pd.DataFrame:
        init_tau = kwargs.get("init_tau", None)
        if hasattr(witness_raw.sim.ifo, "arml_mod_f"):
            f_ref = witness_raw.sim.ifo.arml_mod_f
        else:
            logging.warning("Reference frequency `f_ref` not found in witness config. Assuming 0 Hz.")
            f_ref = 0.0
        if init_tau is not None:
            tau = init_tau
        else:
            tau = (main_raw.sim.ifo.meas_arml - main_raw.sim.ifo.ref_arml) / sc.c
        return self._run(main_raw, witness_raw, tau, f_ref=f_ref)


FITTER_MAP = {
    "nls": StandardNLSFitter,
    "ekf": EKFFitter,
    "wdfmi_nls": WDFMI_NLSFitter,
    "wdfmi_ortho": WDFMI_OrthogonalFitter,
    "wdfmi_seq": WDFMI_SequentialFitter,
    "hwdfmi": HWDFMI_Fitter,
}
