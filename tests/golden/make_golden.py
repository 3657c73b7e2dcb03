"""Generate the golden parity fixtures from the reference DeepFMKit (run HERE only).

This script imports the read-only reference at /root/reference (it never travels
to the GPU box) and writes small, data-only fixtures into tests/golden/:

  bessel.npz        scipy.special.jv(n, x) table (the reference's Bessel, fit.py:3,106-108)
  lm_vectors.npz    (QI, guess) -> fit.fit (status, p, ssq)               fit.py:322-361
  records.npz       per-record outputs of StandardNLSFitter / fit.py      fitters.py:330-447
                    (sequential, parallel chunk-size-1, parallel n_cores=8) plus the
                    demodulated QI/dc of every buffer (fit.py:18-66, fitters.py:45-57)
  asd_pair.npz      config-3 two-channel asd-mode input + independent fits (core.py:519-588)
  ekf.npz           EKFFitter snapshot states                              fitters.py:214-320
  manifest.json     generator parameters + SHA-256 of every regenerated input array

Inputs of snr-mode records are NOT stored: the build regenerates them with its own
restatement of physics.py:475-530 (deepfmkit_amd.physics) and the tests check the
SHA-256 recorded here, which pins the input bit-for-bit.

Usage:  python tests/golden/make_golden.py
Environment: numpy 2.2.6, scipy 1.15.3 (recorded in manifest.json).
"""
import hashlib
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_PARENT = "/tmp/dfmk_golden"


def _import_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    os.makedirs(REF_PARENT, exist_ok=True)
    link = os.path.join(REF_PARENT, "DeepFMKit")
    if not os.path.islink(link):
        os.symlink("/root/reference", link)
    sys.path.insert(0, REF_PARENT)
    # physics.py:5 imports pyplnoise unconditionally; it is only used for coloured
    # ASD noise (physics.py:599-605), which no fixture here exercises.
    sys.modules.setdefault("pyplnoise", types.ModuleType("pyplnoise"))
    import logging
    import DeepFMKit.core as dfm  # noqa: E402
    import DeepFMKit.fit as rfit  # noqa: E402
    import DeepFMKit.fitters as rfitters  # noqa: E402
    logging.getLogger().setLevel(logging.WARNING)
    return dfm, rfit, rfitters


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def make_bessel(rfit):
    from scipy.special import jv
    n = np.arange(0, 65)
    x = np.concatenate([np.linspace(-64.0, 64.0, 513),
                        np.array([0.0, 1e-300, 1e-12, -1e-12, 1e-6, 1e-3, 0.5, 2.404825557695773,
                                  5.520078110286311, 6.0, 7.3, 31.4, -31.4, 19.999, 63.99])])
    table = jv(n[:, None], x[None, :])
    np.savez_compressed(os.path.join(HERE, "bessel.npz"), n=n, x=x, jv=table)
    return {"n_orders": int(n.size), "n_x": int(x.size)}


def analytic_qi(ndata, p):
    from scipy.special import jv
    a, m, phi, psi = p
    j = np.arange(1, ndata + 1)
    common = a * np.cos(phi + j * np.pi / 2.0) * jv(j, m)
    return np.concatenate([common * np.cos(j * psi), -common * np.sin(j * psi)])


def reference_fuzz(rfit, ndata, qis, guesses, p, reps=3):
    """The reference's own sensitivity: max |d p| of fit.fit when every QI entry is
    perturbed by about one ulp (relative 2^-52 Gaussian), over `reps` draws (wrapped
    phi). A parity tolerance below this is asking for bits the reference itself
    does not determine."""
    rng = np.random.RandomState(777)
    fz = np.zeros((qis.shape[0], 4))
    for i in range(qis.shape[0]):
        for _ in range(reps):
            q2 = qis[i] * (1.0 + 2.0 ** -52 * rng.randn(qis.shape[1]))
            _, pp, _ = rfit.fit(ndata, q2, guesses[i].copy())
            d = np.abs(pp - p[i])
            d[2] = abs((pp[2] - p[i][2] + np.pi) % (2 * np.pi) - np.pi)
            fz[i] = np.maximum(fz[i], d)
    return fz


def reference_radius(rfit, ndata, qis, p):
    """Stopping radius of the reference's LM: |p_ref - p*| where p* continues the
    reference's own _run_lma_fit (fit.py:208-258) from p_ref with the convergence
    test disabled (it then stops only when no damping value lowers ssq, i.e. at
    the machine-precision minimum). Two correct implementations of the same LM
    may stop anywhere inside this radius, so parity is judged against it."""
    saved = (rfit.MAX_LMA_STEPS, rfit.LMA_CONVERGENCE_IMPROVE, rfit.LMA_CONVERGENCE_PARAM_CHANGE)
    rfit.MAX_LMA_STEPS, rfit.LMA_CONVERGENCE_IMPROVE, rfit.LMA_CONVERGENCE_PARAM_CHANGE = 500, -1.0, -1.0
    try:
        rad = np.zeros((qis.shape[0], 4))
        for i in range(qis.shape[0]):
            ps, _ = rfit._run_lma_fit(ndata, qis[i].copy(), p[i].copy())
            d = np.abs(ps - p[i])
            d[2] = abs((ps[2] - p[i][2] + np.pi) % (2 * np.pi) - np.pi)
            rad[i] = d
    finally:
        rfit.MAX_LMA_STEPS, rfit.LMA_CONVERGENCE_IMPROVE, rfit.LMA_CONVERGENCE_PARAM_CHANGE = saved
    return rad


def make_lm_vectors(rfit):
    rng = np.random.RandomState(12345)
    groups = {}
    for ndata, count in [(10, 300), (5, 40), (20, 60), (30, 40), (62, 20)]:
        qis, guesses, truths = [], [], []
        for k in range(count):
            a = rng.uniform(0.3, 2.0)
            if ndata >= 30:
                m = rng.uniform(5.0, 0.8 * ndata)
            else:
                m = rng.uniform(1.5, min(25.0, 1.2 * ndata))
            phi = rng.uniform(-np.pi, np.pi)
            psi = rng.uniform(-0.8, 0.8)
            truth = np.array([a, m, phi, psi])
            qi = analytic_qi(ndata, truth)
            noise = [0.0, 1e-6, 1e-4, 1e-3, 1e-2, 0.05, 0.3][k % 7]
            qi = qi + noise * rng.randn(2 * ndata)
            kind = k % 5
            if kind == 0:
                guess = np.array([1.6, 6.0, 0.0, 0.0])
            elif kind == 1:
                guess = truth * (1 + 0.02 * rng.randn(4))
            elif kind == 2:
                guess = np.array([-a, m, phi + np.pi, psi]) * (1 + 0.01 * rng.randn(4))
            elif kind == 3:
                guess = np.array([a, -m, phi + np.pi, psi]) * (1 + 0.01 * rng.randn(4))
            else:
                guess = np.array([rng.uniform(0.5, 2), rng.uniform(2, 20), rng.uniform(-3, 3),
                                  rng.uniform(-1, 1)])
            qis.append(qi)
            guesses.append(guess)
            truths.append(truth)
        qis = np.array(qis)
        guesses = np.array(guesses)
        status = np.zeros(count, np.int32)
        p = np.zeros((count, 4))
        ssq = np.zeros(count)
        for i in range(count):
            s, pp, q = rfit.fit(ndata, qis[i].copy(), guesses[i].copy())
            status[i], p[i], ssq[i] = s, pp, q
        groups[ndata] = dict(qi=qis, guess=guesses, truth=np.array(truths), status=status, p=p, ssq=ssq,
                             fuzz=reference_fuzz(rfit, ndata, qis, guesses, p),
                             radius=reference_radius(rfit, ndata, qis, p))
    # A few hand-made edge vectors at ndata=10: all-zero data, a=0 guess, m=0 guess
    ndata = 10
    edge_qi = [np.zeros(20), analytic_qi(10, [1.0, 6.0, 0.3, 0.1]), analytic_qi(10, [1.0, 6.0, 0.3, 0.1]),
               analytic_qi(10, [1.2, 0.5, -2.0, 0.0]), analytic_qi(10, [1.0, 28.0, 1.0, 0.2])]
    edge_guess = [np.array([1.6, 6.0, 0.0, 0.0]), np.array([0.0, 6.0, 0.0, 0.0]),
                  np.array([1.6, 0.0, 0.0, 0.0]), np.array([1.6, 6.0, 0.0, 0.0]),
                  np.array([1.6, 6.0, 0.0, 0.0])]
    es, ep, eq = [], [], []
    for qi, g in zip(edge_qi, edge_guess):
        s, pp, q = rfit.fit(ndata, qi.copy(), g.copy())
        es.append(s), ep.append(pp), eq.append(q)
    groups["edge10"] = dict(qi=np.array(edge_qi), guess=np.array(edge_guess), truth=np.zeros((5, 4)),
                            status=np.array(es, np.int32), p=np.array(ep), ssq=np.array(eq),
                            fuzz=reference_fuzz(rfit, ndata, np.array(edge_qi), np.array(edge_guess), np.array(ep)),
                            radius=reference_radius(rfit, ndata, np.array(edge_qi), np.array(ep)))
    out = {}
    for key, g in groups.items():
        for name, arr in g.items():
            out[f"g{key}_{name}"] = arr
    np.savez_compressed(os.path.join(HERE, "lm_vectors.npz"), **out)
    return {"groups": [str(k) for k in groups]}


# --- snr-mode records -------------------------------------------------------------
# Each record: laser/ifo parameters, n_seconds, snr_db, seed, fit kwargs.
RECORDS = [
    dict(name="config1", m=6.0, f_mod=1000.0, f_samp=200000.0, n_seconds=10.0, snr_db=40.0, seed=0,
         phi=0.0, psi=0.0, n=20, ndata=10, init_m=6.0),
    dict(name="m20_init6", m=20.0, f_mod=1000.0, f_samp=200000.0, n_seconds=0.1, snr_db=40.0, seed=3,
         phi=0.0, psi=0.0, n=20, ndata=10, init_m=6.0),
    dict(name="snr0", m=6.0, f_mod=1000.0, f_samp=200000.0, n_seconds=0.2, snr_db=0.0, seed=5,
         phi=0.0, psi=0.0, n=20, ndata=10, init_m=6.0),
    dict(name="snrm10", m=6.0, f_mod=1000.0, f_samp=200000.0, n_seconds=0.2, snr_db=-10.0, seed=6,
         phi=0.0, psi=0.0, n=20, ndata=10, init_m=6.0),
    dict(name="quick_nd30", m=31.4, f_mod=1000.0, f_samp=200000.0, n_seconds=0.1, snr_db=40.0, seed=0,
         phi=0.0, psi=0.0, n=20, ndata=30, init_m=6.0),
    dict(name="quick_nd62", m=31.4, f_mod=1000.0, f_samp=200000.0, n_seconds=0.1, snr_db=40.0, seed=0,
         phi=0.0, psi=0.0, n=20, ndata=62, init_m=6.0),
    dict(name="phi1_psi05", m=6.0, f_mod=1000.0, f_samp=200000.0, n_seconds=0.1, snr_db=40.0, seed=7,
         phi=1.0, psi=0.5, n=20, ndata=10, init_m=6.0),
    dict(name="legacy30k", m=6.0, f_mod=400.0, f_samp=30000.0, n_seconds=0.5, snr_db=40.0, seed=8,
         phi=-1.0, psi=-0.1416, n=20, ndata=10, init_m=6.0),
    dict(name="odd_R", m=7.3, f_mod=400.0, f_samp=30000.0, n_seconds=0.21, snr_db=30.0, seed=9,
         phi=0.4, psi=0.2, n=7, ndata=12, init_m=6.0),
    dict(name="nonint_period", m=5.0, f_mod=1500.0, f_samp=200000.0, n_seconds=0.079981, snr_db=40.0, seed=10,
         phi=2.0, psi=-0.3, n=20, ndata=10, init_m=6.0),
    dict(name="ragged_tail", m=6.0, f_mod=1000.0, f_samp=200000.0, n_seconds=0.1, snr_db=40.0, seed=11,
         phi=0.0, psi=0.0, n=20, ndata=10, init_m=6.0),
]


def build_sim(dfm, rec):
    from scipy.constants import c, pi
    laser = dfm.LaserConfig(label="laser")
    laser.f_mod = rec["f_mod"]
    laser.psi = rec["psi"]
    ifo = dfm.InterferometerConfig(label="ifo")
    ifo.phi = rec["phi"]
    opd = abs(ifo.meas_arml - ifo.ref_arml)
    laser.df = (rec["m"] * c) / (2 * pi * opd)  # helpers.set_laser_df_for_effect
    sim = dfm.DFMIObject(label=rec["name"], laser_config=laser, ifo_config=ifo, f_samp=rec["f_samp"])
    return sim


def df_to_arrays(df):
    return {k: df[k].to_numpy() for k in ["amp", "m", "phi", "psi", "dc", "ssq", "fitok"]}


def make_records(dfm, rfit, rfitters):
    manifest = []
    out = {}
    for rec in RECORDS:
        dff = dfm.DeepFitFramework()
        sim = build_sim(dfm, rec)
        dff.load_sim(sim)
        dff.simulate(rec["name"], n_seconds=rec["n_seconds"], mode="snr", snr_db=rec["snr_db"],
                     trial_num=rec["seed"])
        raw = dff.raws[rec["name"]]
        x = raw.data["ch0"].to_numpy()
        R, fs, nbuf = dff.fit_init(rec["name"], rec["n"])
        entry = dict(rec)
        entry.update(N=int(x.size), R=int(R), fs=float(fs), nbuf=int(nbuf), sha256=sha(x),
                     df=float(sim.laser.df), m_eff=float(sim.m))
        name = rec["name"]
        if rec["name"] == "ragged_tail":
            # Drop 123 samples so N % R != 0: reference raises ValueError on reshape
            # (fitters.py:375/412). Record only that fact.
            x2 = x[:-123]
            entry.update(N_trunc=int(x2.size), sha256_trunc=sha(x2))
            raw.data = raw.data.iloc[:-123]
            errs = []
            for par in (False, True):
                try:
                    rfitters.StandardNLSFitter({"n": rec["n"]}).fit(raw, parallel=par, ndata=rec["ndata"],
                                                                  n_cores=2)
                    errs.append("none")
                except ValueError as e:
                    errs.append("ValueError")
            entry["errors"] = errs
            manifest.append(entry)
            continue
        # Demodulated QI and dc of every buffer (fit.py:18-66; fitters.py:45-57)
        w0 = 2.0 * np.pi * raw.f_mod / raw.f_samp
        bufs = x[: nbuf * R].reshape(nbuf, R)
        nd = rec["ndata"]
        qi = np.zeros((nbuf, 2 * nd))
        for b in range(nbuf):
            for n in range(nd):
                Q, I = rfit.calculate_quadratures(n, bufs[b], w0)
                qi[b, n] = Q.mean()
                qi[b, n + nd] = I.mean()
        dc = bufs.mean(axis=1)
        out[f"{name}_qi"] = qi
        out[f"{name}_dc"] = dc
        kw = dict(ndata=nd, init_m=rec["init_m"])
        # (i) sequential: fitters.py:370-393
        seq = rfitters.StandardNLSFitter({"n": rec["n"]}).fit(raw, parallel=False, **kw)
        for k, v in df_to_arrays(seq).items():
            out[f"{name}_seq_{k}"] = v
        # (ii) parallel with chunk size 1 (every buffer seeded from buffer 0): fitters.py:395-428
        fitter = rfitters.StandardNLSFitter({"n": rec["n"]})
        seed_guess = np.array([1.6, rec["init_m"], 0.0, 0.0])
        first = fitter._fit_single_buffer(raw, 0, R, nd, seed_guess)
        seed = np.array([first["amp"], first["m"], first["phi"], first["psi"]])
        rows = [first]
        for b in range(1, nbuf):
            rows.extend(rfitters._process_fit_chunk((bufs[b:b + 1], seed, R, nd, raw.f_mod, raw.f_samp)))
        import pandas as pd
        c1 = pd.DataFrame(rows)
        for k, v in df_to_arrays(c1).items():
            out[f"{name}_c1_{k}"] = v
        # (iii) the reference's own parallel path with n_cores=4 (array_split chunks)
        if nbuf > 2:
            # NB: passing init_m together with parallel=True raises TypeError in the reference
            # (fitters.py:366 forwards **kwargs that still hold init_m); every record uses the
            # default init_m=6.0, so it is omitted here.
            assert rec["init_m"] == 6.0
            par = rfitters.StandardNLSFitter({"n": rec["n"]}).fit(raw, parallel=True, n_cores=4, ndata=nd)
            for k, v in df_to_arrays(par).items():
                out[f"{name}_par4_{k}"] = v
        # (iv) the drop-in facade: DeepFitFramework.fit (core.py:424-517) incl. tau/time
        fobj = dff.fit(rec["name"], n=rec["n"], parallel=False, **kw)
        out[f"{name}_facade_tau"] = fobj.tau
        out[f"{name}_facade_time"] = fobj.time
        entry["facade"] = dict(R=int(fobj.R), fs=float(fobj.fs), nbuf=int(fobj.nbuf), n=int(fobj.n),
                               ndata=int(fobj.ndata), init_a=float(fobj.init_a), init_m=float(fobj.init_m))
        manifest.append(entry)
    np.savez_compressed(os.path.join(HERE, "records.npz"), **out)
    return manifest


def make_asd_pair(dfm):
    """Config 3: main (dynamic, m=6) + witness (m=4.3) sharing one laser, asd mode with
    all noise ASDs zero (no pyplnoise needed).  notebooks/0.1_quickstart-2-ch.ipynb."""
    import scipy.constants as sc
    dff = dfm.DeepFitFramework()
    laser = dfm.LaserConfig(label="main_laser")
    laser.f_mod = 1000
    ifo = dfm.InterferometerConfig(label="dynamic_ifo")
    ifo.ref_arml, ifo.meas_arml = 0.1, 0.3
    ifo.arml_mod_f, ifo.arml_mod_amp = 1.0, 1e-9
    opd = ifo.meas_arml - ifo.ref_arml
    laser.df = (6.0 * sc.c) / (2 * np.pi * opd)
    main = dfm.DFMIObject(label="dynamic_channel", laser_config=laser, ifo_config=ifo, f_samp=int(200e3))
    dff.sims["dynamic_channel"] = main
    dff.create_witness_channel(main_channel_label="dynamic_channel", witness_channel_label="reference_channel",
                               m_witness=4.3)
    dff.simulate(main_label="dynamic_channel", witness_label="reference_channel", n_seconds=0.06)
    out = {}
    meta = {}
    for key in ["dynamic_channel", "reference_channel"]:
        raw = dff.raws[key]
        out[f"{key}_x"] = raw.data["ch0"].to_numpy()
        fobj = dff.fit(key, fit_label=f"fit_{key}", n=20, parallel=False)
        for k in ["amp", "m", "phi", "psi", "dc", "ssq", "tau", "time"]:
            out[f"{key}_{k}"] = getattr(fobj, k)
        df = dff.fits_df[f"fit_{key}"]
        out[f"{key}_fitok"] = df["fitok"].to_numpy()
        meta[key] = dict(f_samp=float(raw.f_samp), f_mod=float(raw.f_mod), df=float(raw.sim.laser.df),
                         m_eff=float(raw.sim.m))
    np.savez_compressed(os.path.join(HERE, "asd_pair.npz"), **out)
    return meta


def make_ekf(dfm):
    dff = dfm.DeepFitFramework()
    rec = dict(name="ekf", m=6.0, f_mod=1000.0, f_samp=200000.0, n_seconds=0.05, snr_db=40.0, seed=1,
               phi=0.0, psi=0.0, n=20)
    sim = build_sim(dfm, rec)
    dff.load_sim(sim)
    dff.simulate("ekf", n_seconds=rec["n_seconds"], mode="snr", snr_db=rec["snr_db"], trial_num=rec["seed"])
    raw = dff.raws["ekf"]
    x = raw.data["ch0"].to_numpy()
    out = {}
    f1 = dff.fit("ekf", method="ekf", fit_label="ekf_default", n=20, verbose=False)
    f2 = dff.fit("ekf", method="ekf", fit_label="ekf_tuned", n=20, verbose=False,
                 Q_diag=[1e-9, 1e-9, 1e-7, 1e-7, 1e-9], R_val=0.001)
    for lab in ["ekf_default", "ekf_tuned"]:
        df = dff.fits_df[lab]
        for k in ["amp", "m", "phi", "psi", "dc", "ssq", "fitok"]:
            out[f"{lab}_{k}"] = df[k].to_numpy()
    np.savez_compressed(os.path.join(HERE, "ekf.npz"), **out)
    rec.update(N=int(x.size), sha256=sha(x), df=float(sim.laser.df))
    return rec


def main():
    import scipy
    dfm, rfit, rfitters = _import_reference()
    manifest = {
        "generator": "tests/golden/make_golden.py",
        "reference": "/root/reference (mdovale/DeepFMKit @ 2025-07-18, read-only)",
        "numpy": np.__version__, "scipy": scipy.__version__,
        "fit_constants": {k: getattr(rfit, k) for k in
                          ["NPARMS", "MAX_LMA_STEPS", "LMA_CONVERGENCE_IMPROVE", "LMA_CONVERGENCE_PARAM_CHANGE",
                           "FITOK_THRESHOLD", "M_GRID_MIN", "M_GRID_MAX", "M_GRID_STEP",
                           "BESSEL_AMP_THRESHOLD", "SINCOS_AMP_THRESHOLD"]},
    }
    manifest["bessel"] = make_bessel(rfit)
    manifest["lm_vectors"] = make_lm_vectors(rfit)
    manifest["records"] = make_records(dfm, rfit, rfitters)
    manifest["asd_pair"] = make_asd_pair(dfm)
    manifest["ekf"] = make_ekf(dfm)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote fixtures to", HERE)


if __name__ == "__main__":
    main()
