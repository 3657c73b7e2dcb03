"""Generate the W-DFMI golden fixtures from the reference DeepFMKit (run HERE only).

Imports the read-only reference at /root/reference (never travels to the GPU box),
simulates main + witness channel pairs with the reference's own asd-mode generator
(physics.py:615-722, white amplitude noise only, so pyplnoise is not needed), runs
the four witness-based fitters through DeepFitFramework.fit (core.py:424-517) and
stores inputs and outputs as data in tests/golden/wdfmi.npz:

  <case>_main, <case>_witness       the raw channels (float64)
  <case>_hw_witness                 beat-frequency witness for HWDFMI_Fitter
  <case>_<method>_<col>             amp, m, phi, psi, tau, dc, ssq, fitok per buffer
  <case>_cfg                        [f_samp, f_mod, df, meas_arml, ref_arml, f_ref, n]

Methods: wdfmi_nls (WDFMI_NLSFitter, fitters.py:481-570), wdfmi_ortho
(WDFMI_OrthogonalFitter, 572-648), wdfmi_seq (WDFMI_SequentialFitter, 650-776),
hwdfmi (HWDFMI_Fitter, 778-891).

Usage:  python tests/golden/make_wdfmi_golden.py
Environment: numpy 2.2.6, scipy 1.15.3.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _import_reference  # noqa: E402

COLS = ["amp", "m", "phi", "psi", "tau", "dc", "ssq", "fitok"]

# (name, m_main, m_witness, ifo.phi, laser.psi, waveform distortion, amp_n, n_seconds, fitter kwargs)
CASES = [
    dict(name="cos", m_main=6.0, m_witness=0.5, phi=0.7, psi=0.3, dist=0.0, amp_n=2e-5, n_seconds=0.06,
         nls=dict(init_a=1.0, init_phi=0.0, init_psi=0.3), ortho=dict(init_psi=0.3), seq=dict(init_psi=0.25)),
    dict(name="dist", m_main=20.3, m_witness=0.5, phi=2.0, psi=-0.4, dist=0.05, amp_n=1e-4, n_seconds=0.06,
         nls=dict(init_a=1.0, init_phi=0.0, init_psi=-0.4), ortho=dict(init_psi=-0.35), seq=dict(init_psi=-0.4)),
]


def _second_harmonic(t_phase, distortion_amp=0.0, distortion_phase=0.0):
    return np.cos(t_phase) + distortion_amp * np.cos(2 * t_phase + distortion_phase)


def make_case(dfm, c):
    import scipy.constants as sc
    dff = dfm.DeepFitFramework()
    laser = dfm.LaserConfig(label="laser")
    laser.f_mod = 1000
    laser.psi = c["psi"]
    laser.amp_n = c["amp_n"]
    if c["dist"]:
        laser.waveform_func = _second_harmonic
        laser.waveform_kwargs = {"distortion_amp": c["dist"], "distortion_phase": 0.6}
    ifo = dfm.InterferometerConfig(label="main_ifo")
    ifo.ref_arml, ifo.meas_arml = 0.1, 0.3
    ifo.phi = c["phi"]
    opd = ifo.meas_arml - ifo.ref_arml
    laser.df = (c["m_main"] * sc.c) / (2 * np.pi * opd)
    main = dfm.DFMIObject(label="main", laser_config=laser, ifo_config=ifo, f_samp=int(200e3))
    dff.sims["main"] = main
    dff.create_witness_channel(main_channel_label="main", witness_channel_label="witness",
                               m_witness=c["m_witness"])
    dff.simulate(main_label="main", witness_label="witness", n_seconds=c["n_seconds"])
    x_main = dff.raws["main"].data["ch0"].to_numpy().copy()
    x_wit = dff.raws["witness"].data["ch0"].to_numpy().copy()

    # HW-DFMI witness: the beatnote frequency f_beat(t) = df * g(t) (g the normalised
    # modulation waveform), f_ref from the witness ifo's arml_mod_f (fitters.py:827-831)
    t = np.arange(len(x_main)) / main.f_samp
    g = laser.waveform_func(2 * np.pi * laser.f_mod * t + laser.psi, **laser.waveform_kwargs)
    f_beat = laser.df * g / np.max(np.abs(g)) + 2.5e6
    hw = dfm.DeepRawObject(data=__import__("pandas").DataFrame(f_beat, columns=["ch0"]))
    hw.label, hw.f_samp, hw.f_mod, hw.sim = "hw_witness", main.f_samp, laser.f_mod, dff.sims["witness"]
    dff.raws["hw_witness"] = hw

    out = {f"{c['name']}_main": x_main, f"{c['name']}_witness": x_wit, f"{c['name']}_hw_witness": f_beat}
    f_ref = float(dff.sims["witness"].ifo.arml_mod_f)
    out[f"{c['name']}_cfg"] = np.array([main.f_samp, laser.f_mod, laser.df, ifo.meas_arml, ifo.ref_arml, f_ref, 20.0])
    runs = [("wdfmi_nls", "witness", c["nls"]), ("wdfmi_ortho", "witness", c["ortho"]),
            ("wdfmi_seq", "witness", c["seq"]), ("hwdfmi", "hw_witness", {})]
    for method, wl, kw in runs:
        fobj = dff.fit("main", method=method, fit_label=f"f_{method}", n=20, witness_label=wl, **kw)
        df = dff.fits_df[f"f_{method}"]
        for k in COLS:
            out[f"{c['name']}_{method}_{k}"] = df[k].to_numpy().astype(np.float64)
        print(c["name"], method, {k: df[k].to_numpy()[:3].tolist() for k in ("amp", "m", "phi", "psi", "tau")},
              flush=True)
        assert fobj is not None
    return out


def main():
    dfm, _, _ = _import_reference()
    out = {}
    for c in CASES:
        out.update(make_case(dfm, c))
    np.savez_compressed(os.path.join(HERE, "wdfmi.npz"), **out)
    with open(os.path.join(HERE, "wdfmi_cases.json"), "w") as f:
        json.dump({"cases": CASES, "numpy": np.__version__, "scipy": __import__("scipy").__version__}, f, indent=1)


if __name__ == "__main__":
    main()
