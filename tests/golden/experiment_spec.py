"""Shared definition of the golden Experiment sweeps (reference experiments.py /
factories.py), used by make_experiment_golden.py (against the reference package) and
by tests/test_gpu_experiments.py (against deepfmkit_amd). Data only plus a factory body
parameterised by the physics module, so both sides build identical configurations."""
import numpy as np
import scipy.constants as sc

SEED = 1234  # np.random.seed before Experiment.run: the stochastic draws happen in the parent


def noisy_config(physics, params):
    """Experiment A: white amplitude noise (amp_n, alpha = 0: no pyplnoise), OPD 0.1 m,
    interferometer phase from the stochastic variable 'phi'."""
    laser = physics.LaserConfig()
    laser.amp_n = params["amp_noise"]
    laser.df = (params["m_main"] * sc.c) / (2 * np.pi * 0.1)
    ifo = physics.InterferometerConfig(label="main_ifo")
    ifo.ref_arml = 0.1
    ifo.meas_arml = 0.2
    ifo.phi = params["phi"]
    return {"laser_config": laser, "main_ifo_config": ifo}


NOISY_KEYS = {"m_main", "amp_noise", "phi"}


def phi_generator():
    return np.random.uniform(0.0, 2 * np.pi)


def setup_noisy(exp, factory):
    """2-axis sweep (m_main x amp_noise) x 3 trials, a stochastic phase, three analyses."""
    exp.set_config_factory(factory)
    exp.add_axis("m_main", np.array([4.0, 6.5, 9.0]))
    exp.add_axis("amp_noise", np.array([1e-4, 4e-4]))
    exp.add_stochastic_variable("phi", phi_generator)
    exp.n_trials = 3
    exp.add_analysis("NLS", "nls", fitter_kwargs={"ndata": 10})
    exp.add_analysis("NLS12", "nls", result_cols=["m", "ssq", "fitok"], fitter_kwargs={"ndata": 12, "init_m": 6.0})
    exp.add_analysis("EKF", "ekf", result_cols=["amp", "m", "phi", "psi", "dc"])


def setup_witness(exp, factory):
    """StandardWDFMIExperimentFactory(second_harmonic_distortion): m_main x distortion_amp
    x 2 trials, no noise, NLS and the orthogonal witness fitter."""
    exp.set_config_factory(factory)
    exp.add_axis("m_main", np.array([5.0, 8.0]))
    exp.add_axis("distortion_amp", np.array([0.0, 0.05]))
    exp.set_static({"m_witness": 0.5, "phi": 0.3, "distortion_phase": 0.4})
    exp.n_trials = 2
    exp.add_analysis("NLS", "nls", fitter_kwargs={"ndata": 10})
    exp.add_analysis("ORTHO", "wdfmi_ortho")


def flatten(results):
    """{analysis/col: all_trials} for np.savez / comparison."""
    out = {}
    for name, res in results.items():
        if name == "axes":
            continue
        for col, stats in res.items():
            out[f"{name}/{col}"] = np.asarray(stats["all_trials"], dtype=np.float64)
    return out
