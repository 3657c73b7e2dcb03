"""Declarative Monte-Carlo experiments (reference experiments.py), batched on the GPU.

The reference runs every trial as one `multiprocessing.Pool.imap` task
(experiments.py:381-384): `_run_single_trial` (experiments.py:15-88) builds the
trial's physics objects from the factory, simulates an asd-mode record of
`n_fit_buffers_per_trial` modulation cycles, fits it with each analysis
(`DeepFitFramework.fit(..., parallel=False, n=n_fit_buffers_per_trial)`) and keeps
the column means of each fit's DataFrame. `Experiment.run` then aggregates the
trials into (axes..., n_trials) grids with mean / std / min / max / worst.

Here `Experiment.run` keeps that API, the job list (same parameter dicts, the same
stochastic-generator calls in the same order on numpy's global RandomState, the same
trial numbers) and the aggregation, and replaces the Pool:

* every trial's record is generated ON THE GPU in one `dfmi_synth_asd` launch per
  group of equal-length trials (physics.synthesize_asd_trials; the default cosine or
  the second-harmonic distortion waveform with white or zero noise — other trials use
  the host generator), witness channels included;
* each analysis fits ALL trials in one engine call: 'nls' as the records of one
  `dfmi_nls_record` (per-trial seed, _fit_sequential semantics), 'ekf' as the lanes
  of one `dfmi_ekf_fit`, the witness methods as the records of one `dfmi_wdfmi_fit`
  per distinct fitter configuration; any other method falls back to the reference's
  per-trial path (an in-process DeepFitFramework per trial, still on the GPU);
* the per-trial DataFrame means are formed as pandas does.

`run(engine="loop")` runs the reference's per-trial path for every trial (one
DeepFitFramework per trial, host generator): the batched engine must agree with it.
"""
from __future__ import annotations

import copy
import itertools
import logging
import os
import pickle
from typing import Any, Callable, Dict, List, Optional, Union

import numpy as np
import pandas as pd

from . import core as dfm
from . import fitters as _fitters
from .data import DeepRawObject
from .factories import ExperimentFactory
from .physics import DFMIObject, SignalGenerator, device_synth_supported, synthesize_asd_trials

log = logging.getLogger(__name__)

_BATCHED = ("nls", "ekf", "wdfmi_nls", "wdfmi_ortho", "wdfmi_seq", "hwdfmi")


def _trial_geometry(laser_config, num_fit_buffers, f_samp):
    """experiments.py:27-38: R = int(f_samp / f_mod) samples per modulation cycle, the
    record is num_fit_buffers * R samples (1 if that is 0), simulated for N / f_samp s."""
    R = int(f_samp / laser_config.f_mod)
    need = num_fit_buffers * R
    if need == 0:
        logging.warning("Calculated num_samples_needed is zero. Setting to 1 to avoid division by zero.")
        need = 1
    return need / f_samp


class _Trial:
    """One job packet after the factory ran: its channels' configurations."""
    __slots__ = ("params", "num", "main", "witness", "n_seconds", "f_samp", "x_main", "x_wit")

    def __init__(self, params, num, configs, num_fit_buffers, f_samp):
        self.params, self.num, self.f_samp = params, num, f_samp
        laser = configs["laser_config"]
        self.main = DFMIObject(label="main", laser_config=laser, ifo_config=configs["main_ifo_config"], f_samp=f_samp)
        self.witness = None
        if "witness_ifo_config" in configs:
            self.witness = DFMIObject(label="witness", laser_config=laser, ifo_config=configs["witness_ifo_config"],
                                      f_samp=f_samp)
        self.n_seconds = _trial_geometry(laser, num_fit_buffers, f_samp)
        self.x_main = self.x_wit = None


class _Raw:
    """The fields of a DeepRawObject the fitters read, over an array/tensor already
    synthesised (host numpy or a CUDA tensor row)."""

    def __init__(self, x, sim):
        self._x, self.sim = x, sim
        self.f_samp, self.f_mod, self.label = sim.f_samp, sim.laser.f_mod, sim.label

    def samples(self):
        return self._x

    def n_samples(self):
        return int(self._x.shape[0])


def _frame_means(df):
    """results_df.mean().to_dict() (experiments.py:80-83)."""
    return df.mean().to_dict()


def _trial_means(cols, names, ntrial, nbuf):
    """_frame_means of each trial's nbuf-row frame with the columns `names` (cols: one
    (ntrial * nbuf,) array per column, trial-major). One row per trial (the Experiment
    default: the record is one buffer of n_fit_buffers cycles): the mean of one value is
    that value (as float), no DataFrame needed."""
    if nbuf == 1:
        arrs = [np.asarray(c, dtype=np.float64) for c in cols]
        return [{k: float(a[j]) for k, a in zip(names, arrs)} for j in range(ntrial)]
    return [_frame_means(pd.DataFrame({k: np.asarray(c)[j * nbuf:(j + 1) * nbuf] for k, c in zip(names, cols)},
                                      columns=names)) for j in range(ntrial)]


def _synthesize(trials):
    """Every trial's channels: the GPU generator for the trials it covers (grouped by
    record length), the host generator (physics.SignalGenerator) for the rest."""
    groups: Dict[tuple, List[_Trial]] = {}
    for t in trials:
        dev = device_synth_supported(t.main) and (t.witness is None or device_synth_supported(t.witness))
        groups.setdefault((t.f_samp, t.n_seconds, dev, t.witness is not None), []).append(t)
    for (f_samp, n_seconds, dev, wit), ts in groups.items():
        if dev:
            xm = synthesize_asd_trials([t.main for t in ts], [t.num for t in ts], n_seconds, dynamic=True)
            xw = synthesize_asd_trials([t.witness for t in ts], [t.num for t in ts], n_seconds,
                                       dynamic=False) if wit else None
            for i, t in enumerate(ts):
                t.x_main = xm[i]
                t.x_wit = xw[i] if wit else None
        else:
            for t in ts:
                ch = SignalGenerator().generate(t.main, n_seconds, mode="asd", trial_num=t.num, witness_config=t.witness)
                t.x_main = np.asarray(ch["main"].samples(), dtype=np.float64)
                t.x_wit = np.asarray(ch["witness"].samples(), dtype=np.float64) if t.witness is not None else None


def _tau_col(m, df):
    return m / (2 * np.pi * df)


def _stack(xs):
    if hasattr(xs[0], "is_cuda"):
        import torch
        return torch.stack(xs).contiguous()
    return np.ascontiguousarray(np.stack(xs))


def _fit_loop_one(t: _Trial, analysis, num_fit_buffers):
    """_run_single_trial's fit of one analysis (experiments.py:62-86) over the trial's
    synthesised record: one DeepFitFramework, as the reference worker builds it."""
    dff = dfm.DeepFitFramework()
    dff.sims["main"] = t.main
    raw = DeepRawObject(data=pd.DataFrame({"ch0": _host(t.x_main)}))
    raw.label, raw.f_samp, raw.f_mod, raw.sim, raw.t0 = "main", t.f_samp, t.main.laser.f_mod, t.main, 0
    dff.raws["main"] = raw
    if t.witness is not None:
        dff.sims["witness"] = t.witness
        w = DeepRawObject(data=pd.DataFrame({"ch0": _host(t.x_wit)}))
        w.label, w.f_samp, w.f_mod, w.sim, w.t0 = "witness", t.f_samp, t.witness.laser.f_mod, t.witness, 0
        dff.raws["witness"] = w
    args = copy.deepcopy(analysis.get("fitter_kwargs", {}))
    args.update({"method": analysis["fitter_method"], "main_label": "main"})
    if analysis["fitter_method"] in ("nls", "ekf"):
        args["parallel"] = False
    if "wdfmi" in analysis["fitter_method"] or "hwdfmi" in analysis["fitter_method"]:
        args["witness_label"] = "witness" if t.witness is not None else None
    args["n"] = num_fit_buffers
    fit_obj = dff.fit(**args)
    if fit_obj:
        return _frame_means(dff.fits_df[fit_obj.label])
    return {}


def _host(x):
    return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)


def _fit_batched(trials: List[_Trial], analysis, num_fit_buffers):
    """One analysis over all trials, one engine call per group of trials that share
    the fit geometry (and, for the witness methods, the fitter configuration)."""
    method = analysis["fitter_method"]
    kw = copy.deepcopy(analysis.get("fitter_kwargs", {}))
    kw.pop("n", None)  # experiments.py:78 overrides it
    out: List[Optional[dict]] = [None] * len(trials)
    if method not in _BATCHED or ("wdfmi" in method and any(t.witness is None for t in trials)):
        for i, t in enumerate(trials):
            out[i] = _fit_loop_one(t, analysis, num_fit_buffers)
        return out
    n = num_fit_buffers
    groups: Dict[tuple, List[int]] = {}
    for i, t in enumerate(trials):
        f_mod = t.main.laser.f_mod
        key = (t.f_samp, f_mod, int(t.x_main.shape[0]))
        if "wdfmi" in method:
            key += _wdfmi_key(method, t, kw)
        groups.setdefault(key, []).append(i)
    for key, idx in groups.items():
        f_samp, f_mod, N = key[:3]
        R = int(f_samp / f_mod * n)  # fit_init, core.py:390-422
        nbuf = int(N / R) if R > 0 else 0
        if nbuf == 0:
            logging.error("Check buffer size !! Calculated nbuf is zero.")
            for i in idx:
                out[i] = {}
            continue
        ts = [trials[i] for i in idx]
        if method == "nls":
            if N % R != 0:  # _fit_sequential's reshape(-1, R) (fitters.py:375)
                raise ValueError(f"cannot reshape array of size {N} into shape ({R})")
            g = (kw.get("init_a", 1.6), kw.get("init_m", 6.0), 0.0, kw.get("init_psi", 0.0))
            cols, ok = _fitters.nls_records(_stack([t.x_main for t in ts]), f_samp, f_mod, R, nbuf,
                                            int(kw.get("ndata", 10)), g, parallel=False)
            cols, ok = _host(cols), _host(ok)
            dfs = np.repeat(np.array([trials[i].main.laser.df for i in idx], dtype=np.float64), nbuf)
            names = _fitters.COLUMNS + ["tau"]
            means = _trial_means([cols[0], cols[1], cols[2], cols[3], cols[4], cols[5], ok.astype(np.int64),
                                  _tau_col(cols[1], dfs)], names, len(idx), nbuf)
            for j, i in enumerate(idx):
                out[i] = means[j]
        elif method == "ekf":
            raws = [_Raw(_host(t.x_main), t.main) for t in ts]
            states = _fitters.ekf_records(raws, n, **{k: v for k, v in kw.items() if k != "parallel"})
            st = states.reshape(-1, 5)
            dfs = np.repeat(np.array([trials[i].main.laser.df for i in idx], dtype=np.float64), nbuf)
            means = _trial_means([st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4], np.zeros(st.shape[0]),
                                  np.ones(st.shape[0], dtype=np.int64), _tau_col(st[:, 1], dfs)],
                                 _fitters.COLUMNS + ["tau"], len(idx), nbuf)
            for j, i in enumerate(idx):
                out[i] = means[j]
        else:
            wkw = dict(zip(("df", "f_ref", "tau_init", "ndata", "init_a", "init_phi", "init_psi"), key[3:]))
            mains = _stack([t.x_main[: nbuf * R] for t in ts])
            wits = _stack([t.x_wit[:R] for t in ts])
            cols, ok = _fitters.wdfmi_records(method, mains, wits, f_samp, f_mod, R, nbuf, **wkw)
            cols, ok = _host(cols), _host(ok)
            means = _trial_means([cols[k] for k in range(7)] + [ok.astype(np.int64)], _fitters.WDFMI_COLUMNS,
                                 len(idx), nbuf)
            for j, i in enumerate(idx):
                out[i] = means[j]
    return out


def _wdfmi_key(method, t: _Trial, kw):
    """The witness fitters' per-call configuration, as fitters.py:481-891 derive it
    from the trial's channels (fitters._WitnessFitter and subclasses)."""
    import scipy.constants as sc
    laser, ifo = t.main.laser, t.main.ifo
    if method == "wdfmi_nls":
        tau = (ifo.meas_arml - ifo.ref_arml) / sc.c
        return (laser.df, 0.0, tau, 10, kw.get("init_a", 1.6), kw.get("init_phi", 0.0), kw.get("init_psi", 0.0))
    if method == "hwdfmi":
        f_ref = getattr(t.witness.ifo, "arml_mod_f", 0.0)
        tau = kw.get("init_tau", None)
        if tau is None:
            tau = (ifo.meas_arml - ifo.ref_arml) / sc.c
        return (laser.df, f_ref, tau, 10, 1.6, 0.0, 0.0)
    tau = (ifo.meas_arml - ifo.ref_arml) / sc.c if laser.df > 0 else 0.0
    return (laser.df, 0.0, tau, 10, 1.6, 0.0, kw.get("init_psi", 0.0))


class Experiment:
    """experiments.py:90-458 (run batched on the GPU; see the module docstring)."""

    def __init__(self, description: str = "Unnamed Experiment", filename: Optional[str] = None):
        self.description = description
        self.axes: Dict[str, np.ndarray] = {}
        self.static_params: Dict[str, Any] = {}
        self.stochastic_vars: Dict[str, Dict[str, Any]] = {}
        self.config_factory: Optional[ExperimentFactory] = None
        self._expected_params_keys: set = set()
        self.analyses: List[Dict[str, Any]] = []
        self.n_trials: int = 1
        self.n_fit_buffers_per_trial: int = 10
        self.f_samp: int = 200000
        self.results: Optional[Dict[str, Any]] = None
        if filename is not None:
            self.load_results(filename)

    # --- definition (experiments.py:127-186) ---------------------------------
    def _validate_param_name(self, name: str):
        if not self._expected_params_keys:
            logging.warning("No config factory set yet. Parameter validation will be skipped until "
                            "set_config_factory() is called.")
            return
        if name not in self._expected_params_keys:
            raise ValueError(
                f"Parameter '{name}' is not recognized by the current ExperimentFactory "
                f"({type(self.config_factory).__name__}).\nExpected parameters are: "
                f"{sorted(list(self._expected_params_keys))}.\nPlease update your ExperimentFactory to handle this "
                f"parameter or remove it from your experiment configuration.")

    def add_axis(self, name: str, values: np.ndarray):
        self._validate_param_name(name)
        self.axes[name] = np.asarray(values)

    def set_static(self, params: Dict[str, Any]):
        for name in params.keys():
            self._validate_param_name(name)
        self.static_params.update(params)

    def add_stochastic_variable(self, name: str, generator_func: Callable, depends_on: Optional[str] = None):
        self._validate_param_name(name)
        if depends_on is not None:
            self._validate_param_name(depends_on)
        self.stochastic_vars[name] = {"generator": generator_func, "depends_on": depends_on}

    def set_config_factory(self, factory: ExperimentFactory):
        if not isinstance(factory, ExperimentFactory):
            raise TypeError("factory must be an instance of a class that inherits from ExperimentFactory.")
        self.config_factory = factory
        self._expected_params_keys = self.config_factory._get_expected_params_keys()

    def add_analysis(self, name: str, fitter_method: str, result_cols: Optional[List[str]] = None,
                     fitter_kwargs: Optional[Dict[str, Any]] = None):
        self.analyses.append({"name": name, "fitter_method": fitter_method, "result_cols": result_cols,
                              "fitter_kwargs": fitter_kwargs or {}})

    def _filter(self, params):
        return {k: v for k, v in params.items() if k in self._expected_params_keys or k.startswith("_exp_")}

    def _draw_stochastic(self, params):
        for var_name, info in self.stochastic_vars.items():
            dep = info.get("depends_on")
            params[var_name] = info["generator"](params[dep]) if dep else info["generator"]()

    def get_params_for_point(self, axis_idx: Union[int, tuple]) -> Dict[str, Any]:
        """experiments.py:187-277: the point's parameters, stochastic values drawn under
        np.random.seed(0) with the global state restored afterwards."""
        params = copy.deepcopy(self.static_params)
        axis_names = list(self.axes.keys())
        if isinstance(axis_idx, int):
            axis_idx = (axis_idx,)
        if len(axis_idx) != len(axis_names):
            raise ValueError(f"Dimension of axis_idx ({len(axis_idx)}) does not match the number "
                             f"of defined axes ({len(axis_names)}).")
        for i, axis_name in enumerate(axis_names):
            params[axis_name] = self.axes[axis_name][axis_idx[i]]
        state = np.random.get_state()
        np.random.seed(0)
        try:
            for var_name, info in self.stochastic_vars.items():
                dep = info.get("depends_on")
                if dep and dep not in params:
                    raise ValueError(f"Stochastic variable '{var_name}' depends on '{dep}', which is not a defined "
                                     f"axis or static parameter.")
                params[var_name] = info["generator"](params[dep]) if dep else info["generator"]()
        finally:
            np.random.set_state(state)
        return self._filter(params)

    def save_results(self, filename: str):
        if self.results is None:
            raise RuntimeError("No results to save. Run the experiment first.")
        with open(filename, "wb") as f:
            pickle.dump(self.results, f)

    def load_results(self, filename: str):
        """Results files this class wrote (pickle, as the reference's save_results)."""
        with open(filename, "rb") as f:
            self.results = pickle.load(f)

    # --- execution ------------------------------------------------------------
    def _job_list(self):
        """experiments.py:326-375: every grid point x n_trials, in itertools.product
        order, stochastic variables drawn per trial in definition order."""
        axis_names = list(self.axes.keys())
        jobs = []
        counter = 0
        for point in itertools.product(*[range(len(ax)) for ax in self.axes.values()]):
            point_params = copy.deepcopy(self.static_params)
            for i, name in enumerate(axis_names):
                point_params[name] = self.axes[name][point[i]]
            for j in range(self.n_trials):
                tp = copy.deepcopy(point_params)
                tp["_exp_point_idx"] = point
                tp["_exp_trial_idx"] = j
                self._draw_stochastic(tp)
                jobs.append((self._filter(tp), counter))
                counter += 1
        return jobs

    def run(self, n_cores: Optional[int] = None, filename: Optional[str] = None, engine: str = "gpu"
            ) -> Dict[str, Any]:
        """experiments.py:288-458. engine "gpu": batched synthesis + one fit call per
        analysis (module docstring); "loop": the reference's per-trial path (host
        generator, one DeepFitFramework per trial). n_cores is accepted for drop-in
        compatibility (no process pool: the GPU batch replaces it)."""
        if self.config_factory is None:
            raise ValueError("A configuration factory must be set using set_config_factory().")
        if not self.axes and not self.n_trials > 0:
            raise ValueError("At least one parameter axis must be defined using add_axis(), or n_trials must be > 0.")
        if engine not in ("gpu", "loop"):
            raise ValueError("engine must be 'gpu' or 'loop'")
        jobs = self._job_list()
        trials = [_Trial(p, num, self.config_factory(p), self.n_fit_buffers_per_trial, self.f_samp)
                  for p, num in jobs]
        per_analysis: Dict[str, List[dict]] = {}
        if engine == "gpu":
            _synthesize(trials)
            for a in self.analyses:
                per_analysis[a["name"]] = _fit_batched(trials, a, self.n_fit_buffers_per_trial)
        else:
            for t in trials:
                ch = SignalGenerator().generate(t.main, t.n_seconds, mode="asd", trial_num=t.num,
                                                witness_config=t.witness)
                t.x_main = np.asarray(ch["main"].samples(), dtype=np.float64)
                t.x_wit = np.asarray(ch["witness"].samples(), dtype=np.float64) if t.witness is not None else None
            for a in self.analyses:
                per_analysis[a["name"]] = [_fit_loop_one(t, a, self.n_fit_buffers_per_trial) for t in trials]
        flat = [{"point_params": t.params, "results": {a["name"]: per_analysis[a["name"]][k] for a in self.analyses}}
                for k, t in enumerate(trials)]
        self.results = self._aggregate(flat)
        if filename is not None:
            self.save_results(filename)
        return self.results

    def _aggregate(self, flat_results):
        """experiments.py:386-447."""
        axis_names = list(self.axes.keys())
        results = {"axes": self.axes}
        shape = (self.n_trials,) if not axis_names else tuple(len(ax) for ax in self.axes.values()) + (self.n_trials,)
        for analysis in self.analyses:
            name = analysis["name"]
            results[name] = {}
            cols = analysis.get("result_cols")
            if cols is None:
                keys = set()
                for pk in flat_results:
                    if name in pk["results"]:
                        keys.update(pk["results"][name].keys())
                cols = sorted(list(keys))
            for col in cols:
                results[name][col] = {"all_trials": np.full(shape, np.nan, dtype=float)}
        for pk in flat_results:
            point_idx = pk["point_params"]["_exp_point_idx"]
            trial_idx = pk["point_params"]["_exp_trial_idx"]
            full_idx = (trial_idx,) if not axis_names else point_idx + (trial_idx,)
            for analysis in self.analyses:
                name = analysis["name"]
                if name in pk["results"]:
                    for col, stats in results[name].items():
                        stats["all_trials"][full_idx] = pk["results"][name].get(col, np.nan)
        for name, res in results.items():
            if name == "axes":
                continue
            for col, stats in res.items():
                a = stats["all_trials"]
                stats["mean"] = np.nanmean(a, axis=-1)
                stats["std"] = np.nanstd(a, axis=-1)
                stats["min"] = np.nanmin(a, axis=-1)
                stats["max"] = np.nanmax(a, axis=-1)
                dev = np.abs(a - stats["mean"][..., np.newaxis])
                worst = np.nanargmax(dev, axis=-1)
                stats["worst"] = np.take_along_axis(a, worst[..., np.newaxis], axis=-1).squeeze(-1)
        return results

    def plot(self, *args, **kwargs):
        raise NotImplementedError("plotting is out of scope for deepfmkit_amd (DESIGN.md §9)")


def cpu_count():
    return os.cpu_count()
