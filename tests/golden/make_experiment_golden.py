"""Golden fixtures for Experiment.run (reference experiments.py:288-458 with
factories.py), generated HERE by running the read-only reference (its own
multiprocessing.Pool) on the sweeps of experiment_spec.py. Stored: every analysis'
all_trials grid (tests/golden/experiment.npz) and the run metadata (experiment.json).

Usage: python tests/golden/make_experiment_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import experiment_spec as S  # noqa: E402
from make_golden import _import_reference  # noqa: E402

_import_reference()
import DeepFMKit.experiments as rexp  # noqa: E402
import DeepFMKit.factories as rfac  # noqa: E402
import DeepFMKit.physics as rphys  # noqa: E402
import DeepFMKit.waveforms as rwf  # noqa: E402


class NoisyFactory(rfac.ExperimentFactory):  # module level: the reference's Pool pickles it
    def _get_expected_params_keys(self):
        return set(S.NOISY_KEYS)

    def __call__(self, params):
        return S.noisy_config(rphys, params)


def main():
    out, meta = {}, {}
    exp = rexp.Experiment("golden noisy")
    S.setup_noisy(exp, NoisyFactory())
    np.random.seed(S.SEED)
    res = exp.run(n_cores=4)
    for k, v in S.flatten(res).items():
        out["noisy/" + k] = v
    exp = rexp.Experiment("golden witness")
    S.setup_witness(exp, rfac.StandardWDFMIExperimentFactory(rwf.second_harmonic_distortion))
    np.random.seed(S.SEED)
    res = exp.run(n_cores=4)
    for k, v in S.flatten(res).items():
        out["witness/" + k] = v
    np.savez_compressed(os.path.join(HERE, "experiment.npz"), **out)
    meta = {"source": "DeepFMKit.experiments.Experiment.run (experiments.py:288-458), factories.py",
            "spec": "tests/golden/experiment_spec.py", "seed": S.SEED, "numpy": np.__version__,
            "keys": sorted(out)}
    with open(os.path.join(HERE, "experiment.json"), "w") as f:
        json.dump(meta, f, indent=1)
    for k in sorted(out):
        print(k, out[k].ravel()[:4])


if __name__ == "__main__":
    main()
