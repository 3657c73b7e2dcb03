"""Golden table of scipy.special.jv (the reference's Bessel, fit.py:3,106-108,160,275-276)
at LARGE arguments: orders 0..17, |x| in [64, 1e4] (both signs) — the range a descent runs
into when it walks away from a guess that cannot reach the data, where the
engine switches from Miller's backward recurrence to the Hankel expansion + upward
recurrence (dfmi_math.h dfmi_bessel_j01_large). scipy 1.15.3 / numpy 2.2.6 here.
Usage: python tests/golden/make_bessel_large.py"""
import os

import numpy as np
from scipy.special import jv

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    rng = np.random.default_rng(2024)
    x = np.concatenate([[64.0, 64.5, 100.0, 886.67583162, 999.0, 5000.0, 9999.0],
                        rng.uniform(64.0, 200.0, 120), rng.uniform(200.0, 10000.0, 120)])
    x = np.concatenate([x, -x[::3]])
    n = np.arange(18)
    np.savez_compressed(os.path.join(HERE, "bessel_large.npz"), n=n, x=x, jv=jv(n[:, None], x[None, :]))
    print("wrote bessel_large.npz", x.size, "arguments")


if __name__ == "__main__":
    main()
