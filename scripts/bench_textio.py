"""§8f-3: the reference's text formats on the host (csrc/textio.cpp), measured against
the reference's own loaders on the same files:

  raw_data, config-1 size (10 s at 200 kS/s = 2,000,000 rows) x `channels` columns:
    load_raw (core.py:279-280): pandas.read_csv(sep=' ', skiprows=13, usecols=[c],
    names=['ch'+str(c)]) once per channel  vs  textio.read_raw (all channels, one pass)
  fit_data, 100,000 rows x 6 columns (config 2's fit of one channel):
    load_fit (core.py:306-330): numpy.genfromtxt(skip_header=13, invalid_raise=False)
    vs textio.read_fit; DeepFitObject.to_txt (data.py:178-208, a Python loop of
    str(float)) restated vs textio.write_fit

Host code only (no GPU). One JSON line: seconds, MB/s, speed-ups, and that every
value equals the reference loader's bit for bit (and the written file its bytes)."""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def best(fn, reps=3):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), r


def main():
    import pandas as pd

    from deepfmkit_amd import textio
    from deepfmkit_amd.data import DeepFitObject

    nch = int(os.environ.get("CHANNELS", 2))
    nrow = int(os.environ.get("ROWS", 2_000_000))
    nfit = int(os.environ.get("FIT_ROWS", 100_000))
    rng = np.random.default_rng(0)
    out = {"metric": "text formats (host)", "threads": textio._threads()}
    with tempfile.TemporaryDirectory() as d:
        raw = os.path.join(d, "raw.txt")
        chans = [1.0 + np.cos(6.0 * np.cos(np.arange(nrow) * (2 * np.pi / 200))) + 1e-3 * rng.standard_normal(nrow)
                 for _ in range(nch)]
        textio.write_raw(raw, chans, 0, 200000.0, 1000.0)
        mb = os.path.getsize(raw) / 1e6
        t_ref, ref = best(lambda: [pd.read_csv(raw, sep=" ", skiprows=13, usecols=[c], names=["ch" + str(c)])
                                   ["ch" + str(c)].to_numpy() for c in range(nch)], reps=2)
        t_ours, (_, ours) = best(lambda: textio.read_raw(raw))
        out["raw"] = {"rows": nrow, "channels": nch, "MB": round(mb, 1), "pandas_s": t_ref, "ours_s": t_ours,
                      "ours_MBps": mb / t_ours, "speedup": t_ref / t_ours,
                      "bit_exact": all(np.array_equal(a, b) for a, b in zip(ours, ref))}

        fo = DeepFitObject()
        fo.label, fo.t0, fo.f_samp, fo.f_mod, fo.n, fo.R, fo.fs = "x", 0, 200000.0, 1000.0, 20, 4000, 50.0
        fo.init_a, fo.init_m = 1.6, 6.0
        for k, scale in (("ssq", 1e-4), ("amp", 1.0), ("m", 6.0), ("phi", 1.0), ("psi", 0.1), ("dc", 1.0)):
            setattr(fo, k, scale * (1 + 1e-3 * rng.standard_normal(nfit)))
        fit = os.path.join(d, "fit.txt")
        fit_ref = os.path.join(d, "fit_ref.txt")

        def to_txt_ref():  # data.py:194-207 restated: header, then a str(float) loop per row
            with open(fit_ref, "w") as f:
                f.write(textio.fit_header_text(fo))
                for i in range(nfit):
                    f.write("".join(str(getattr(fo, k)[i]) + " " for k in ("ssq", "amp", "m", "phi", "psi", "dc"))
                            + "\n")

        t_wref, _ = best(to_txt_ref, reps=1)
        t_w, _ = best(lambda: textio.write_fit(fo, fit))
        same_bytes = open(fit, "rb").read() == open(fit_ref, "rb").read()
        mbf = os.path.getsize(fit) / 1e6
        t_gref, g = best(lambda: np.genfromtxt(fit, skip_header=13, invalid_raise=False), reps=1)
        t_r, (_, arr) = best(lambda: textio.read_fit(fit))
        out["fit"] = {"rows": nfit, "MB": round(mbf, 1), "to_txt_loop_s": t_wref, "write_s": t_w,
                      "write_speedup": t_wref / t_w, "bytes_identical": same_bytes, "genfromtxt_s": t_gref,
                      "read_s": t_r, "read_speedup": t_gref / t_r,
                      "bit_exact": bool(np.array_equal(arr[0], g.T))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
