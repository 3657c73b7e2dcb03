"""A/B of two builds of libdfmi.so in ONE process (same box, same clocks, interleaved):
LIBS="name=path;name=path" (default: ab/libdfmi_A.so vs deepfmkit_amd/libdfmi.so).
Each library is loaded with its own ctypes handle (RTLD_LOCAL: its own HIP code object).

Workloads (config-2 shapes unless noted), median of ROUNDS interleaved rounds:
  step      dfmi_nls_record over 100k segments (fused seed + demod + LM), ms per call
  demod     dfmi_demod_rows over the same segments (the bulk demodulation alone)
  lm        dfmi_lm over component-major QI of the same segments (every segment its own chunk)
  seq500    dfmi_nls_record parallel=0 over 500 segments (one warm-start chain, config 1)
  seqall    (SEQALL=1) dfmi_nls_record parallel=0 over all NSEG segments (one chain)
and the outputs' bitwise equality between the libraries (results must not depend on
the build unless the change is meant to move rounding). One JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHI = float(os.environ.get("PHI", 0.0))  # the record's interferometric phase (bench: 0)
PSI = float(os.environ.get("PSI", 0.0))


def main():
    import torch

    import bench
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of
    spec = os.environ.get("LIBS", f"A={ROOT}/ab/libdfmi_A.so;B={ROOT}/deepfmkit_amd/libdfmi.so")
    libs = {}
    for item in spec.split(";"):
        name, path = item.split("=")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        libs[name] = lib
    rounds = int(os.environ.get("ROUNDS", 5))
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream()
    R, nd = 4000, 10
    nseg = int(os.environ.get("NSEG", 100000))
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    x = torch.empty(nseg * R, dtype=torch.float64, device=dev)
    synth_snr(SnrSpec(seed=bench.SEED, f_samp=200000.0, f_mod=1000.0, m=6.0, phi=PHI, psi=PSI, snr_db=40.0), 0,
              nseg * R, out=x)
    w0 = w0_of(1000.0, 200000.0)
    cfg = F.lm_config()
    g = np.array([1.6, 6.0, 0.0, 0.0])
    gd = torch.tensor([1.0, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    P = ctypes.c_void_p
    i64, i32, d = ctypes.c_int64, ctypes.c_int32, ctypes.c_double
    for lib in libs.values():
        lib.dfmi_nls_record.argtypes = [P, i64, i64, i64, i32, i32, d, i32, P, i32, i64, ctypes.POINTER(_lib.LMConfig),
                                        P, P, i32, P]
        lib.dfmi_demod.argtypes = [P, i64, i64, i32, i32, d, i32, P, P, i32, P]
        lib.dfmi_lm.argtypes = [P, i64, i32, P, i32, i64, ctypes.POINTER(_lib.LMConfig), P, P, P, i32, P]
        lib.dfmi_demod_rows.argtypes = [P, i64, i64, i32, i32, d, i32, P, i32, P]
        lib.dfmi_last_error.restype = ctypes.c_char_p
    out = {k: torch.empty((6, nseg), dtype=torch.float64, device=dev) for k in libs}
    ok = {k: torch.empty(nseg, dtype=torch.int32, device=dev) for k in libs}
    qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
    dc = torch.empty(nseg, dtype=torch.float64, device=dev)
    lp = {k: torch.empty((4, nseg), dtype=torch.float64, device=dev) for k in libs}
    ls = {k: torch.empty(nseg, dtype=torch.float64, device=dev) for k in libs}
    lt = {k: torch.empty(nseg, dtype=torch.int32, device=dev) for k in libs}
    s1 = {k: torch.empty((6, 500), dtype=torch.float64, device=dev) for k in libs}
    k1 = {k: torch.empty(500, dtype=torch.int32, device=dev) for k in libs}
    seqall = os.environ.get("SEQALL") == "1"
    sa = {k: torch.empty((6, nseg), dtype=torch.float64, device=dev) for k in libs} if seqall else {}
    ka = {k: torch.empty(nseg, dtype=torch.int32, device=dev) for k in libs} if seqall else {}

    def chk(rc, lib):
        if rc != 0:
            raise RuntimeError(lib.dfmi_last_error().decode())

    def step(k):
        lib = libs[k]
        chk(lib.dfmi_nls_record(x.data_ptr(), 1, nseg * R, nseg, R, nd, w0, 0, g.ctypes.data, 1, nseg - 1, cfg,
                                out[k].data_ptr(), ok[k].data_ptr(), 1, P(st.cuda_stream)), lib)

    def lm(k):
        lib = libs[k]
        chk(lib.dfmi_lm(qi.data_ptr(), nseg, nd, gd.data_ptr(), 0, nseg, cfg, lp[k].data_ptr(), ls[k].data_ptr(),
                        lt[k].data_ptr(), 1, P(st.cuda_stream)), lib)

    rows = torch.empty((nseg, 32), dtype=torch.float64, device=dev)

    def demod(k):
        lib = libs[k]
        chk(lib.dfmi_demod_rows(x.data_ptr(), nseg, R, R, nd, w0, 0, rows.data_ptr(), 1, P(st.cuda_stream)), lib)

    def seq(k):
        lib = libs[k]
        chk(lib.dfmi_nls_record(x.data_ptr(), 1, 500 * R, 500, R, nd, w0, 0, g.ctypes.data, 0, 1, cfg,
                                s1[k].data_ptr(), k1[k].data_ptr(), 1, P(st.cuda_stream)), lib)

    def seqa(k):
        lib = libs[k]
        chk(lib.dfmi_nls_record(x.data_ptr(), 1, nseg * R, nseg, R, nd, w0, 0, g.ctypes.data, 0, 1, cfg,
                                sa[k].data_ptr(), ka[k].data_ptr(), 1, P(st.cuda_stream)), lib)

    for kv in filter(None, os.environ.get("TUNE", "").split(",")):  # e.g. TUNE=lm_general=1 on every library
        k, v = kv.split("=")
        for lib in libs.values():
            lib.dfmi_set_tuning.argtypes = [ctypes.c_char_p, ctypes.c_int64]
            chk(lib.dfmi_set_tuning(k.encode(), int(v)), lib)
    first = next(iter(libs.values()))
    chk(first.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dc.data_ptr(), 1, P(st.cuda_stream)),
        first)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, reps):
        fn()
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    for k in libs:  # clock ramp + warm caches of both libraries
        for _ in range(20):
            step(k)
    res = {k: {"step": [], "demod": [], "lm": [], "seq500": []} for k in libs}
    if seqall:
        for k in libs:
            res[k]["seqall"] = []
    for _ in range(rounds):
        for k in libs:
            res[k]["step"].append(timed(lambda: step(k), 20))
            res[k]["demod"].append(timed(lambda: demod(k), 20))
            res[k]["lm"].append(timed(lambda: lm(k), 20))
            res[k]["seq500"].append(timed(lambda: seq(k), 3))
            if seqall:
                res[k]["seqall"].append(timed(lambda: seqa(k), 1))
    torch.cuda.synchronize()
    names = list(libs)
    summary = {k: {w: round(float(np.median(v)), 5) for w, v in r.items()} for k, r in res.items()}
    a = names[0]
    eq = {}
    for b in names[1:]:
        eq[f"{a}_vs_{b}"] = {
            "step": bool(torch.equal(out[a], out[b]) and torch.equal(ok[a], ok[b])),
            "lm": bool(torch.equal(lp[a], lp[b]) and torch.equal(ls[a], ls[b]) and torch.equal(lt[a], lt[b])),
            "seq500": bool(torch.equal(s1[a], s1[b]) and torch.equal(k1[a], k1[b])),
            "step_max_abs_dm": float((out[a][1] - out[b][1]).abs().max()),
            "step_max_abs_dphi": float((out[a][2] - out[b][2]).abs().max()),
            "seq_max_abs_dm": float((s1[a][1] - s1[b][1]).abs().max())}
        if seqall:
            eq[f"{a}_vs_{b}"]["seqall"] = bool(torch.equal(sa[a], sa[b]) and torch.equal(ka[a], ka[b]))
    print(json.dumps({"ms": summary, "bit_identical": eq, "libs": spec, "rounds": rounds, "tune": os.environ.get("TUNE", ""),
                      "phi": PHI, "psi": PSI}), flush=True)


if __name__ == "__main__":
    main()
