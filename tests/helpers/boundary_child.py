"""Child process of tests/test_gpu_binding_no_torch.py: the boundary used as the reference
would use it, in a FRESH interpreter started by subprocess.run([sys.executable, ...]) (never a
re-exec of the test process). Prints one JSON line; exits non-zero on any failure.

  binding  INTEGRATION.md §B (numpy + ctypes, no torch) on every golden record in seq / c1 /
           par4 modes against the reference's own outputs (tests/golden/records.npz), with
           'torch' never imported and libdfmi.so bound to the system HIP runtime
           /opt/rocm/lib/libamdhip64.so.7 (the runtime it links; /proc/self/maps is checked).
  fork     libdfmi.so loaded with NO GPU call, then multiprocessing's 'fork' Pool(2) whose
           workers each run dff.fit(label, n=20, parallel=False) on a golden record, as the
           reference's Experiment does (experiments.py:381-384) and its _fit_parallel does
           with fit.fit (fitters.py:421-423); the parent makes no GPU call before the fork.
  torch_after
           the library loaded by deepfmkit_amd._lib and initialised by a host-memory EKF call
           BEFORE torch is imported; then torch must still see the GPU and compute, and only
           one HIP runtime is mapped (the round-4 probe scripts/probe_init_order.py had torch
           report no GPU in that order).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def _maps(pattern):
    with open("/proc/self/maps") as f:
        return sorted({ln.split()[-1] for ln in f if pattern in ln and "/" in ln})


def _golden():
    import numpy as np
    with open(os.path.join(ROOT, "tests", "golden", "manifest.json")) as f:
        manifest = json.load(f)
    return manifest, np.load(os.path.join(ROOT, "tests", "golden", "records.npz"))


def _ref(records_npz, name, mode):
    return {k: records_npz[f"{name}_{mode}_{k}"] for k in ("amp", "m", "phi", "psi", "dc", "ssq", "fitok")}


def binding():
    from conftest import compare_fit, make_record, record_tol, sha
    from test_integration_binding import _binding_module
    m = _binding_module()  # INTEGRATION.md §B executed as written (library path substituted)
    manifest, rec = _golden()
    done = []
    for e in manifest["records"]:
        if e["name"] == "ragged_tail":
            continue
        raw = make_record(e).raws[e["name"]]
        assert sha(raw.samples()) == e["sha256"], e["name"]
        for mode in ("seq", "c1", "par4"):
            if f"{e['name']}_{mode}_amp" not in rec.files:
                continue
            kw = dict(ndata=e["ndata"], init_m=e["init_m"])
            f = m.HipNLSFitter({"n": e["n"]})
            if mode == "seq":
                df = f.fit(raw, parallel=False, **kw)
            elif mode == "c1":
                df = f.fit(raw, parallel=True, **kw)
            else:
                df = f.fit(raw, parallel=True, n_cores=4, **kw)
            ref = _ref(rec, e["name"], mode)
            compare_fit({k: df[k].to_numpy() for k in ref}, ref, tol=record_tol(e["ndata"], rec[f"{e['name']}_qi"], ref))
            done.append(f"{e['name']}:{mode}")
    hip = _maps("libamdhip64")
    out = {"fits": len(done), "torch_imported": "torch" in sys.modules, "hip_runtimes": hip,
           "hsa_runtimes": _maps("libhsa-runtime64")}
    assert not out["torch_imported"], out
    assert len(hip) == 1 and hip[0].startswith("/opt/rocm") and ".so.7" in hip[0], out
    assert len(done) >= 15, done
    return out


def _fork_worker(name):
    """One Pool worker: the reference's per-trial call shape (experiments.py:66-77 / 381-384:
    a framework per trial, fit with parallel=False) on a golden record."""
    import numpy as np
    from conftest import compare_fit, make_record, record_tol
    manifest, rec = _golden()
    e = next(x for x in manifest["records"] if x["name"] == name)
    dff = make_record(e)
    fobj = dff.fit(name, n=e["n"], parallel=False, ndata=e["ndata"], init_m=e["init_m"])
    df = dff.fits_df[f"{name}_nls"]
    ours = {k: df[k].to_numpy() for k in ("amp", "m", "phi", "psi", "dc", "ssq", "fitok")}
    assert np.array_equal(ours["m"], fobj.m)
    ref = _ref(rec, name, "seq")
    compare_fit(ours, ref, tol=record_tol(e["ndata"], rec[f"{name}_qi"], ref))
    return {"pid": os.getpid(), "name": name, "rows": int(np.asarray(fobj.m).size), "torch": "torch" in sys.modules}


def fork():
    import multiprocessing as mp
    from deepfmkit_amd import _lib
    lib = _lib.load()  # loaded, no GPU call: HIP is initialised lazily, in each worker
    before = {"hip_runtimes": _maps("libamdhip64"), "kfd_open": _kfd_open()}
    names = ["phi1_psi05", "m20_init6", "legacy30k", "snr0"]
    with mp.get_context("fork").Pool(2) as pool:
        res = pool.map(_fork_worker, names)
    assert sorted(r["name"] for r in res) == sorted(names), res
    assert len({r["pid"] for r in res}) >= 1
    # the parent still has not touched the GPU, and can now (after its children)
    after_fork_kfd = _kfd_open()
    assert lib.dfmi_device_count() >= 1, _lib.load().dfmi_last_error()
    return {"workers": res, "parent_before_fork": before, "parent_kfd_open_after_pool": after_fork_kfd,
            "runtime": _lib.RUNTIME, "torch_imported": "torch" in sys.modules}


def _kfd_open():
    """Whether this process holds /dev/kfd open (HIP initialised)."""
    try:
        return any(os.path.realpath(os.path.join("/proc/self/fd", fd)) == "/dev/kfd"
                   for fd in os.listdir("/proc/self/fd"))
    except OSError:
        return None


def torch_after():
    import numpy as np
    from deepfmkit_amd import _lib
    lib = _lib.load()
    x = np.cos(np.arange(8192) * 0.03)
    st = np.zeros((2, 5))
    _lib.check(lib.dfmi_ekf_fit(_lib.ptr(x), 1, x.size, x.size, _lib.ptr(np.array([1.0, 6.0, 0.0, 0.0])),
                                _lib.ptr(np.ones(5)), _lib.ptr(np.full(5, 1e-8)), None, 2 * np.pi * 1000.0,
                                200000.0, 4000, 2, _lib.ptr(st), _lib.DFMI_MEM_HOST, None), "dfmi_ekf_fit")
    assert np.isfinite(st).all()
    import torch
    ok = torch.cuda.is_available()
    s = float(torch.arange(10, dtype=torch.float64, device="cuda").sum().item()) if ok else None
    out = {"torch_cuda_available": ok, "torch_sum": s, "hip_runtimes": _maps("libamdhip64"),
           "hsa_runtimes": _maps("libhsa-runtime64"), "runtime": _lib.RUNTIME}
    assert ok and s == 45.0, out
    assert len(out["hip_runtimes"]) == 1 and len(out["hsa_runtimes"]) == 1, out
    return out


if __name__ == "__main__":
    what = sys.argv[1]
    res = {"binding": binding, "fork": fork, "torch_after": torch_after}[what]()
    print(json.dumps({what: res}))
